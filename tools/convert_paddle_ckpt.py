"""Convert a reference (PaddleFleetX) GPT ``model.pdparams`` into this
framework's checkpoint payload (SURVEY §5.4 importer).

    python tools/convert_paddle_ckpt.py --src ckpt/GPT_345M/mp_00_sharding_00_pp_00/model.pdparams \
        --dst ckpt/converted [--num_heads 16]

``--dst`` then works as ``Engine.save_load.ckpt_dir`` for eval / generation /
export (model weights only: the reference optimizer state is not imported).
The source is read with a restricted unpickler (numpy arrays only).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", required=True)
    ap.add_argument("--dst", required=True)
    ap.add_argument("--num_heads", type=int, default=None,
                    help="only for checkpoints with split q/k/v projections")
    ap.add_argument("--dtype", default="float32", choices=["float32", "bfloat16", "float16"])
    a = ap.parse_args()
    import torch
    from fleetx_amd.utils import paddle_import as PI
    from fleetx_amd.utils import checkpoint as ckpt
    sd = PI.convert_gpt_state(PI.load_paddle_state(a.src), num_heads=a.num_heads)
    dt = getattr(torch, a.dtype)
    sd = {k: v.to(dt) for k, v in sd.items()}
    ckpt.save_payloads(a.dst, {"model.pdparams": sd})
    n = sum(v.numel() for v in sd.values())
    print("wrote {} tensors ({:.1f}M params) to {}".format(len(sd), n / 1e6, a.dst))


if __name__ == "__main__":
    main()

"""Column-sum kernels in isolation (csrc/kernels/norm_eltwise.hip: the bias /
LayerNorm-weight gradients of a [tokens, h] activation): fused last-arriver
reduction into an fp32 vector, against torch's ``sum(0)`` over the same
tensor.  One JSON line per shape; ``FLEETX_COLSUM_BLOCKS`` (read once per
process) sets the workgroups per reduction.

    python tools/bench_colsum.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    from fleetx_amd.ops.norm import col_sum_f32
    blocks = os.environ.get("FLEETX_COLSUM_BLOCKS", "1024")
    for M, h in ((8192, 4096), (8192, 2048), (8192, 1024), (16448, 1408)):
        x = torch.randn(M, h, device="cuda", dtype=torch.bfloat16)
        dst = torch.zeros(h, device="cuda", dtype=torch.float32)
        us = timeit(lambda: col_sum_f32(x, dst, False))
        ref = x.float().sum(0)
        err = float((dst - ref).abs().max() / ref.abs().max())
        ut = timeit(lambda: x.sum(0))
        print(json.dumps({"M": M, "h": h, "blocks": int(blocks), "colsum_us": round(us, 2),
                          "colsum_TB_s": round(M * h * 2 / us / 1e6, 2),
                          "torch_sum_us": round(ut, 2), "max_rel_err": err}), flush=True)


if __name__ == "__main__":
    main()

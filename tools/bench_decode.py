"""Decode-attention bandwidth microbenchmark (split-K kernel, csrc/kernels/quant_decode.hip).

Prints one JSON line per case: bytes of K+V cache read / kernel time.  The op
is HBM bound, so the figure of merit is TB/s against the ~8 TB/s peak.

    python tools/bench_decode.py [--dtype bf16|fp16]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    from fleetx_amd import ops
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float16
    for B, H, D, L in ((1, 32, 128, 32768), (8, 32, 128, 4096), (32, 32, 128, 2048),
                       (64, 16, 64, 1024), (4, 32, 128, 16384)):
        q = torch.randn(B, H, D, device="cuda", dtype=dt)
        kc = torch.randn(B, L, H, D, device="cuda", dtype=dt)
        vc = torch.randn(B, L, H, D, device="cuda", dtype=dt)
        lens = torch.full((B,), L, device="cuda", dtype=torch.int32)
        res = {}
        for ns in (1, None):
            for _ in range(3):
                ops.decode_attention(q, kc, vc, lens, nsplit=ns)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                ops.decode_attention(q, kc, vc, lens, nsplit=ns)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.iters
            nbytes = 2 * B * L * H * D * kc.element_size()
            res["split1" if ns == 1 else "auto"] = {"us": round(us, 1),
                                                    "TBps": round(nbytes / us / 1e6, 3)}
        print(json.dumps({"B": B, "H": H, "D": D, "L": L, "dtype": a.dtype,
                          "nsplit_auto": ops.attention.decode_splits(B, H, L), **res}), flush=True)
        del kc, vc


if __name__ == "__main__":
    main()

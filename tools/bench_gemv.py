"""Decode GEMV (csrc/kernels/decode_gemv.hip) micro-benchmark: us per call and
weight-stream TB/s for the decoder-layer shapes of GPT 1.3B / 6.7B, against
hipBLASLt (F.linear) on the same operands.  

    python tools/bench_gemv.py [--m 1 8 16]"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"1.3B_qkv": (6144, 2048), "1.3B_out": (2048, 2048), "1.3B_fc1": (8192, 2048),
          "1.3B_fc2": (2048, 8192), "6.7B_qkv": (12288, 4096), "6.7B_out": (4096, 4096),
          "6.7B_fc1": (16384, 4096), "6.7B_fc2": (4096, 16384), "lm_head_1.3B": (50304, 2048)}


def timeit(fn, iters=200):
    for _ in range(10):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000.0 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[1, 16])
    ap.add_argument("--warm", action="store_true",
                    help="also time a weight resident in the Infinity Cache")
    args = ap.parse_args()
    from fleetx_amd.ops import gemm as G
    for name, (N, K) in SHAPES.items():
        # enough weight copies (>= 1 GiB) that successive calls stream from HBM,
        # as in a decode step over all layers, not from the 256 MB Infinity Cache
        ncopy = max(1, -(-(1 << 30) // (N * K * 2)))
        ws = [(torch.randn(N, K, device="cuda") * K ** -0.5).bfloat16() for _ in range(ncopy)]
        b = torch.randn(N, device="cuda").bfloat16()
        for M in args.m:
            x = torch.randn(M, K, device="cuda").bfloat16()
            it = [0]

            def nxt():
                it[0] = (it[0] + 1) % ncopy
                return ws[it[0]]
            us = timeit(lambda: G.decode_linear(x, nxt(), b))
            ub = timeit(lambda: F.linear(x, nxt(), b))
            rec = {"shape": name, "M": M, "N": N, "K": K,
                   "gemv_us": round(us, 2), "gemv_TB_s": round(N * K * 2 / us / 1e6, 2),
                   "hipblaslt_us": round(ub, 2),
                   "hipblaslt_TB_s": round(N * K * 2 / ub / 1e6, 2)}
            if args.warm:
                # the same weight every call: it stays in the 256 MB Infinity
                # Cache (MALL) -- what a prefetch of the next GEMV's weights
                # under the current phase would buy
                w0 = ws[0]
                uw = timeit(lambda: G.decode_linear(x, w0, b))
                rec.update(gemv_warm_us=round(uw, 2), gemv_warm_TB_s=round(N * K * 2 / uw / 1e6, 2))
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()

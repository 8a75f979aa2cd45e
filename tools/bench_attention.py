"""Fused attention micro-benchmark on MI355X (forward and backward, causal /
non-causal, attention dropout on / off) at the GPT-3 6.7B training shape.
Forward and backward are each timed over ``--iters`` back-to-back launches
(no host gaps; matches rocprofv3 kernel time within a few percent).

Prints one JSON line per case with milliseconds and achieved TFLOP/s
(forward 4*B*H*S^2*D, backward 2.5x that, both halved when causal -- the
useful FLOPs, not what a kernel happens to execute).

    python tools/bench_attention.py [--b 8 --s 1024 --h 32 --d 128 --iters 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=8)
    ap.add_argument("--s", type=int, default=1024)
    ap.add_argument("--h", type=int, default=32)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"])
    args = ap.parse_args()
    from fleetx_amd import ops
    B, S, H, D = args.b, args.s, args.h, args.d
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float16
    qkv = torch.randn(B, S, H, 3, D, device="cuda", dtype=dt, requires_grad=True)
    g = torch.randn(B, S, H, D, device="cuda", dtype=dt)
    for causal in (True, False):
        for p in (0.0, 0.1):
            def fwd():
                return ops.flash_attention_qkvpacked(qkv, causal=causal, dropout_p=p, key=12345)
            for _ in range(3):
                torch.autograd.grad(fwd(), qkv, g)
            torch.cuda.synchronize()
            # back-to-back launches between two events: the host enqueues
            # ahead of the GPU, so the time is the kernels' (no launch gaps)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                fwd()
            e1.record()
            torch.cuda.synchronize()
            tf = e0.elapsed_time(e1) / args.iters
            outs = [fwd() for _ in range(args.iters)]
            torch.cuda.synchronize()
            e0.record()
            for o in outs:
                torch.autograd.grad(o, qkv, g)
            e1.record()
            torch.cuda.synchronize()
            tb = e0.elapsed_time(e1) / args.iters
            del outs
            flops = 4.0 * B * H * S * S * D * (0.5 if causal else 1.0)
            print(json.dumps({"B": B, "S": S, "H": H, "D": D, "dtype": args.dtype,
                              "causal": causal, "dropout": p,
                              "fwd_ms": round(tf, 4), "bwd_ms": round(tb, 4),
                              "fwd_tflops": round(flops / tf / 1e9, 1),
                              "bwd_tflops": round(2.5 * flops / tb / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()

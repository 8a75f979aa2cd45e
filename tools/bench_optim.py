"""Bandwidth of the fused AdamW kernel (csrc/kernels/loss_optim_embed.hip) in
isolation: 30 B per parameter (fp32 p/g/m/v in, p/m/v + bf16 copy out).

    python tools/bench_optim.py [--n 1e9 --iters 10]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=float, default=1e9)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--sweep", action="store_true", help="grid / non-temporal variants")
    ap.add_argument("--capped", action="store_true",
                    help="capped grids (32-128 workgroups) in both block shapes")
    a = ap.parse_args()
    from fleetx_amd.ops import _lib
    k = _lib.kernels()
    n = int(a.n)
    dev = "cuda"
    p = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev) * 1e-3
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    p16 = torch.empty(n, device=dev, dtype=torch.bfloat16)
    gs = torch.ones(1, device=dev)
    skip = torch.zeros(1, device=dev, dtype=torch.int32)
    step = torch.ones(1, device=dev, dtype=torch.int32)

    def run():
        k.adamw_flat(0, p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p16.data_ptr(), n,
                     1e-4, 0.9, 0.95, 1e-8, 0.01, 0.0, gs.data_ptr(), skip.data_ptr(),
                     step.data_ptr(), _lib.stream())
    def timeit(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters

    # streaming references: copy (1 read + 1 write) and a*b -> c (2 reads + 1 write)
    ms = timeit(lambda: m.copy_(p))
    print(json.dumps({"kernel": "torch_copy_f32", "n": n, "ms": round(ms, 3),
                      "TB_s": round(8.0 * n / ms / 1e9, 3)}))
    ms = timeit(lambda: torch.mul(p, g, out=v))
    print(json.dumps({"kernel": "torch_mul_f32", "n": n, "ms": round(ms, 3),
                      "TB_s": round(12.0 * n / ms / 1e9, 3)}))
    m.zero_()
    v.zero_()
    cases = [(0, 1, 0)]
    if a.sweep:
        cases += [(0, 0, 0), (1024, 1, 0), (2048, 1, 0), (4096, 1, 0)]
    if a.capped:
        # the forward-overlapped update: few workgroups (CUs), deep per-CU
        # memory-level parallelism -- bandwidth per CU decides how much of the
        # chip the update takes from the GEMMs beside it
        cases += [(g, 1, w) for w in (0, 1) for g in (32, 48, 64, 96, 128)]
    for grid, nt, wide in cases:
        k.adamw_tune(grid, nt, wide)
        ms = timeit(run)
        tb = 30.0 * n / ms / 1e9
        print(json.dumps({"kernel": "adamw_flat", "grid": grid or "auto", "nontemporal": nt,
                          "block": 1024 if wide else 256, "float4_per_thread": 4 if wide else 2,
                          "n": n, "ms": round(ms, 3), "TB_s": round(tb, 3),
                          "GB_s_per_workgroup": round(1000 * tb / grid, 1) if grid else None,
                          "ms_per_6.65B_params": round(ms * 6.65e9 / n, 2)}))
    k.adamw_tune(0, 1, 0)


if __name__ == "__main__":
    main()

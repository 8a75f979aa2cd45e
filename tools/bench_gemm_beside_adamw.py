"""Forward-GEMM throughput BESIDE the forward-overlapped AdamW.

In the training step each layer's forward GEMMs share the chip with the
previous step's AdamW, which streams ~30 B per parameter on a side stream
(128-workgroup cap, ``optims/optimizer.py _update_overlapped``).  An isolated
GEMM benchmark misses that interaction (a forward GEMM 10 % faster alone made
the 6.7B step 22 ms slower, ``profiles/r4_route/``).  This tool runs a GEMM
back to back on the main stream while the side stream runs AdamW over a
flat buffer of ``--params`` elements, and reports each GEMM path's time
alone and beside the update, plus the update's own streaming rate.

    python tools/bench_gemm_beside_adamw.py [--tokens 8192 --hidden 4096]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--params", type=int, default=1_000_000_000)
    ap.add_argument("--grid", type=int, default=128, help="AdamW workgroup cap (0 = uncapped)")
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--only", default="", help="comma list of shape names (qkv,out,fc1,fc2)")
    ap.add_argument("--paths", default="blas,hip", help="comma list of GEMM paths")
    ap.add_argument("--wide", type=int, default=0,
                    help="1024-thread AdamW workgroups (16 waves: one workgroup per CU)")
    ap.add_argument("--grid-sweep", default="",
                    help="comma list of AdamW grids to time alone (e.g. 32,64,96,128) and exit")
    ap.add_argument("--chunks", type=int, default=1,
                    help="split the update into this many launches (the step launches one "
                         "per layer unit: ~66 at 6.7B)")
    a = ap.parse_args()
    from fleetx_amd.ops import _lib
    from fleetx_amd.ops import gemm as G
    k = _lib.kernels()
    dev, bf = "cuda", torch.bfloat16
    M, h = a.tokens, a.hidden
    n = a.params
    master = torch.randn(n, device=dev) * 0.02
    grad = torch.randn(n, device=dev) * 1e-3
    m1 = torch.zeros(n, device=dev)
    v1 = torch.zeros(n, device=dev)
    p16 = master.to(bf)
    gs = torch.ones(1, device=dev)
    fi = torch.zeros(1, dtype=torch.int32, device=dev)
    ds = torch.ones(1, dtype=torch.int32, device=dev)
    side = torch.cuda.Stream()

    def adamw_once():
        c = n // a.chunks
        for i in range(a.chunks):
            o = i * c
            ln = n - o if i == a.chunks - 1 else c
            k.adamw_flat(0, master[o:].data_ptr(), grad[o:].data_ptr(), m1[o:].data_ptr(),
                         v1[o:].data_ptr(), p16[o:].data_ptr(), ln, 1e-4, 0.9, 0.95, 1e-8, 0.01,
                         0.0, gs.data_ptr(), fi.data_ptr(), ds.data_ptr(), _lib.stream())

    shapes = {"qkv": (h, 3 * h), "out": (h, h), "fc1": (h, 4 * h), "fc2": (4 * h, h)}
    only = [s for s in a.only.split(",") if s]
    rows = []
    if a.grid_sweep:
        # AdamW alone on a limited number of workgroups: how many CUs the
        # update needs to stream at HBM rate
        for g in [int(x) for x in a.grid_sweep.split(",")]:
            k.adamw_tune(g, 1, a.wide)
            adamw_once()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            adamw_once()
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1)
            print(json.dumps({"case": "adamw_grid", "grid": g, "wide": a.wide, "ms": round(t, 3),
                              "TB_s": round(30.0 * n / t / 1e9, 2)}), flush=True)
        return
    # AdamW alone (rate)
    with torch.cuda.stream(side):
        if a.grid:
            k.adamw_tune(a.grid, 1, a.wide)
        adamw_once()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(side)
        adamw_once()
        e1.record(side)
    torch.cuda.synchronize()
    t_adam = e0.elapsed_time(e1)
    rows.append({"case": "adamw_alone", "ms": round(t_adam, 3),
                 "TB_s": round(30.0 * n / t_adam / 1e9, 2), "grid": a.grid,
                 "chunks": a.chunks})
    print(json.dumps(rows[-1]), flush=True)
    for name, (K, N) in shapes.items():
        if only and name not in only:
            continue
        x = torch.randn(M, K, device=dev, dtype=bf)
        w = torch.randn(N, K, device=dev, dtype=bf) * 0.02
        flops = 2.0 * M * N * K
        paths = {}
        if "blas" in a.paths:
            paths["blas"] = lambda: F.linear(x, w)
        if "hip" in a.paths:
            paths["hip"] = lambda: G.linear_fwd(x, w)
        for pname, fn in paths.items():
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            alone = e0.elapsed_time(e1) / a.iters
            # beside: start the update on the side stream, then the GEMMs
            torch.cuda.synchronize()
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(side):
                s0.record(side)
                adamw_once()
                s1.record(side)
            g0.record()
            for _ in range(a.iters):
                fn()
            g1.record()
            torch.cuda.synchronize()
            beside = g0.elapsed_time(g1) / a.iters
            t_up = s0.elapsed_time(s1)
            rows.append({"case": "%s_%s" % (name, pname), "M": M, "N": N, "K": K,
                         "alone_ms": round(alone, 4), "alone_TF": round(flops / alone / 1e9, 1),
                         "beside_ms": round(beside, 4),
                         "beside_TF": round(flops / beside / 1e9, 1),
                         "adamw_ms_beside": round(t_up, 3),
                         "gemm_window_ms": round(a.iters * beside, 3)})
            print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()

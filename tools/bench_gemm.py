"""GEMM micro-benchmark for the transformer-layer shapes (fwd / dgrad / wgrad)
under the weight layouts the framework can use, sustained back-to-back like a
training step.

    python tools/bench_gemm.py [--tokens 8192 --hidden 4096 --iters 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--geom", default="", help="comma list of nf:split lab geometries for the "
                                               "hip_wgrad cases, e.g. 4:1,4:2,8:4 (0:0 = plan)")
    ap.add_argument("--ffn", type=int, default=0, help="MLP width (default 4 x hidden)")
    ap.add_argument("--vocab", type=int, default=0, help="also time the LM head (h -> vocab)")
    ap.add_argument("--only", default="", help="comma list of case names")
    ap.add_argument("--gm", default="", help="comma list of tile-order M-group heights to A/B "
                                             "on the hip_* cases (interleaved, one process)")
    a = ap.parse_args()
    from fleetx_amd.ops.elementwise import transpose2d
    from fleetx_amd.ops import gemm as G
    M, h = a.tokens, a.hidden
    dev, bf = "cuda", torch.bfloat16
    ffn = a.ffn or 4 * h
    shapes = {"qkv": (h, 3 * h), "out": (h, h), "fc1": (h, ffn), "fc2": (ffn, h)}
    if a.vocab:
        shapes["head"] = (h, a.vocab)
    for name, (K, N) in shapes.items():
        x = torch.randn(M, K, device=dev, dtype=bf)
        w = torch.randn(N, K, device=dev, dtype=bf) * 0.02       # [out, in]
        wt = w.t().contiguous()                                   # [in, out]
        dy = torch.randn(M, N, device=dev, dtype=bf)
        dw32 = torch.empty(N, K, device=dev, dtype=torch.float32)
        bias = torch.randn(N, device=dev, dtype=bf) * 0.1
        hpre = torch.randn(M, K, device=dev, dtype=bf)
        dyT = dy.t().contiguous()                                 # [N, M]
        xT = x.t().contiguous()                                   # [K, M]
        fl = 2.0 * M * N * K
        res = {"gemm": name, "M": M, "N": N, "K": K}
        cases = {
            "fwd_x_wT": lambda: torch.nn.functional.linear(x, w),
            "fwd_x_wT_bias": lambda: torch.nn.functional.linear(x, w, bias),
            "fwd_x_wt": lambda: torch.mm(x, wt),
            "dgrad_dy_w": lambda: torch.mm(dy, w),
            "dgrad_dy_wtT": lambda: torch.mm(dy, wt.t()),
            "wgrad_bf16": lambda: torch.mm(dy.t(), x),
            "wgrad_f32out": lambda: torch.ops.aten.mm.dtype_out(dy.t(), x, torch.float32, out=dw32),
            "wgrad_f32acc": lambda: torch.ops.aten.addmm.dtype_out(dw32, dy.t(), x, torch.float32,
                                                                   out=dw32),
            # wgrad as a "TN" GEMM on transposed (token-contiguous) operands
            "wgradTN_bf16": lambda: torch.nn.functional.linear(dyT, xT),
            "wgradTN_f32out": lambda: torch.ops.aten.mm.dtype_out(dyT, xT.t(), torch.float32,
                                                                  out=dw32),
            "wgradTN_f32acc": lambda: torch.ops.aten.addmm.dtype_out(dw32, dyT, xT.t(),
                                                                     torch.float32, out=dw32),
            "transpose_dy": lambda: dyT.copy_(dy.t()),
            "transpose_dy_hip": lambda: transpose2d(dy, out=dyT),
            "wgrad_tn_path": lambda: torch.ops.aten.addmm.dtype_out(
                dw32, transpose2d(dy), transpose2d(x).t(), torch.float32, out=dw32),
            "dgrad_tn_path": lambda: torch.nn.functional.linear(dy, transpose2d(w)),
            # hand-written MFMA GEMM (csrc/kernels/gemm.hip), native layouts
            "hip_fwd": lambda: G.linear_fwd(x, w),
            "hip_fwd_bias": lambda: G.linear_fwd(x, w, bias),
            "hip_fwd_gelu": lambda: G.linear_fwd(x, w, bias, act="gelu"),
            "hip_dgrad": lambda: G.linear_dgrad(dy, w),
            "hip_dgrad_dgelu": lambda: G.linear_dgrad(dy, w, act_input=hpre),
            "hip_wgrad_f32acc": lambda: G.linear_wgrad(dy, x, dw32, True),
        }
        gms = [int(g) for g in a.gm.split(",")] if a.gm else [None]
        geoms = [tuple(int(v) for v in g.split(":")) for g in a.geom.split(",")] if a.geom else [None]
        items = []
        for k, fn in cases.items():
            if a.only and k not in a.only.split(","):
                continue
            if k.startswith("hip_wgrad"):
                items += [(k + ("" if g is None else "_gm%d" % g) +
                           ("" if q is None else "_g%d:%d" % q), fn, g, q) for g in gms for q in geoms]
            elif k.startswith("hip_"):
                items += [(k if g is None else "%s_gm%d" % (k, g), fn, g, None) for g in gms]
            else:
                items.append((k, fn, None, None))
        from fleetx_amd.ops import _lib
        for k, fn, g, q in items:
            if g is not None:
                _lib.kernels().gemm_set_gm(g)
            _lib.kernels().gemm_set_geom(*(q or (0, 0)))
            ms = timeit(fn, a.iters)
            # TFLOP/s of the GEMM (for transposes: us per call)
            res[k] = round(ms * 1e3, 1) if k.startswith("transpose") else round(fl / ms / 1e9, 1)
        print(json.dumps(res), flush=True)
    if a.gm or a.geom:
        from fleetx_amd.ops import _lib
        _lib.kernels().gemm_set_gm(0)
        _lib.kernels().gemm_set_geom(0, 0)


if __name__ == "__main__":
    main()

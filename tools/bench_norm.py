"""Bandwidth of the row-wise LayerNorm / residual / GeLU kernels at the GPT-3
6.7B activation shape (8192 tokens x 4096; 16384 for the GeLU), in isolation.

    python tools/bench_norm.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402


def timeit(fn, iters=30):
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
    from fleetx_amd import ops
    from fleetx_amd.ops.elementwise import gelu_plain
    M, h = 8192, 4096
    bf = torch.bfloat16
    x = torch.randn(M, h, device="cuda", dtype=bf)
    r = torch.randn(M, h, device="cuda", dtype=bf)
    b = torch.randn(h, device="cuda", dtype=bf)
    g = torch.ones(h, device="cuda", dtype=bf)
    be = torch.zeros(h, device="cuda", dtype=bf)
    hh = torch.randn(M, 4 * h, device="cuda", dtype=bf)
    E = M * h * 2  # bytes of one activation
    cases = [
        ("layer_norm", lambda: ops.layer_norm(x, g, be), 2 * E),
        ("add_ln_bias_res_p0", lambda: ops.add_layer_norm(x, b, r, g, be, p=0.0, key=1), 4 * E),
        ("add_ln_bias_res_p0.1", lambda: ops.add_layer_norm(x, b, r, g, be, p=0.1, key=1), 4 * E),
        ("bias_dropout_add_p0.1", lambda: ops.bias_dropout_add(x, b, r, p=0.1, key=1), 3 * E),
        ("gelu_tanh_16k", lambda: gelu_plain(hh), 2 * 4 * E),
    ]
    from fleetx_amd.ops import _lib
    k = _lib.kernels()
    mean = torch.zeros(M, device="cuda")
    rstd = torch.ones(M, device="cuda")
    ds = torch.empty_like(x)
    dx = torch.empty_like(x)

    def ln_bwd(ds_in, p):
        k.ln_bwd_row(0, x.data_ptr(), r.data_ptr(), mean.data_ptr(), rstd.data_ptr(), g.data_ptr(),
                     _lib.ptr(ds_in), ds.data_ptr(), (dx if p > 0 else ds).data_ptr(), M, h,
                     float(p), 7, _lib.stream())
    # the row pass of the two-pass LayerNorm backward (h > 2048): dy, s (+ ds_in)
    # read, ds (+ dropout'd dx) written
    cases += [("ln_bwd_row_dsin_p0.1", lambda: ln_bwd(x, 0.1),
               5 * E),
              ("ln_bwd_row_p0", lambda: ln_bwd(None, 0.0), 3 * E)]
    for name, fn, nbytes in cases:
        ms = timeit(fn)
        print(json.dumps({"kernel": name, "us": round(ms * 1e3, 1),
                          "TB_s": round(nbytes / ms / 1e9, 3)}), flush=True)
    # LayerNorm backward through autograd (dy, s read; dx written; + column partials)
    xs = x.clone().requires_grad_(True)
    gg = g.clone().requires_grad_(True)
    bb = be.clone().requires_grad_(True)
    y = ops.layer_norm(xs, gg, bb)
    dy = torch.randn_like(y)
    ms = timeit(lambda: torch.autograd.grad(y, (xs, gg, bb), dy, retain_graph=True))
    print(json.dumps({"kernel": "layer_norm_bwd", "us": round(ms * 1e3, 1),
                      "TB_s": round(3 * E / ms / 1e9, 3)}), flush=True)


if __name__ == "__main__":
    main()

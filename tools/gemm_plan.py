"""Generate the shipped GEMM plan (``fleetx_amd/ops/gemm_plan_gfx950.json``).

For every transformer-layer shape of the model zoo (GPT 345M / 1.3B / 6.7B,
the 6.7B tensor-parallel shards of BASELINE config 3, ViT-g/14) and every GEMM
kind of a linear layer (forward, data gradient, fp32 weight gradient), this
times the MFMA kernel at each tile-order M-group height and the vendor path,
in interleaved rounds of back-to-back launches, and keeps the median of each
candidate.  The plan then fixes, per shape, the tile order and (for the data
gradient) the route, so a run never decides them from a first-call race on a
noisy box (``ops/gemm.py load_plan``).

Forward routes are not decided here: in the training step the forward GEMMs
share the chip with the forward-overlapped AdamW, which an isolated timing
cannot see (``tools/bench_gemm_beside_adamw.py``); ``--fwd-route kernel``
writes them explicitly after a step A/B.

    python tools/gemm_plan.py [--models 6.7B,1.3B,345M,vitg,6.7B-tp2] [--out plan.json]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402

# name: (tokens, [(layer, in, out), ...])
MODELS = {
    "345M": (8192, [("qkv", 1024, 3072), ("out", 1024, 1024), ("fc1", 1024, 4096),
                    ("fc2", 4096, 1024)]),
    "1.3B": (8192, [("qkv", 2048, 6144), ("out", 2048, 2048), ("fc1", 2048, 8192),
                    ("fc2", 8192, 2048)]),
    "6.7B": (8192, [("qkv", 4096, 12288), ("out", 4096, 4096), ("fc1", 4096, 16384),
                    ("fc2", 16384, 4096)]),
    # BASELINE config 3 family: TP2 shards, micro-batch 4 (N=4/8) and 8 (N=2)
    "6.7B-tp2": (4096, [("qkv", 4096, 6144), ("out", 2048, 4096), ("fc1", 4096, 8192),
                        ("fc2", 8192, 4096)]),
    "6.7B-tp2-m8": (8192, [("qkv", 4096, 6144), ("out", 2048, 4096), ("fc1", 4096, 8192),
                           ("fc2", 8192, 4096)]),
    "vitg": (16448, [("qkv", 1408, 4224), ("out", 1408, 1408), ("fc1", 1408, 6144),
                     ("fc2", 6144, 1408)]),
}
# tile-order codes: M-group height, + 32 = inside XCD rectangles, + 64 = the runner-up
# rectangle cut (csrc/kernels/gemm5.hip g5_tile_mn / g5_xrect_rows)
GMS = (1, 2, 4, 8, 16, 33, 34, 36, 40, 48, 97, 98, 100, 104)


def med_time(fns, rounds, iters):
    """{name: median ms per launch} over interleaved rounds."""
    t = {k: [] for k in fns}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for k, fn in fns.items():  # warm every candidate (first-call work, caches)
        fn()
    torch.cuda.synchronize()
    for _ in range(rounds):
        for k, fn in fns.items():
            ev[0].record()
            for _ in range(iters):
                fn()
            ev[1].record()
            ev[1].synchronize()
            t[k].append(ev[0].elapsed_time(ev[1]) / iters)
    return {k: statistics.median(v) for k, v in t.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default=",".join(MODELS))
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "fleetx_amd",
                                                   "ops", "gemm_plan_gfx950.json"))
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--margin", type=float, default=0.03)
    ap.add_argument("--fwd-route", default="", choices=["", "kernel", "vendor"])
    ap.add_argument("--dtypes", default="bf16")
    a = ap.parse_args()
    from fleetx_amd.ops import _lib
    from fleetx_amd.ops import gemm as G
    from fleetx_amd.parallel import linear as L  # registers the vendor paths  # noqa: F401
    k = _lib.kernels()
    k.gemm_set_tune(0)
    G.set_mode("hip")
    dev = "cuda"
    entries, seen = [], set()
    t0 = time.time()
    for dtn in a.dtypes.split(","):
        dt = torch.bfloat16 if dtn == "bf16" else torch.float16
        for model in a.models.split(","):
            M, layers = MODELS[model]
            for lname, kin, kout in layers:
                x = torch.randn(M, kin, device=dev, dtype=dt)
                w = torch.randn(kout, kin, device=dev, dtype=dt) * 0.02
                dy = torch.randn(M, kout, device=dev, dtype=dt)
                dw = torch.empty(kout, kin, device=dev, dtype=torch.float32)
                kinds = {
                    # kind: (plan key (M, N, K), kernel fn, vendor fn)
                    "fwd": ((M, kout, kin), lambda: G.linear_fwd(x, w), lambda: G.VENDOR["fwd"](x, w)),
                    "dgrad": ((M, kin, kout), lambda: G.linear_dgrad(dy, w),
                              lambda: G.VENDOR["dgrad"](dy, w)),
                    "wgrad": ((M, kout, kin), lambda: G.linear_wgrad(dy, x, dw, False), None),
                }
                for kind, (key, fk, fv) in kinds.items():
                    if (kind, dtn) + key in seen:
                        continue
                    seen.add((kind, dtn) + key)
                    fns = {}
                    for g in GMS:
                        fns["gm%d" % g] = (lambda g=g, fk=fk: (k.gemm_set_gm(g), fk()))
                    if fv is not None:
                        fns["vendor"] = (lambda fv=fv: (k.gemm_set_gm(0), fv()))
                    t = med_time(fns, a.rounds, a.iters)
                    k.gemm_set_gm(0)
                    best = min(GMS, key=lambda g: t["gm%d" % g])
                    kms = t["gm%d" % best]
                    flops = 2.0 * key[0] * key[1] * key[2]
                    e = {"kind": kind, "dtype": dtn, "M": key[0], "N": key[1], "K": key[2],
                         "gm": best, "kernel_ms": round(kms, 4),
                         "kernel_TF": round(flops / kms / 1e9, 1), "model": model, "layer": lname,
                         "gm_ms": {g: round(t["gm%d" % g], 4) for g in GMS}}
                    if fv is not None:
                        e["vendor_ms"] = round(t["vendor"], 4)
                        e["vendor_TF"] = round(flops / t["vendor"] / 1e9, 1)
                    if kind == "dgrad":
                        e["route"] = "kernel" if kms < (1 - a.margin) * t["vendor"] else "vendor"
                    elif kind == "fwd" and a.fwd_route:
                        e["route"] = a.fwd_route
                    elif kind == "wgrad":
                        e["route"] = "kernel"
                    entries.append(e)
                    print(json.dumps(e), flush=True)
    doc = {"arch": "gfx950", "generated_by": "tools/gemm_plan.py",
           "method": "median of %d interleaved rounds x %d launches per candidate; dgrad route = "
                     "kernel when %.0f%% faster than the vendor path" % (a.rounds, a.iters,
                                                                          100 * a.margin),
           "seconds": round(time.time() - t0, 1), "entries": entries}
    with open(a.out, "w") as f:
        json.dump(doc, f, indent=1)
    print("wrote", a.out, len(entries), "entries", file=sys.stderr)


if __name__ == "__main__":
    main()

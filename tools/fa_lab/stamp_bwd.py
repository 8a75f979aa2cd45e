"""Per-wave timeline of the flash-attention dK/dV pass from in-kernel
s_memrealtime stamps (100 MHz; lab build only, as ``stamp_fwd.py``).

Per workgroup (128 keys, one key block ``kblock`` of one head): prologue
(entry -> K/V fragments and the first Q / dO tile in), per query tile the
slowest / fastest wave's compute and the barrier wait, the dK / dV store
tail.  Printed per key block (causal: block k runs (S - 128 k) / QT tiles)
and overall, for causal and full attention.  Slots: 0 kblock, 1 entry, 2
prologue done, 3 + 2 t after tile t's compute, 4 + 2 t after its barrier,
126 before the stores, 127 end.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

import numpy as np  # noqa: E402
import torch  # noqa: E402

TICKS_PER_US = 100.0


def run(args, causal, p):
    from fleetx_amd import ops
    from fleetx_amd.ops import _lib
    k = _lib.kernels()
    B, S, H, D = args.b, args.s, args.h, args.d
    qkv = torch.randn(B, S, H, 3, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    nw = 4
    nk = (S + 127) // 128
    nblk = nk * B * H
    buf = torch.zeros(nblk * nw * 128, dtype=torch.int64, device="cuda")
    for _ in range(3):
        o = ops.flash_attention_qkvpacked(qkv, causal=causal, dropout_p=p, key=1)
        torch.autograd.grad(o, qkv, g)
    o = ops.flash_attention_qkvpacked(qkv, causal=causal, dropout_p=p, key=1)
    torch.cuda.synchronize()
    if not k.fa_set_stamps(buf.data_ptr()):
        raise SystemExit("not a lab build (fa_set_stamps returned 0)")
    torch.autograd.grad(o, qkv, g)
    torch.cuda.synchronize()
    k.fa_set_stamps(0)
    st = buf.view(nblk, nw, 128).cpu().numpy().astype(np.int64)
    kb = st[:, 0, 0]
    ent = st[:, :, 1].min(axis=1)
    pro = st[:, :, 2].max(axis=1)
    s0 = st[:, :, 126].min(axis=1)
    end = st[:, :, 127].max(axis=1)
    t0 = ent.min()
    out = {"causal": causal, "dropout": p, "span_us": round((end.max() - t0) / TICKS_PER_US, 2),
           "workgroups": int(nblk), "by_kblock": []}
    allt, alls, allw = [], [], []
    for kbv in sorted(set(kb.tolist())):
        sel = kb == kbv
        n = int((st[sel][0, 0, 4:126:2] > 0).sum())  # tiles run by this key block
        comp = st[sel][:, :, 3:3 + 2 * n:2]
        bar = st[sel][:, :, 4:4 + 2 * n:2]
        prev = np.concatenate([st[sel][:, :, 2:3], bar[:, :, :-1]], axis=2)
        cd = comp - prev
        slow, fast = cd.max(axis=1), cd.min(axis=1)
        tile = bar[:, 0, :] - prev[:, 0, :]
        allt.append(tile.ravel())
        alls.append(slow.ravel())
        allw.append((tile - slow).ravel())
        out["by_kblock"].append({
            "kblock": kbv, "wgs": int(sel.sum()), "tiles": n,
            "wg_us": round(float(np.mean(end[sel] - ent[sel])) / TICKS_PER_US, 2),
            "prologue_us": round(float(np.mean(pro[sel] - ent[sel])) / TICKS_PER_US, 2),
            "tile_us": round(float(np.mean(tile)) / TICKS_PER_US, 3),
            "first4_tile_us": [round(float(np.mean(tile[:, i])) / TICKS_PER_US, 3)
                               for i in range(min(4, n))],
            "tile_slowest_us": round(float(np.mean(slow)) / TICKS_PER_US, 3),
            "tile_fastest_us": round(float(np.mean(fast)) / TICKS_PER_US, 3),
            "store_us": round(float(np.mean(end[sel] - s0[sel])) / TICKS_PER_US, 2),
        })
    out["tile_us_mean"] = round(float(np.mean(np.concatenate(allt))) / TICKS_PER_US, 3)
    out["tile_slowest_us_mean"] = round(float(np.mean(np.concatenate(alls))) / TICKS_PER_US, 3)
    out["tile_barrier_wait_us_mean"] = round(float(np.mean(np.concatenate(allw))) / TICKS_PER_US,
                                             3)
    # slot fill: sum of workgroup durations over (span x resident slots)
    slots = 2 * 256
    out["slot_fill"] = round(float(np.sum(end - ent)) / (float(end.max() - t0) * slots), 3)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=8)
    ap.add_argument("--s", type=int, default=1024)
    ap.add_argument("--h", type=int, default=32)
    ap.add_argument("--d", type=int, default=128)
    args = ap.parse_args()
    for causal in (True, False):
        for p in (0.1,):
            print(json.dumps(run(args, causal, p)), flush=True)


if __name__ == "__main__":
    main()

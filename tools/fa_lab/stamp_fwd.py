"""Per-wave timeline of the flash-attention forward from in-kernel
s_memrealtime stamps (100 MHz) (lab build only: ``python tools/fa_lab/build.py``, then
``FLEETX_KERNELS_LIB=tools/fa_lab/_kernels<EXT> python tools/fa_lab/stamp_fwd.py``).

For causal and full attention at one shape it prints, per workgroup on
average: prologue (entry -> first tiles landed), the tiles' compute (slowest
wave) and barrier waits, the paired-item switch, the final O / lse store; and
the workgroup-duration spread and the CU slot occupancy over the launch.
Slots: 0 XCC / HW id, 1 entry, 2 prologue done, 3 + 2 t after tile t's
compute, 4 + 2 t after its barrier, 62 before the last finish, 63 end.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def run(args, causal, p):
    from fleetx_amd import ops
    from fleetx_amd.ops import _lib
    k = _lib.kernels()
    B, S, H, D = args.b, args.s, args.h, args.d
    qkv = torch.randn(B, S, H, 3, D, device="cuda", dtype=torch.bfloat16)
    nw = 4
    nq = (S + 32 * nw - 1) // (32 * nw)
    nblk = ((nq + 1) // 2 if causal else nq) * B * H
    buf = torch.zeros(nblk * nw * 64, dtype=torch.int64, device="cuda")
    for _ in range(3):
        ops.flash_attention_qkvpacked(qkv, causal=causal, dropout_p=p, key=1)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if not k.fa_set_stamps(buf.data_ptr()):
        raise SystemExit("not a lab build (fa_set_stamps returned 0)")
    e0.record()
    ops.flash_attention_qkvpacked(qkv, causal=causal, dropout_p=p, key=1)
    e1.record()
    torch.cuda.synchronize()
    k.fa_set_stamps(0)
    ms = e0.elapsed_time(e1)
    st = buf.view(nblk, nw, 64).cpu().numpy().astype(np.int64)
    # 64-key tiles per workgroup (S a multiple of 256: every causal pair full)
    ntile = (nq + 1) * (32 * nw // 64) if causal else S // 64
    assert S % 256 == 0 and ntile <= 29
    ent, pro = st[:, :, 1], st[:, :, 2]
    comp = st[:, :, 3:3 + 2 * ntile:2]
    bar = st[:, :, 4:4 + 2 * ntile:2]
    fin0, end = st[:, :, 62], st[:, :, 63]
    t0 = ent.min()
    span = end.max() - t0
    cyc_per_us = 100.0  # s_memrealtime ticks
    prev = np.concatenate([pro[:, :, None], bar[:, :, :-1]], axis=2)
    cdur = comp - prev                      # per wave, per tile
    wg_tile = bar - prev                    # per wave (same for all waves after the barrier)
    slow = cdur.max(axis=1)                 # slowest wave's compute per tile
    fast = cdur.min(axis=1)
    wait = wg_tile[:, 0, :] - slow          # barrier wait of the slowest wave
    wg_dur = end.max(axis=1) - ent.min(axis=1)
    us = lambda c: float(np.mean(c)) / cyc_per_us  # noqa: E731
    # slot occupancy: workgroups resident over time per (xcc, cu)
    hw = st[:, 0, 0]
    res = {
        "causal": causal, "dropout": p, "ms": round(ms, 4), "workgroups": int(nblk),
        "tiles_per_wg": int(ntile), "span_us": round(float(span) / cyc_per_us, 2),
        "wg_us_mean": round(us(wg_dur), 2),
        "wg_us_min": round(float(wg_dur.min()) / cyc_per_us, 2),
        "wg_us_max": round(float(wg_dur.max()) / cyc_per_us, 2),
        "prologue_us": round(us(pro.max(axis=1) - ent.min(axis=1)), 2),
        "tile_us_mean": round(us(wg_tile[:, 0, :]), 3),
        "tile_compute_slowest_us": round(us(slow), 3),
        "tile_compute_fastest_us": round(us(fast), 3),
        "tile_barrier_wait_us": round(us(wait), 3),
        "tiles_us_per_wg": round(us(wg_tile[:, 0, :].sum(axis=1)), 2),
        "finish_us": round(us(end.max(axis=1) - fin0.min(axis=1)), 2),
        "start_spread_us": round(float(np.percentile(ent.min(axis=1) - t0, 99)) / cyc_per_us, 2),
        "distinct_hw": int(len(np.unique(hw))),
    }
    # per tile position: mean WG tile time and wave imbalance
    res["tile_us_by_pos"] = [round(float(np.mean(wg_tile[:, 0, i])) / cyc_per_us, 3)
                             for i in range(ntile)]
    res["imbalance_us_by_pos"] = [round(float(np.mean(slow[:, i] - fast[:, i])) / cyc_per_us, 3)
                                  for i in range(ntile)]
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=8)
    ap.add_argument("--s", type=int, default=1024)
    ap.add_argument("--h", type=int, default=32)
    ap.add_argument("--d", type=int, default=128)
    args = ap.parse_args()
    for causal in (True, False):
        for p in (0.0, 0.1):
            print(json.dumps(run(args, causal, p)), flush=True)


if __name__ == "__main__":
    main()

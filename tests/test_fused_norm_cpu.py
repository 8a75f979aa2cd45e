"""The fused gradient norm's launch plan (``FlatParamGradBuffer._fused_norm_plan``)
on the CPU: the (address, length) chunks the segmented sum-of-squares kernel
reads must cover every gradient element exactly once -- squared where it is a
raw gradient, summed as-is where it is an epilogue slot -- whatever subset of
weights produced epilogue partials this step.  The kernel is emulated by
reading the chunks through ctypes."""
import ctypes

import pytest
import torch
import torch.nn as nn

from fleetx_amd.ops import gemm as G
from fleetx_amd.parallel.grad_buffer import FlatParamGradBuffer


def _buffer():
    torch.manual_seed(0)
    emb = nn.Embedding(100, 64)
    m = nn.Sequential(nn.Linear(64, 128), nn.LayerNorm(128), nn.Linear(128, 64),
                      nn.Linear(64, 300))
    named = list(emb.named_parameters(prefix="emb")) + list(m.named_parameters())
    for n, p in named:
        if p.dim() == 2 and not n.startswith("emb"):
            p._fx_fused_wgrad_ok = True
            p._fx_gemm_wgrad = True
    buf = FlatParamGradBuffer(named)
    # enable_fused_norm() needs a GPU; set the slots up the same way here
    buf._fused_norm = {}
    for c in buf.categories:
        elig = [p for n, p in c.params if getattr(p, "_fx_gemm_wgrad", False)]
        if not elig:
            continue
        sizes = [G.sq_slots(*p.shape) for p in elig]
        slots = torch.zeros(sum(sizes))
        o = 0
        for p, k in zip(elig, sizes):
            p._fx_sq = slots[o:o + k]
            o += k
        buf._fused_norm[id(c)] = (slots, elig)
    return buf


def _emulate(addr, lens, nch, nd, extra=None):
    part = []
    for a, n in zip(addr.tolist()[:nch], lens.tolist()[:nch]):
        vals = (ctypes.c_float * abs(n)).from_address(a)
        part.append(sum(float(x) for x in vals) if n < 0 else sum(float(x) ** 2 for x in vals))
    ex = extra or {True: [], False: []}   # uncovered 16-bit gradients (summed by torch)
    return (sum(part[:nd]) + sum(float(t.double().pow(2).sum()) for t in ex[True]),
            sum(part[nd:]) + sum(float(t.double().pow(2).sum()) for t in ex[False]))


@pytest.mark.parametrize("covered", ["all", "some", "none"])
def test_plan_covers_every_gradient_once(covered):
    buf = _buffer()
    buf.grad_flat.normal_()
    elig = [p for _, e in buf._fused_norm.values() for p in e]
    assert len(elig) == 3
    for i, p in enumerate(elig):
        ok = covered == "all" or (covered == "some" and i % 2 == 0)
        p._fx_sq_ok = ok
        p._fx_sq.zero_()
        if ok:  # what the epilogue leaves: per-wave partials, any split
            sq = p.main_grad.double().pow(2).sum()
            p._fx_sq[0] = sq * 0.25
            p._fx_sq[3] = sq * 0.75
    okey = tuple(p._fx_sq_ok for p in elig)
    dist_sq, rep_sq = _emulate(*buf._fused_norm_plan(okey))
    ref = float(buf.grad_flat.double().pow(2).sum())
    assert dist_sq == 0.0  # nothing is tensor-parallel here
    assert abs(rep_sq - ref) < 1e-4 * ref, (rep_sq, ref)

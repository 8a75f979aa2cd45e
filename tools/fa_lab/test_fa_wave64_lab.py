"""The one-wave-per-SIMD backward passes of ``flash_attn.hip`` (D = 128): dK/dV
with 64 keys per wave (``dkdv64_body``, FLEETX_FA_DKDV64) and dQ with 64
queries per wave (``fa_bwd_dq64_kernel``, FLEETX_FA_DQ64), against the
32-per-wave passes they replace and against the fp32 reference.  Each runs
the same MFMA sequence per 32-row block as the pass it replaces, so dQ / dK /
dV must agree bitwise.  ``vreg``: the 2-wave dK/dV pass with V in registers
(``fa_bwd_dkdv_v128_kernel``, FLEETX_FA_DKDV_VREG).  Shapes cover a key tail (Sk not a multiple of the 256-key
workgroup), causal + dropout, key lengths and fp16."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
# lab-only kernels: run with the lab library, e.g.
#   python tools/fa_lab/build.py && FLEETX_KERNELS_LIB=tools/fa_lab/_kernels*.so \
#     python -m pytest tools/fa_lab/test_fa_wave64_lab.py


@pytest.fixture(autouse=True)
def _lab_library():
    from fleetx_amd.ops import _lib
    if not _lib.kernels().fa_lab():
        pytest.skip("production kernel library: build tools/fa_lab (FLEETX_KERNELS_LIB)")


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _grads(ops, q, k, v, g, **kw):
    q, k, v = [t.detach().clone().requires_grad_() for t in (q, k, v)]
    out = ops.flash_attention(q, k, v, **kw)
    out.backward(g)
    return q.grad, k.grad, v.grad


@pytest.mark.parametrize("variant", ["wave64", "vreg"])
@pytest.mark.parametrize("case", ["causal_drop", "causal", "full_kvlens", "causal_fp16"])
def test_dkdv64_bitwise_and_reference(case, variant):
    from fleetx_amd import ops
    from fleetx_amd.ops import _lib
    k_ = _lib.kernels()
    dtype = torch.float16 if case == "causal_fp16" else torch.bfloat16
    B, S, H, D = 2, 600, 3, 128
    torch.manual_seed(0)
    q, k, v = [(0.5 * torch.randn(B, S, H, D, device=DEV)).to(dtype) for _ in range(3)]
    g = torch.randn(B, S, H, D, device=DEV).to(dtype)
    kw = dict(causal=case != "full_kvlens")
    if case == "causal_drop":
        kw.update(dropout_p=0.1, key=987654321)
    if case == "full_kvlens":
        kw["kv_lens"] = torch.tensor([333, 600], device=DEV, dtype=torch.int32)
    try:
        k_.fa_set_dkdv64(0)
        k_.fa_set_dq64(0)
        k_.fa_set_dkdv_vreg(0)
        base = _grads(ops, q, k, v, g, **kw)
        if variant == "wave64":
            k_.fa_set_dkdv64(1)
            k_.fa_set_dq64(1)
        else:
            k_.fa_set_dkdv_vreg(1)
        new = _grads(ops, q, k, v, g, **kw)
    finally:
        k_.fa_set_dkdv64(-1)
        k_.fa_set_dq64(-1)
        k_.fa_set_dkdv_vreg(-1)
    torch.cuda.synchronize()
    for a, b in zip(new, base):
        if dtype == torch.float16:
            # fp16: the production row store (store_row16) lets hipcc fold the
            # scale multiply and the conversion into one v_fma_mix (a single
            # rounding); the lab kernels round twice -- at most one ulp apart
            d = (a.float() - b.float()).abs()
            assert bool((d <= b.float().abs() * 2.0 ** -10 + 2.0 ** -24).all()), d.max()
        else:
            assert torch.equal(a, b), (a.float() - b.float()).abs().max()
    qr, kr, vr = [t.detach().float().requires_grad_() for t in (q, k, v)]
    ref = ops.attention_reference(qr, kr, vr, **kw)
    ref.backward(g.float())
    for a, r in ((new[0], qr.grad), (new[1], kr.grad), (new[2], vr.grad)):
        assert _rel(a, r) < 3e-2, _rel(a, r)

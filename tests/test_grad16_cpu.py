"""16-bit gradient storage (``Distributed.comm.grad_dtype``; reference O2
``GradStorage`` in the parameter dtype, ``tensor_fusion_helper.py:56,72-74``):
GEMM-written weight matrices keep their gradient in bf16 inside the fp32 flat
buffer's own bytes, everything else stays fp32, and one update matches the
fp32-gradient update within bf16 rounding of the gradient."""
import pytest
import torch
import torch.nn as nn

from fleetx_amd.parallel.grad_buffer import FlatParamGradBuffer, grad16_eligible
from fleetx_amd.parallel.linear import linear
from fleetx_amd.optims.optimizer import FusedAdamW, ClipGradByGlobalNorm


class _Toy(nn.Module):
    def __init__(self, h=64, dt=torch.bfloat16):
        super().__init__()
        self.w1 = nn.Parameter(torch.randn(2 * h, h, dtype=dt) * 0.05)
        self.b1 = nn.Parameter(torch.zeros(2 * h, dtype=dt))
        self.w2 = nn.Parameter(torch.randn(h, 2 * h, dtype=dt) * 0.05)
        self.gain = nn.Parameter(torch.ones(h, dtype=dt))
        for w in (self.w1, self.w2):
            w._fx_fused_wgrad_ok = True
            w._fx_gemm_wgrad = True

    def forward(self, x):
        y = torch.relu(linear(x, self.w1, self.b1))
        return (linear(y, self.w2) * self.gain).float().pow(2).mean()


def _run(grad_dtype, steps=2):
    torch.manual_seed(0)
    m = _Toy()
    buf = FlatParamGradBuffer(m.named_parameters(), grad_dtype=grad_dtype)
    opt = FusedAdamW(1e-2, buf, grad_clip=ClipGradByGlobalNorm(1.0))
    g = torch.Generator().manual_seed(1)
    for _ in range(steps):
        x = torch.randn(32, 64, generator=g).to(torch.bfloat16)
        m(x).backward()
        grads = {n: p.main_grad.float().clone() for n, p in m.named_parameters()}
        buf.finish()
        opt.step()
        opt.clear_grad()
    return m, buf, opt, grads


def test_grad16_layout_and_aliasing():
    m, buf, _, _ = _run(torch.bfloat16, steps=1)
    assert grad16_eligible(m.w1) and not grad16_eligible(m.b1)
    assert m.w1.main_grad.dtype == torch.bfloat16 and m.w2.main_grad.dtype == torch.bfloat16
    assert m.b1.main_grad.dtype == torch.float32 and m.gain.main_grad.dtype == torch.float32
    # the 16-bit gradients live inside the fp32 flat buffer's storage (no extra memory)
    lo = buf.grad_flat.data_ptr()
    hi = lo + buf.grad_flat.numel() * 4
    assert lo <= m.w1.main_grad.data_ptr() < hi
    cats = [c for c in buf.categories if c.grad16]
    assert len(cats) == 1 and {id(p) for _, p in cats[0].params} == {id(m.w1), id(m.w2)}
    # every owned range reports its storage dtype to the optimizer
    dts = {c.grad16: buf.grad_slice(c.start, c.end).dtype for c in buf.categories}
    assert dts == {True: torch.bfloat16, False: torch.float32}


def test_grad16_update_matches_fp32_gradients():
    m16, _, opt16, g16 = _run(torch.bfloat16)
    m32, _, opt32, g32 = _run(torch.float32)
    for n in g32:  # the gradients agree to bf16 rounding
        assert torch.allclose(g16[n], g32[n], rtol=1e-2, atol=1e-5), n
    for (n, a), (_, b) in zip(m16.named_parameters(), m32.named_parameters()):
        # masters after two AdamW steps: within a small fraction of the update
        assert torch.allclose(a.float(), b.float(), rtol=2e-2, atol=2e-3), n
    assert abs(float(opt16.last_grad_norm) - float(opt32.last_grad_norm)) < \
        1e-2 * float(opt32.last_grad_norm)


def test_grad16_only_in_the_model_dtype_and_unsharded():
    torch.manual_seed(0)
    m = _Toy(dt=torch.float32)
    buf = FlatParamGradBuffer(m.named_parameters(), grad_dtype=torch.bfloat16)
    assert buf.grad_dtype == torch.float32
    assert all(p.main_grad.dtype == torch.float32 for _, p in m.named_parameters())


def test_grad16_accumulates_micro_batches():
    """Micro-batch accumulation keeps 16-bit gradient storage (each
    micro-batch adds into it: one fp32 add + one rounding per write, as the
    reference's 16-bit GradStorage accumulates) and matches the fp32-storage
    accumulation to bf16 rounding."""
    grads = {}
    for gd in (torch.bfloat16, torch.float32):
        torch.manual_seed(0)
        m = _Toy()
        buf = FlatParamGradBuffer(m.named_parameters(), grad_dtype=gd)
        g = torch.Generator().manual_seed(1)
        for mb in range(2):
            buf.set_last_micro_batch(mb == 1)
            m(torch.randn(32, 64, generator=g).to(torch.bfloat16)).backward()
        buf.finish()
        assert m.w1.main_grad.dtype == (torch.bfloat16 if gd == torch.bfloat16 else torch.float32)
        grads[gd] = {n: p.main_grad.float().clone() for n, p in m.named_parameters()}
    for n in grads[torch.float32]:
        a, b = grads[torch.bfloat16][n], grads[torch.float32][n]
        assert torch.allclose(a, b, rtol=2e-2, atol=2e-4), (n, (a - b).abs().max())


def _dp_rank(rank, world, grad_dtype):
    from fleetx_amd.parallel import topology as topo
    topo.reset_hcg()
    hcg = topo.init_hcg(dp=world)
    torch.manual_seed(0)
    m = _Toy()
    buf = FlatParamGradBuffer(m.named_parameters(), dp_group=hcg.get_data_parallel_group(),
                              grad_dtype=grad_dtype, reduce_dtype=torch.bfloat16)
    g = torch.Generator().manual_seed(1 + rank)
    x = torch.randn(32, 64, generator=g).to(torch.bfloat16)
    m(x).backward()
    buf.finish()
    return {n: p.main_grad.float().clone() for n, p in m.named_parameters()}


def test_grad16_data_parallel_reduction():
    """The 16-bit gradient buckets are all-reduced in place (no wire copy) and
    averaged; they match the fp32-storage reduction to bf16 rounding."""
    from tests import dist_utils
    a = dist_utils.run(_dp_rank, 2, torch.bfloat16)
    b = dist_utils.run(_dp_rank, 2, torch.float32)
    for n in a[0]:
        assert torch.equal(a[0][n], a[1][n]), n          # every rank holds the same mean
        assert torch.allclose(a[0][n], b[0][n], rtol=2e-2, atol=1e-5), n


def test_sequence_parallel_weights_keep_fp32_gradients():
    """The SP-overlapped backward writes a weight's gradient chunk by chunk
    (``parallel/sp_overlap.py _wgrad_chunks``): 16-bit storage would round it
    once per chunk, so those weights are not eligible."""
    from fleetx_amd.parallel import layers as L
    from fleetx_amd.parallel import topology as topo
    old = topo.mp_world_size
    try:
        topo.mp_world_size = lambda: 2  # construction only reads the TP degree
        col = L.ColumnParallelLinear(32, 64, sequence_parallel=True, dtype=torch.bfloat16)
        row = L.RowParallelLinear(64, 32, sequence_parallel=True, dtype=torch.bfloat16)
        plain = L.ColumnParallelLinear(32, 64, sequence_parallel=False, dtype=torch.bfloat16)
    finally:
        topo.mp_world_size = old
    assert not grad16_eligible(col.weight) and not grad16_eligible(row.weight)
    assert grad16_eligible(plain.weight)

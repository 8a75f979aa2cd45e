"""Packed fp32 master (``Optimizer.packed_master``): the bf16 parameter is the
master's high half (rounded to nearest on the low half, ties toward zero) and
a 16-bit array keeps the low half, so the master is exact fp32 while the
update moves 26 instead of 28 B per parameter.

Reference parity: ``multi_precision`` AdamW keeps an fp32 master per bf16 /
fp16 parameter (``ppfleetx/optims/optimizer.py:29-50``); here the same fp32
values, stored split.  Checked against the unpacked path bitwise."""
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _k():
    from fleetx_amd.ops import _lib
    return _lib.kernels(), _lib.stream()


def test_split_join_roundtrip_and_rounding():
    k, st = _k()
    torch.manual_seed(0)
    x = torch.cat([torch.randn(1 << 20, device="cuda") * s for s in (1e-30, 1e-3, 1.0, 1e4)])
    x = torch.cat([x, torch.tensor([0.0, -0.0, 1.0, -1.0, 3.0e38], device="cuda")])
    n = x.numel()
    hi = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    lo = torch.empty(n, dtype=torch.int16, device="cuda")
    k.pk_split(x.data_ptr(), hi.data_ptr(), lo.data_ptr(), n, st)
    back = torch.empty_like(x)
    k.pk_join(hi.data_ptr(), lo.data_ptr(), back.data_ptr(), n, st)
    torch.cuda.synchronize()
    assert torch.equal(back.view(torch.int32), x.view(torch.int32))  # every fp32 bit kept
    # the parameter half is the round-to-nearest bf16 value except at exact ties
    low = x.view(torch.int32) & 0xFFFF
    rne = x.to(torch.bfloat16)
    tie = low == 0x8000
    assert torch.equal(hi[~tie].view(torch.int16), rne[~tie].view(torch.int16))


class _Toy(nn.Module):
    def __init__(self):
        super().__init__()
        self.w = nn.Parameter((torch.randn(512, 384) * 0.05).bfloat16())
        self.b = nn.Parameter(torch.zeros(512, dtype=torch.bfloat16))
        self.g = nn.Parameter(torch.ones(384, dtype=torch.bfloat16))
        self.w._fx_fused_wgrad_ok = True  # a GEMM-written weight: bf16 gradient storage
        self.w._fx_gemm_wgrad = True


def _train(packed, steps=3, g16=False):
    from fleetx_amd.parallel.grad_buffer import FlatParamGradBuffer
    from fleetx_amd.optims.optimizer import FusedAdamW, ClipGradByGlobalNorm
    torch.manual_seed(0)
    m = _Toy().cuda()
    buf = FlatParamGradBuffer(m.named_parameters(), grad_dtype=torch.bfloat16 if g16 else
                              torch.float32)
    opt = FusedAdamW(3e-3, buf, grad_clip=ClipGradByGlobalNorm(1.0), weight_decay=0.1,
                     packed_master=packed)
    assert (opt._lo is not None) == packed
    gen = torch.Generator(device="cuda").manual_seed(1)
    for _ in range(steps):
        for n_, p in m.named_parameters():
            p.main_grad.copy_(torch.randn(p.shape, device="cuda", generator=gen) * 0.1)
            p._fx_fresh = False
        buf.finish()
        opt.step()
        opt.clear_grad()
    torch.cuda.synchronize()
    return m, opt


@pytest.mark.parametrize("g16", [False, True])
def test_packed_update_is_bitwise_the_fp32_master_update(g16):
    m0, o0 = _train(False, g16=g16)
    m1, o1 = _train(True, g16=g16)
    for a, b in zip(o0.master, o1.master):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    for (n, a), (_, b) in zip(m0.named_parameters(), m1.named_parameters()):
        diff = (a.view(torch.int16) != b.view(torch.int16)).float().mean().item()
        assert diff < 1e-3, (n, diff)  # round-half-down vs half-even on exact ties only


def test_packed_state_dict_roundtrip():
    m, opt = _train(True, steps=2)
    sd = opt.state_dict()
    ref = [x.clone() for x in opt.master]
    params = [p.detach().clone() for p in m.parameters()]
    for lo in opt._lo:  # clobber, then restore from the checkpoint
        lo.fill_(123)
    opt.set_state_dict(sd)
    torch.cuda.synchronize()
    for a, b in zip(opt.master, ref):
        assert torch.equal(a.cpu(), b.cpu())
    for p, q in zip(m.parameters(), params):
        assert torch.equal(p.detach(), q)

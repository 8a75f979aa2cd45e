"""Optimizer / loss-scaler semantics: an fp16-overflow step
does not advance Adam's bias corrections; Adam's L2 term is added after
clipping; the scaler halves only after N consecutive overflows.  CPU tests run
the reference math; the GPU tests drive the HIP ``adamw_flat`` kernel against
an fp32 PyTorch oracle."""
import pytest
import torch


def _make(device, decoupled=True, clip=None, wd=0.1):
    from fleetx_amd.parallel.grad_buffer import FlatParamGradBuffer
    from fleetx_amd.optims import optimizer as O
    torch.manual_seed(0)
    lin = torch.nn.Linear(32, 48).to(device)
    if device == "cuda":
        lin = lin.bfloat16()
    buf = FlatParamGradBuffer(lin.named_parameters())
    cls = O.FusedAdamW if decoupled else O.Adam
    opt = cls(1e-2, buf, grad_clip=O.ClipGradByGlobalNorm(clip) if clip else None,
              weight_decay=wd)
    return lin, buf, opt


def _grad_step(lin, buf, opt, x, inject_inf=False):
    lin(x.to(next(lin.parameters()).dtype)).float().pow(2).mean().backward()
    buf.finish()
    if inject_inf:
        buf.grad_flat[0] = float("inf")
    opt.step()
    opt.clear_grad()


def _torch_adam(params, grads_per_step, lr, wd, decoupled, clip):
    ref = [p.detach().float().clone().requires_grad_(True) for p in params]
    if decoupled:
        topt = torch.optim.AdamW([{"params": [ref[0]], "weight_decay": wd},
                                  {"params": [ref[1]], "weight_decay": 0.0}], lr=lr, eps=1e-8)
    else:
        topt = torch.optim.Adam([{"params": [ref[0]], "weight_decay": wd},
                                 {"params": [ref[1]], "weight_decay": 0.0}], lr=lr, eps=1e-8)
    for gs in grads_per_step:
        for r, g in zip(ref, gs):
            r.grad = g.clone()
        if clip:
            torch.nn.utils.clip_grad_norm_(ref, clip)   # torch Adam adds L2 after this too
        topt.step()
        topt.zero_grad()
    return ref


@pytest.mark.parametrize("decoupled", [True, False])
def test_overflow_step_does_not_age_adam_cpu(decoupled):
    """A skipped (found-inf) step in the middle leaves the result identical to
    the run without it (bias corrections follow applied updates only)."""
    torch.manual_seed(1)
    xs = [torch.randn(16, 32) for _ in range(3)]
    lin_a, buf_a, opt_a = _make("cpu", decoupled, clip=0.5)
    lin_b, buf_b, opt_b = _make("cpu", decoupled, clip=0.5)
    opt_b.loss_scale = torch.ones(())        # fp16-style path: found-inf detection on
    opt_a.loss_scale = torch.ones(())
    _grad_step(lin_a, buf_a, opt_a, xs[0])
    _grad_step(lin_b, buf_b, opt_b, xs[0])
    _grad_step(lin_b, buf_b, opt_b, xs[1], inject_inf=True)   # skipped on b only
    _grad_step(lin_a, buf_a, opt_a, xs[2])
    _grad_step(lin_b, buf_b, opt_b, xs[2])
    assert int(opt_b.dev_step.item()) == 2 and opt_b.step_count == 3
    for pa, pb in zip(lin_a.parameters(), lin_b.parameters()):
        assert torch.equal(pa, pb)


def test_adam_l2_after_clip_matches_torch_cpu():
    torch.manual_seed(2)
    lin, buf, opt = _make("cpu", decoupled=False, clip=0.05, wd=0.3)
    p0 = [p.detach().clone() for p in lin.parameters()]
    grads = []
    for _ in range(3):
        x = torch.randn(16, 32)
        lin(x).float().pow(2).mean().backward()
        buf.finish()
        grads.append([p.main_grad.clone() for _, p in buf.params])
        opt.step()
        opt.clear_grad()
    ref = _torch_adam(p0, grads, 1e-2, 0.3, decoupled=False, clip=0.05)
    for p, r in zip(lin.parameters(), ref):
        assert torch.allclose(p, r, rtol=1e-5, atol=1e-6)


def test_loss_scaler_consecutive_overflows():
    from fleetx_amd.core.engine.eager_engine import DynamicLossScaler
    s = DynamicLossScaler(1024.0, incr_every=3, decr_every=2)
    one, zero = torch.ones(1, dtype=torch.int32), torch.zeros(1, dtype=torch.int32)
    s.update(one)
    assert float(s.scale) == 1024.0          # first overflow: keep
    s.update(one)
    assert float(s.scale) == 512.0           # second consecutive: halve
    s.update(one)
    s.update(zero)                           # finite step resets the bad streak
    s.update(one)
    assert float(s.scale) == 512.0
    for _ in range(3):
        s.update(zero)
    assert float(s.scale) == 1024.0          # 3 good steps: grow


@pytest.mark.gpu
@pytest.mark.parametrize("decoupled", [True, False])
def test_adamw_kernel_matches_torch_gpu(decoupled):
    """HIP adamw_flat (device step counter, clip, decoupled decay / L2) vs
    torch.optim on the same fp32 gradients, with one injected overflow."""
    torch.manual_seed(3)
    lin, buf, opt = _make("cuda", decoupled, clip=0.5, wd=0.1)
    opt.loss_scale = torch.ones((), device="cuda")
    p0 = [p.detach().float().clone() for p in lin.parameters()]
    grads = []
    for i in range(4):
        x = torch.randn(64, 32, device="cuda")
        lin(x.bfloat16()).float().pow(2).mean().backward()
        buf.finish()
        if i == 2:
            buf.grad_flat[0] = float("inf")
        else:
            grads.append([p.main_grad.float().clone() for _, p in buf.params])
        opt.step()
        opt.clear_grad()
    torch.cuda.synchronize()
    assert int(opt.dev_step.item()) == 3
    ref = _torch_adam(p0, grads, 1e-2, 0.1, decoupled, clip=0.5)
    full = torch.zeros(buf.param_flat.numel(), device="cuda")
    for (s, e, _), m in zip(opt.ranges, opt.master):
        full[s:e] = m
    ref_of = dict(zip([id(q) for q in lin.parameters()], ref))
    for _, p in buf.params:
        o, n = buf.offsets[id(p)][0], p.numel()
        got = full[o:o + n].view_as(p)
        assert float((got - ref_of[id(p)].detach()).abs().max()) < 1e-4, (decoupled, p.shape)

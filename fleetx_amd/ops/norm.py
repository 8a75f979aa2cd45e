"""LayerNorm with optional fused residual + bias + dropout prologue.

``add_layer_norm(x, bias, residual, w, b)`` returns ``(s, y)`` with
``s = residual + dropout(x + bias)`` (the new residual stream) and
``y = LayerNorm(s)``: the pre-LN transformer's "dropout + residual add,
then LN2" in one HBM pass (reference K07 + K09,
``single_model.py:393-394,412``).
"""
import os

import torch

from . import _lib
from ..parallel import rng as _rng


_TICKETS = {}


def colsum_tickets(device, cols):
    """Ticket array of the fused column-sum finalize (the last workgroup of a
    128-column tile sums the splits; csrc/kernels/norm_eltwise.hip
    ``colsum_tail``), one per stream: zeroed once, each launch's last
    workgroup resets its tiles' tickets.  One ticket per 128-byte line (32
    int32 per 128-column tile): arrivals on one line serialise."""
    st = torch.cuda.current_stream(device).cuda_stream
    need = 32 * ((cols + 127) // 128)
    t = _TICKETS.get(st)
    if t is None or t.numel() < need:
        t = torch.zeros(max(4096, need), dtype=torch.int32, device=device)
        _TICKETS[st] = t
    return t.data_ptr()


def _col_reduce_ln(dy, s, mean, rstd, cols, dtype):
    k = _lib.kernels()
    rows = dy.numel() // cols
    splits = k.coltile_splits(rows, cols)
    p0 = torch.empty(splits, cols, device=dy.device, dtype=torch.float32)
    p1 = torch.empty_like(p0)
    st = _lib.stream()
    dc = _lib.dt_code(dtype)
    dg = torch.empty(cols, device=dy.device, dtype=dtype)
    db = torch.empty(cols, device=dy.device, dtype=dtype)
    k.coltile_partial(dc, 0, dy.data_ptr(), s.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                      p0.data_ptr(), p1.data_ptr(), rows, cols, splits, st,
                      cnt=colsum_tickets(dy.device, cols), t0=dg.data_ptr(), t1=db.data_ptr())
    return dg, db


def _fused_param(p):
    return p is not None and getattr(p, "_fx_fused_wgrad", False) and hasattr(p, "main_grad")


def _into_main_grad(p, fill):
    """Write (first contribution of the step) or accumulate a parameter's
    gradient straight into its fp32 ``main_grad`` and report it ready."""
    from ..parallel.linear import grad_part_done
    fill(p.main_grad, not getattr(p, "_fx_fresh", False))
    p._fx_fresh = False
    grad_part_done(p)


def _col_reduce_ln_main_grad(dy, s, mean, rstd, cols, dtype, weight, lnbias):
    """LN weight/bias gradients reduced over rows straight into the fp32
    ``main_grad`` of both parameters (no 16-bit grad, no autograd copy)."""
    k = _lib.kernels()
    rows = dy.numel() // cols
    splits = k.coltile_splits(rows, cols)
    p0 = torch.empty(splits, cols, device=dy.device, dtype=torch.float32)
    p1 = torch.empty_like(p0)
    st = _lib.stream()
    dc = _lib.dt_code(dtype)
    acc = [int(not getattr(prm, "_fx_fresh", False)) for prm in (weight, lnbias)]
    k.coltile_partial(dc, 0, dy.data_ptr(), s.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                      p0.data_ptr(), p1.data_ptr(), rows, cols, splits, st,
                      cnt=colsum_tickets(dy.device, cols), f0=weight.main_grad.data_ptr(),
                      acc0=acc[0], f1=lnbias.main_grad.data_ptr(), acc1=acc[1])
    from ..parallel.linear import grad_part_done
    for prm in (weight, lnbias):
        prm._fx_fresh = False
        grad_part_done(prm)


def col_sum(x, cols):
    """Column sum of a [rows, cols] 16-bit tensor (fp32 accumulation)."""
    if not x.is_cuda:
        return x.reshape(-1, cols).float().sum(0).to(x.dtype)
    k = _lib.kernels()
    rows = x.numel() // cols
    splits = k.coltile_splits(rows, cols)
    p0 = torch.empty(splits, cols, device=x.device, dtype=torch.float32)
    st = _lib.stream()
    dc = _lib.dt_code(x.dtype)
    out = torch.empty(cols, device=x.device, dtype=x.dtype)
    k.coltile_partial(dc, 1, x.data_ptr(), 0, 0, 0, p0.data_ptr(), 0, rows, cols, splits, st,
                      cnt=colsum_tickets(x.device, cols), t0=out.data_ptr())
    return out


def col_sum_f32(x, dst, accumulate=False):
    """``dst (+)= x.reshape(-1, cols).sum(0)`` with ``dst`` a contiguous fp32
    vector (bias gradients straight into ``main_grad``)."""
    cols = dst.numel()
    if not x.is_cuda:
        s = x.reshape(-1, cols).float().sum(0).view_as(dst)
        if accumulate:
            dst.add_(s)
        else:
            dst.copy_(s)
        return dst
    if dst.dtype != torch.float32 or not dst.is_contiguous():
        raise ValueError("col_sum_f32: dst must be contiguous fp32")
    x = x.contiguous()
    k = _lib.kernels()
    rows = x.numel() // cols
    splits = k.coltile_splits(rows, cols)
    p0 = torch.empty(splits, cols, device=x.device, dtype=torch.float32)
    st = _lib.stream()
    dc = _lib.dt_code(x.dtype)
    k.coltile_partial(dc, 1, x.data_ptr(), 0, 0, 0, p0.data_ptr(), 0, rows, cols, splits, st,
                      cnt=colsum_tickets(x.device, cols), f0=dst.data_ptr(),
                      acc0=int(accumulate))
    return dst


def _dropout_ref(x, p, key):
    if p <= 0.0:
        return x
    m = _rng.keep_mask(x.shape, p, key, x.device)
    return torch.where(m, x * (1.0 / (1.0 - p)), torch.zeros_like(x))


def _ln_bwd_cols_max_h():
    """Widest LayerNorm the one-pass backward takes: FLEETX_LN_BWD_FUSED=0
    keeps the row kernel + column-tile passes everywhere, 1 (default) uses
    it up to h 1536 (one wave per row), 2 up to 4096 (2 / 4 waves per row:
    measured slower at 4096, neutral at 2048 -- profiles/r3_colsum/)."""
    mode = os.environ.get("FLEETX_LN_BWD_FUSED", "1")
    return {"0": 0, "2": 4096}.get(mode, 1536)


def _main_grad_target(p):
    return _fused_param(p) and p.main_grad.dtype == torch.float32 and p.main_grad.is_contiguous()


def _ln_bwd_cols(k, dc, dy, s, mean, rstd, weight, ctx, ds_in, ds, dx, rows, h):
    """LayerNorm backward and its column sums (dgamma, dbeta and, with a fused
    residual + bias, the bias gradient ``sum(dx)``) in one row pass plus one
    small finalize launch (csrc/kernels/norm_eltwise.hip ``ln_bwd_cols_kernel``)
    -- written into the fp32 ``main_grad`` where the parameter has one, else
    returned as 16-bit gradients."""
    G = k.ln_bwd_cols_blocks(rows, h, 4096)
    with_db = bool(ctx.has_bias)
    part = torch.empty(3 if with_db else 2, G, h, device=dy.device, dtype=torch.float32)
    outs, grads, done = [], [], []
    for prm, want in ((weight, True), (ctx.lnbias, True), (ctx.bias, with_db)):
        if not want:
            outs.append((0, 0, 0))
            grads.append(None)
        elif _main_grad_target(prm):
            outs.append((prm.main_grad.data_ptr(), 0, int(not getattr(prm, "_fx_fresh", False))))
            grads.append(None)
            done.append(prm)
        else:
            g = torch.empty(h, device=dy.device, dtype=dy.dtype)
            outs.append((0, g.data_ptr(), 0))
            grads.append(g)
    (fg, tg, ag), (fb, tb, ab), (fx, tx, ax) = outs
    rc = k.ln_bwd_cols(dc, dy.data_ptr(), s.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                       weight.data_ptr(), _lib.ptr(ds_in), ds.data_ptr(), dx.data_ptr(), rows, h,
                       float(ctx.p), ctx.key, part.data_ptr(), int(with_db), fg, tg, ag, fb, tb,
                       ab, fx, tx, ax, _lib.stream())
    if rc != 0:
        raise RuntimeError("ln_bwd_cols: shape rows=%d h=%d not covered" % (rows, h))
    if done:
        from ..parallel.linear import grad_part_done
        for prm in done:
            prm._fx_fresh = False
            grad_part_done(prm)
    return grads[0], grads[1], grads[2]


class _AddLayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, residual, weight, lnbias, eps, p, key, store_sum):
        h = x.shape[-1]
        rows = x.numel() // h
        ctx.p, ctx.key, ctx.has_bias, ctx.has_res = p, key, bias is not None, residual is not None
        ctx.h = h
        if x.is_cuda:
            k = _lib.kernels()
            x = x.contiguous()
            fused = bias is not None or residual is not None or p > 0
            # store_sum with nothing to add: s IS x (returned as an alias, no copy)
            s = torch.empty_like(x) if fused else None
            y = torch.empty_like(x)
            mean = torch.empty(rows, device=x.device, dtype=torch.float32)
            rstd = torch.empty_like(mean)
            k.add_ln_fwd(_lib.dt_code(x.dtype), x.data_ptr(), _lib.ptr(bias), _lib.ptr(residual),
                         weight.data_ptr(), lnbias.data_ptr(), _lib.ptr(s), y.data_ptr(),
                         mean.data_ptr(), rstd.data_ptr(), rows, h, float(eps), float(p), key,
                         _lib.stream())
            s_saved = s if s is not None else x
            if s is None and store_sum:
                s = x
        else:
            v = x if bias is None else x + bias
            v = _dropout_ref(v, p, key)
            if residual is not None:
                v = v + residual
            s_saved = v
            s = v if (store_sum or bias is not None or residual is not None or p > 0) else None
            vf = v.float()
            mean = vf.mean(-1).reshape(-1)
            var = ((vf - mean.view(*vf.shape[:-1], 1)) ** 2).mean(-1).reshape(-1)
            rstd = torch.rsqrt(var + eps)
            y = ((vf - mean.view(*vf.shape[:-1], 1)) * rstd.view(*vf.shape[:-1], 1) * weight.float()
                 + lnbias.float()).to(x.dtype)
        ctx.save_for_backward(s_saved, mean, rstd, weight)
        # parameters whose gradients may go straight into main_grad
        ctx.lnbias, ctx.bias = lnbias, bias
        ctx.return_sum = s is not None
        if s is None:
            return y
        return s, y

    @staticmethod
    def backward(ctx, *grads):
        if ctx.return_sum:
            ds_in, dy = grads
        else:
            ds_in, dy = None, grads[0]
        s, mean, rstd, weight = ctx.saved_tensors
        h = ctx.h
        rows = s.numel() // h
        dy = dy.contiguous()
        if ds_in is not None:
            ds_in = ds_in.contiguous()
        if dy.is_cuda:
            k = _lib.kernels()
            dc = _lib.dt_code(dy.dtype)
            ds = torch.empty_like(dy)
            dx = torch.empty_like(dy) if ctx.p > 0 else ds
            if k.ln_bwd_cols_blocks(rows, h, _ln_bwd_cols_max_h()) > 0:
                dw, db, dbias = _ln_bwd_cols(k, dc, dy, s, mean, rstd, weight, ctx, ds_in, ds, dx,
                                             rows, h)
                dres = ds if ctx.has_res else None
                return dx, dbias, dres, dw, db, None, None, None, None
            k.ln_bwd_row(dc, dy.data_ptr(), s.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                         weight.data_ptr(), _lib.ptr(ds_in), ds.data_ptr(), dx.data_ptr(), rows, h,
                         float(ctx.p), ctx.key, _lib.stream())
            if _fused_param(weight) and _fused_param(ctx.lnbias):
                _col_reduce_ln_main_grad(dy, s, mean, rstd, h, dy.dtype, weight, ctx.lnbias)
                dw = db = None
            else:
                dw, db = _col_reduce_ln(dy, s, mean, rstd, h, dy.dtype)
            dbias = None
            if ctx.has_bias:
                if _fused_param(ctx.bias):
                    _into_main_grad(ctx.bias, lambda mg, acc: col_sum_f32(dx, mg, acc))
                else:
                    dbias = col_sum(dx, h)
        else:
            sf = s.float().reshape(rows, h)
            xh = (sf - mean.view(rows, 1)) * rstd.view(rows, 1)
            g = dy.float().reshape(rows, h) * weight.float()
            m1 = g.mean(-1, keepdim=True)
            m2 = (g * xh).mean(-1, keepdim=True)
            dsf = rstd.view(rows, 1) * (g - m1 - xh * m2)
            if ds_in is not None:
                dsf = dsf + ds_in.float().reshape(rows, h)
            ds = dsf.to(dy.dtype).reshape(dy.shape)
            dx = _dropout_ref(ds, ctx.p, ctx.key)
            dw = (dy.float().reshape(rows, h) * xh).sum(0).to(weight.dtype)
            db = dy.float().reshape(rows, h).sum(0).to(weight.dtype)
            dbias = dx.float().reshape(rows, h).sum(0).to(dy.dtype) if ctx.has_bias else None
        dres = ds if ctx.has_res else None
        return dx, dbias, dres, dw, db, None, None, None, None


def add_layer_norm(x, bias, residual, weight, lnbias, eps=1e-5, p=0.0, key=0):
    """Returns ``(s, y)``: s = residual + dropout(x + bias), y = LN(s)."""
    return _AddLayerNorm.apply(x, bias, residual, weight, lnbias, eps, p, key, True)


def layer_norm(x, weight, bias, eps=1e-5):
    return _AddLayerNorm.apply(x, None, None, weight, bias, eps, 0.0, 0, False)


def layer_norm_keep_input(x, weight, bias, eps=1e-5):
    """``(x', LN(x))`` with ``x'`` an alias of ``x`` to use as the residual:
    the gradient that reaches ``x'`` enters the LayerNorm backward kernel as
    its ``ds_in`` instead of autograd adding the two branch gradients of
    ``x`` in a separate pass (pre-LN blocks: ``x + f(LN(x))``)."""
    return _AddLayerNorm.apply(x, None, None, weight, bias, eps, 0.0, 0, True)


class FusedLayerNorm(torch.nn.Module):
    """``nn.LayerNorm`` replacement routed through the HIP kernel."""

    def __init__(self, hidden, eps=1e-5, dtype=None, device=None):
        super().__init__()
        self.weight = torch.nn.Parameter(torch.ones(hidden, dtype=dtype, device=device))
        self.bias = torch.nn.Parameter(torch.zeros(hidden, dtype=dtype, device=device))
        # backward reduces the LN gradients straight into the fp32 main_grad
        self.weight._fx_fused_wgrad_ok = True
        self.bias._fx_fused_wgrad_ok = True
        self.eps = eps
        self.normalized_shape = (hidden,)

    def forward(self, x):
        return layer_norm(x, self.weight, self.bias, self.eps)

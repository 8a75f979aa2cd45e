"""Bias+GeLU, bias+dropout+residual-add and plain dropout.

Reference K08 (``F.gelu(approximate=True)`` after FFN1; ViT uses exact GeLU)
and K09 (``dropout(upscale_in_train)`` + residual).  The GEMM runs bias-free on
hipBLASLt; these kernels carry the epilogue and emit dbias from the same
pass as dx in backward.
"""
import math

import torch

from . import _lib
from .norm import _dropout_ref, col_sum


def _gelu_ref(x, erf):
    if erf:
        return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))
    return 0.5 * x * (1.0 + torch.tanh(0.7978845608028654 * (x + 0.044715 * x ** 3)))


def _gelu_grad_ref(x, erf):
    if erf:
        return 0.5 * (1.0 + torch.erf(x / math.sqrt(2.0))) + x * 0.3989422804014327 * torch.exp(-0.5 * x * x)
    u = 0.7978845608028654 * (x + 0.044715 * x ** 3)
    t = torch.tanh(u)
    return 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * 0.7978845608028654 * (1 + 3 * 0.044715 * x * x)


class _BiasGelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, erf):
        ctx.erf = erf
        ctx.has_bias = bias is not None
        x = x.contiguous()
        cols = x.shape[-1]
        if x.is_cuda:
            y = torch.empty_like(x)
            _lib.kernels().bias_gelu_fwd(_lib.dt_code(x.dtype), int(erf), x.data_ptr(),
                                         _lib.ptr(bias), y.data_ptr(), x.numel(), cols,
                                         _lib.stream())
        else:
            t = x.float() + (bias.float() if bias is not None else 0.0)
            y = _gelu_ref(t, erf).to(x.dtype)
        ctx.save_for_backward(x, bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, bias = ctx.saved_tensors
        dy = dy.contiguous()
        cols = x.shape[-1]
        rows = x.numel() // cols
        if dy.is_cuda:
            k = _lib.kernels()
            splits = k.coltile_splits(rows, cols)
            part = torch.empty(splits, cols, device=x.device, dtype=torch.float32)
            dx = torch.empty_like(x)
            dc = _lib.dt_code(x.dtype)
            st = _lib.stream()
            db = None
            fin = {}
            if ctx.has_bias:
                db = torch.empty(cols, device=x.device, dtype=bias.dtype)
                from .norm import colsum_tickets
                fin = {"cnt": colsum_tickets(x.device, cols), "out_t": db.data_ptr()}
            k.bias_gelu_bwd(dc, int(ctx.erf), dy.data_ptr(), x.data_ptr(), _lib.ptr(bias),
                            dx.data_ptr(), part.data_ptr(), rows, cols, splits, st, **fin)
        else:
            t = x.float() + (bias.float() if bias is not None else 0.0)
            dx = (dy.float() * _gelu_grad_ref(t, ctx.erf)).to(x.dtype)
            db = dx.float().reshape(rows, cols).sum(0).to(bias.dtype) if ctx.has_bias else None
        return dx, db, None


def bias_gelu(x, bias=None, approximate=True):
    return _BiasGelu.apply(x, bias, not approximate)


def gelu_plain(h, erf=False):
    """``gelu(h)`` without autograd (fallback half of the fused FC1 epilogue)."""
    h = h.contiguous()
    if h.is_cuda:
        y = torch.empty_like(h)
        _lib.kernels().bias_gelu_fwd(_lib.dt_code(h.dtype), int(erf), h.data_ptr(), 0,
                                     y.data_ptr(), h.numel(), h.shape[-1], _lib.stream())
        return y
    return _gelu_ref(h.float(), erf).to(h.dtype)


def gelu_grad(dy, h, erf=False, colsum=None):
    """``dy * gelu'(h)`` without autograd (fallback of the fused dGeLU epilogue).
    ``colsum = (dst_f32, accumulate)`` also writes / adds the column sums of the
    result (a bias gradient) from the same pass."""
    dy = dy.contiguous()
    h = h.contiguous()
    if dy.is_cuda:
        k = _lib.kernels()
        cols = h.shape[-1]
        rows = h.numel() // cols
        splits = k.coltile_splits(rows, cols)
        part = torch.empty(splits, cols, device=h.device, dtype=torch.float32)
        dx = torch.empty_like(h)
        dc = _lib.dt_code(h.dtype)
        fin = {}
        if colsum is not None:
            dst, acc = colsum
            from .norm import colsum_tickets
            fin = {"cnt": colsum_tickets(h.device, cols), "out_f32": dst.data_ptr(),
                   "acc": int(acc)}
        k.bias_gelu_bwd(dc, int(erf), dy.data_ptr(), h.data_ptr(), 0,
                        dx.data_ptr(), part.data_ptr(), rows, cols, splits, _lib.stream(), **fin)
        return dx
    dx = (dy.float() * _gelu_grad_ref(h.float(), erf)).to(h.dtype)
    if colsum is not None:
        dst, acc = colsum
        s = dx.float().reshape(-1, dst.numel()).sum(0).view_as(dst)
        dst.add_(s) if acc else dst.copy_(s)
    return dx


class _BiasDropoutAdd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, residual, p, key):
        ctx.p, ctx.key = p, key
        ctx.bias = bias
        ctx.has_bias, ctx.has_res = bias is not None, residual is not None
        x = x.contiguous()
        cols = x.shape[-1]
        ctx.cols = cols
        if x.is_cuda:
            out = torch.empty_like(x)
            if residual is not None:
                residual = residual.contiguous()
            _lib.kernels().bias_dropout_add_fwd(_lib.dt_code(x.dtype), x.data_ptr(),
                                                _lib.ptr(bias), _lib.ptr(residual),
                                                out.data_ptr(), x.numel(), cols, float(p), key,
                                                _lib.stream())
        else:
            v = x if bias is None else x + bias
            v = _dropout_ref(v, p, key)
            out = v + residual if residual is not None else v
        return out

    @staticmethod
    def backward(ctx, dout):
        dout = dout.contiguous()
        cols = ctx.cols
        rows = dout.numel() // cols
        dres = dout if ctx.has_res else None
        if dout.is_cuda:
            k = _lib.kernels()
            dc = _lib.dt_code(dout.dtype)
            st = _lib.stream()
            dx = torch.empty_like(dout) if ctx.p > 0 else dout
            db = None
            if ctx.has_bias:
                splits = k.coltile_splits(rows, cols)
                part = torch.empty(splits, cols, device=dout.device, dtype=torch.float32)
                from .norm import colsum_tickets
                bias = ctx.bias
                fused = bias is not None and getattr(bias, "_fx_fused_wgrad", False) \
                    and hasattr(bias, "main_grad")
                if fused:  # fp32 bias gradient straight into main_grad
                    fin = {"out_f32": bias.main_grad.data_ptr(),
                           "acc": int(not getattr(bias, "_fx_fresh", False))}
                else:
                    db = torch.empty(cols, device=dout.device, dtype=dout.dtype)
                    fin = {"out_t": db.data_ptr()}
                k.dropout_bwd_colsum(dc, dout.data_ptr(), dx.data_ptr() if ctx.p > 0 else 0,
                                     part.data_ptr(), rows, cols, splits, float(ctx.p), ctx.key, st,
                                     cnt=colsum_tickets(dout.device, cols), **fin)
                if fused:
                    from ..parallel.linear import grad_part_done
                    bias._fx_fresh = False
                    grad_part_done(bias)
            elif ctx.p > 0:
                k.dropout_fwd(dc, dout.data_ptr(), dx.data_ptr(), dout.numel(), float(ctx.p),
                              ctx.key, st)
        else:
            dx = _dropout_ref(dout, ctx.p, ctx.key)
            db = dx.float().reshape(rows, cols).sum(0).to(dout.dtype) if ctx.has_bias else None
        return dx, db, dres, None, None


def bias_dropout_add(x, bias, residual, p=0.0, key=0):
    """``residual + dropout(x + bias)`` with a counter-hash mask."""
    return _BiasDropoutAdd.apply(x, bias, residual, float(p), key)


def _dropout_apply(x, p, key):
    x = x.contiguous()
    if x.is_cuda:
        y = torch.empty_like(x)
        _lib.kernels().dropout_fwd(_lib.dt_code(x.dtype), x.data_ptr(), y.data_ptr(),
                                   x.numel(), float(p), key, _lib.stream())
        return y
    return _dropout_ref(x, p, key)


class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, key):
        ctx.p, ctx.key = p, key
        return _dropout_apply(x, p, key)

    @staticmethod
    def backward(ctx, dy):
        return _dropout_apply(dy, ctx.p, ctx.key), None, None


def dropout(x, p, key):
    if p <= 0.0:
        return x
    return _Dropout.apply(x, float(p), key)


__all__ = ["bias_gelu", "bias_dropout_add", "dropout", "col_sum"]


def transpose2d(x, out=None, colsum=None):
    """``x.t().contiguous()`` for a 2-D 16-bit tensor via the LDS-tiled HIP
    transpose (csrc/kernels/layout.hip); rows may be strided (``x.stride(1)``
    must be 1).  CPU tensors and shapes that are not multiples of 8 use
    PyTorch's copy.

    ``colsum``: optional ``(out_f32, accumulate)`` -- the fp32 column sums of
    ``x`` (a bias gradient) are written to / added into ``out_f32`` as a side
    product of the same pass."""
    if x.dim() != 2:
        raise ValueError("transpose2d expects a 2-D tensor")
    R, C = x.shape
    if out is None:
        out = torch.empty((C, R), dtype=x.dtype, device=x.device)
    if not _lib.on_gpu(x) or x.dtype not in (torch.bfloat16, torch.float16) or x.stride(1) != 1 \
            or (R | C | x.stride(0)) % 8 or not out.is_contiguous() \
            or x.data_ptr() % 16 or out.data_ptr() % 16:
        out.copy_(x.t())
        if colsum is not None:
            dst, acc = colsum
            s = x.float().sum(0)
            if acc:
                dst.add_(s.view_as(dst))
            else:
                dst.copy_(s.view_as(dst))
        return out
    k = _lib.kernels()
    part = None
    if colsum is not None:
        part = torch.empty(((R + 63) // 64, C), device=x.device, dtype=torch.float32)
    dc = _lib.dt_code(x.dtype)
    rc = k.transpose16(dc, _lib.ptr(x), _lib.ptr(out), _lib.ptr(part), R, C, x.stride(0), R,
                       _lib.stream())
    if rc != 0:
        raise RuntimeError("transpose16 launch failed ({})".format(rc))
    if colsum is not None:
        dst, acc = colsum
        if dst.dtype != torch.float32 or not dst.is_contiguous():
            raise ValueError("colsum target must be contiguous fp32")
        k.coltile_finalize(dc, part.data_ptr(), part.shape[0], C, dst.data_ptr(), 0, int(acc),
                           _lib.stream())
    _lib.maybe_sync()
    return out

"""Fused GroupNorm (+ FiLM scale/shift) (+ SiLU) on NCHW activations.

``y = silu((GN(x) * gamma + beta) * (1 + scale) + shift)`` with ``scale`` /
``shift`` per (batch, channel) — the Imagen UNet ``Block`` (reference
``imagen/unet.py:331-344``).  GPU: the two-pass HIP kernels of
``csrc/kernels/groupnorm.hip``; CPU: PyTorch reference math.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib


def group_norm_silu_reference(x, groups, weight, bias, scale=None, shift=None, eps=1e-5,
                              silu=True):
    y = F.group_norm(x.float(), groups, weight.float() if weight is not None else None,
                     bias.float() if bias is not None else None, eps)
    B, C = x.shape[:2]
    ext = (B, C) + (1,) * (x.dim() - 2)
    if scale is not None:
        y = y * (scale.float().reshape(ext) + 1)
    if shift is not None:
        y = y + shift.float().reshape(ext)
    if silu:
        y = F.silu(y)
    return y.to(x.dtype)


def _f32(t):
    return None if t is None else t.detach().float().contiguous()


class _GroupNormSiLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, scale, shift, groups, eps, silu):
        k = _lib.kernels()
        x = x.contiguous()
        B, C = x.shape[:2]
        hw = x.numel() // (B * C)
        nseg = k.gn_nseg(B * C, hw)
        y = torch.empty_like(x)
        part = torch.empty(B * C * nseg * 2, device=x.device, dtype=torch.float64)
        mean = torch.empty(B * groups, device=x.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        w, b, s, sh = _f32(weight), _f32(bias), _f32(scale), _f32(shift)
        rc = k.gn_fwd(_lib.dt_code(x.dtype), x.data_ptr(), _lib.ptr(w), _lib.ptr(b), _lib.ptr(s),
                      _lib.ptr(sh), y.data_ptr(), part.data_ptr(), mean.data_ptr(),
                      rstd.data_ptr(), B, C, groups, hw, nseg, float(eps), int(silu),
                      _lib.stream())
        if rc != 0:
            raise RuntimeError("gn_fwd failed (%d): C=%d groups=%d" % (rc, C, groups))
        _lib.maybe_sync()
        ctx.groups, ctx.silu, ctx.nseg, ctx.hw = groups, silu, nseg, hw
        ctx.has = (weight is not None, bias is not None, scale is not None, shift is not None)
        ctx.dtypes = tuple(t.dtype if t is not None else None for t in (weight, bias, scale, shift))
        ctx.save_for_backward(x, mean, rstd, w, b, s, sh)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, rstd, w, b, s, sh = ctx.saved_tensors
        k = _lib.kernels()
        dy = dy.contiguous()
        B, C = x.shape[:2]
        G, hw, nseg = ctx.groups, ctx.hw, ctx.nseg
        dc = _lib.dt_code(x.dtype)
        part = torch.empty(B * C * nseg * 2, device=x.device, dtype=torch.float32)
        k.gn_bwd_reduce(dc, x.data_ptr(), dy.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                        _lib.ptr(w), _lib.ptr(b), _lib.ptr(s), _lib.ptr(sh), part.data_ptr(), B, C,
                        G, hw, nseg, int(ctx.silu), _lib.stream())
        ab = part.view(B, C, nseg, 2).sum(2)
        A, Bz = ab[..., 0], ab[..., 1]  # [B, C]
        s1 = (s.view(B, C) + 1.0) if s is not None else torch.ones_like(A)
        gam = w.view(1, C) if w is not None else torch.ones(1, C, device=x.device)
        kk = gam * s1
        n = float(C // G) * hw
        g1 = ((kk * Bz).view(B, G, C // G).sum(-1) / n).contiguous()
        g2 = ((kk * A).view(B, G, C // G).sum(-1) / n).contiguous()
        dx = torch.empty_like(x)
        k.gn_bwd_apply(dc, x.data_ptr(), dy.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                       _lib.ptr(w), _lib.ptr(b), _lib.ptr(s), _lib.ptr(sh), g1.data_ptr(),
                       g2.data_ptr(), dx.data_ptr(), B, C, G, hw, nseg, int(ctx.silu),
                       _lib.stream())
        _lib.maybe_sync()
        hw_, hb, hs, hsh = ctx.has
        dtw, dtb, dts, dtsh = ctx.dtypes
        dw = (s1 * A).sum(0).to(dtw) if hw_ else None
        db = (s1 * Bz).sum(0).to(dtb) if hb else None
        dscale = None
        if hs:
            bet = b.view(1, C) if b is not None else 0.0
            dscale = (gam * A + bet * Bz).to(dts)
        dshift = Bz.to(dtsh) if hsh else None
        return dx, dw, db, dscale, dshift, None, None, None


def group_norm_silu(x, groups, weight=None, bias=None, scale=None, shift=None, eps=1e-5,
                    silu=True):
    """x: [B, C, *spatial]; scale/shift: [B, C] (FiLM, applied as ``*(1+scale)+shift``)."""
    if not x.is_cuda:
        return group_norm_silu_reference(x, groups, weight, bias, scale, shift, eps, silu)
    if scale is not None:
        scale = scale.reshape(x.shape[0], x.shape[1])
    if shift is not None:
        shift = shift.reshape(x.shape[0], x.shape[1])
    return _GroupNormSiLU.apply(x, weight, bias, scale, shift, int(groups), float(eps), bool(silu))


class GroupNormSiLU(nn.Module):
    def __init__(self, groups, channels, eps=1e-5, silu=True):
        super().__init__()
        self.groups, self.eps, self.silu = groups, eps, silu
        self.weight = nn.Parameter(torch.ones(channels))
        self.bias = nn.Parameter(torch.zeros(channels))

    def forward(self, x, scale=None, shift=None):
        return group_norm_silu(x, self.groups, self.weight, self.bias, scale, shift, self.eps,
                               self.silu)

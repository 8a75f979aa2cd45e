"""Fused scaled (masked) softmax over materialised attention scores.

API parity with the Paddle incubate ops the reference reaches (K04 / N-3):

* ``softmax_mask_fuse_upper_triangle(x)`` -- causal softmax, training path of
  ``core_attn`` (``single_model.py:198``, ``hybrid_model.py:277``,
  ``auto_model.py:190``);
* ``softmax_mask_fuse(x, mask)`` -- additive mask + softmax, the eval path
  (``single_model.py:194-196``).

``x`` is ``[..., Sq, Sk]`` (typically ``[b, heads, s, s]``).  On GPU both
directions run the HIP kernels in ``csrc/kernels/softmax.hip`` (one wave64
per row, register-resident rows up to 4096 columns, fp32 statistics,
masked-out causal columns never read); the backward reads only ``y`` and
``dy``.  CPU tensors use the PyTorch math below (the test oracle).
"""
import torch

from . import _lib

_DT = {torch.bfloat16: 0, torch.float16: 1, torch.float32: 2}


def softmax_reference(x, mask=None, causal=False, scale=1.0):
    """fp32 PyTorch math; fully masked rows give zeros."""
    s = x.float() * scale
    if mask is not None:
        s = s + mask.float()
    if causal:
        Sq, Sk = s.shape[-2:]
        tri = torch.triu(torch.ones(Sq, Sk, dtype=torch.bool, device=x.device), diagonal=1)
        s = s.masked_fill(tri, float("-inf"))
    return torch.nan_to_num(torch.softmax(s, dim=-1), nan=0.0).to(x.dtype)


def _mask_div(x, mask):
    """Rows of ``x`` per mask row-block.  The mask may vary along leading
    axes and broadcast along the trailing ones (e.g. ``[B,1,Sq,Sk]`` or
    ``[1,1,Sq,Sk]`` against ``[B,H,Sq,Sk]``), so one divisor maps a score row
    to its mask row."""
    lead_x = tuple(x.shape[:-2])
    lead_m = (1,) * (len(lead_x) - (mask.dim() - 2)) + tuple(mask.shape[:-2])
    seen_bcast = False
    for dx_, dm in zip(lead_x, lead_m):
        if dm == 1 and dx_ != 1:
            seen_bcast = True
        elif dm != dx_ or seen_bcast:
            raise ValueError("mask shape {} does not broadcast by leading blocks to {}".format(
                tuple(mask.shape), tuple(x.shape)))
    nx = 1
    for d in lead_x:
        nx *= d
    nm = 1
    for d in lead_m:
        nm *= d
    return nx // nm


class _FusedSoftmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mask, causal, scale):
        Sq, Sk = x.shape[-2:]
        if x.dtype not in _DT:
            raise NotImplementedError("fused softmax takes bf16/fp16/fp32 (got %s)" % x.dtype)
        xc = x.contiguous()
        y = torch.empty_like(xc)
        rows = xc.numel() // Sk
        div = 1
        mptr, mdt = 0, 0
        if mask is not None:
            if tuple(mask.shape[-2:]) != (Sq, Sk):
                raise ValueError("mask must end in [Sq, Sk] = [%d, %d]" % (Sq, Sk))
            div = _mask_div(x, mask)
            if mask.dtype not in _DT:
                mask = mask.float()
            mask = mask.contiguous()
            mptr, mdt = mask.data_ptr(), _DT[mask.dtype]
        rc = _lib.kernels().softmax_fwd(_DT[x.dtype], mdt, xc.data_ptr(), mptr, y.data_ptr(), rows,
                                        Sq, Sk, div, float(scale), int(causal), _lib.stream())
        if rc != 0:
            raise RuntimeError("softmax_fwd: bad arguments")
        _lib.maybe_sync()
        ctx.save_for_backward(y)
        ctx.causal, ctx.scale = causal, scale
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        Sq, Sk = y.shape[-2:]
        dy = dy.contiguous().to(y.dtype)
        dx = torch.empty_like(y)
        rc = _lib.kernels().softmax_bwd(_DT[y.dtype], y.data_ptr(), dy.data_ptr(), dx.data_ptr(),
                                        y.numel() // Sk, Sq, Sk, float(ctx.scale), int(ctx.causal),
                                        _lib.stream())
        if rc != 0:
            raise RuntimeError("softmax_bwd: bad arguments")
        _lib.maybe_sync()
        return dx, None, None, None


def fused_softmax(x, mask=None, causal=False, scale=1.0):
    """softmax(scale * x + mask) over the last axis, optionally causal."""
    if not x.is_cuda:
        return softmax_reference(x, mask, causal, scale)
    return _FusedSoftmax.apply(x, mask, bool(causal), float(scale))


def softmax_mask_fuse_upper_triangle(x, scale=1.0):
    """Causal softmax (entries above the diagonal are masked out)."""
    return fused_softmax(x, None, True, scale)


def softmax_mask_fuse(x, mask, scale=1.0):
    """softmax(x + mask) with a broadcastable additive mask ``[b|1, 1|h, Sq, Sk]``."""
    return fused_softmax(x, mask, False, scale)


__all__ = ["fused_softmax", "softmax_mask_fuse", "softmax_mask_fuse_upper_triangle",
           "softmax_reference"]

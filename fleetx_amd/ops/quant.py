"""Symmetric abs-max fake quantisation with a straight-through estimator.

Reference P11 / K23: paddleslim QAT with ``abs_max`` weight quantisation and
``moving_average_abs_max`` activation quantisation at 8 bits
(``pretrain_gpt_345M_mp8_qat.yaml:35-44``).
"""
import torch

from . import _lib


def absmax(x):
    if x.is_cuda:
        out = torch.zeros(1, device=x.device, dtype=torch.float32)
        _lib.kernels().absmax(_lib.dt_code(x.dtype), x.contiguous().data_ptr(), x.numel(),
                              out.data_ptr(), _lib.stream())
        return out
    return x.detach().abs().max().float().reshape(1)


class _FakeQuant(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, scale, bits):
        if x.is_cuda:
            xc = x.contiguous()
            y = torch.empty_like(xc)
            _lib.kernels().fake_quant_fwd(_lib.dt_code(x.dtype), xc.data_ptr(), y.data_ptr(),
                                          scale.data_ptr(), int(bits), x.numel(), _lib.stream())
            return y
        qmax = float(2 ** (bits - 1) - 1)
        s = scale.clamp_min(1e-8)
        return (torch.clamp(torch.round(x.float() / s * qmax), -qmax, qmax) * s / qmax).to(x.dtype)

    @staticmethod
    def backward(ctx, dy):
        return dy, None, None


def fake_quant(x, scale, bits=8):
    """Quantise-dequantise ``x`` with the per-tensor ``scale`` (device scalar)."""
    return _FakeQuant.apply(x, scale.float().reshape(1), bits)

"""Quantization-aware training (int8 fake quant with straight-through grads).

Parity: reference P11 (``paddleslim.dygraph.quant.QAT(config).quantize(model)``
at ``language_module.py:97-100,142-144`` and ``multimodal_module.py:86-89``;
config keys of ``pretrain_gpt_345M_mp8_qat.yaml:35-44``):

* ``weight_quantize_type``: ``abs_max`` (per-tensor scale = max|W| each step)
  or ``channel_wise_abs_max`` (one scale per output channel);
* ``activation_quantize_type``: ``moving_average_abs_max`` (EMA of max|x|,
  rate 0.9) or ``abs_max``;
* ``weight_bits`` / ``activation_bits``;
* ``quantizable_layer_type``: ``Linear``, ``ColumnParallelLinear``,
  ``RowParallelLinear``, ``Conv2D``, ``Conv2DTranspose`` (the reference YAML's
  full list; convolutions are the Imagen UNet's).

The per-tensor quantise-dequantise runs in the HIP ``fake_quant`` kernel
(K23) with a HIP abs-max reduction, and the moving-average update stays on the
device (no host sync per step).  Channel-wise weight scales are a weight-sized
elementwise op done with device tensor math.
"""
import torch
import torch.nn as nn

from .. import ops
from ..ops import quant as Q
from ..parallel import layers as PL


class _QuantState(nn.Module):
    def __init__(self, kind, bits, moving_rate=0.9):
        super().__init__()
        self.kind, self.bits, self.rate = kind, bits, moving_rate
        self.register_buffer("scale", torch.zeros(1))
        self.register_buffer("initialized", torch.zeros(1))

    def forward(self, x):
        cur = Q.absmax(x.detach()).to(self.scale.device)
        if self.kind == "abs_max" or not self.training:
            s = cur if self.kind == "abs_max" else torch.where(self.initialized > 0, self.scale, cur)
        else:
            s = torch.where(self.initialized > 0, self.rate * self.scale + (1 - self.rate) * cur, cur)
        if self.training or self.kind == "abs_max":
            with torch.no_grad():
                self.scale.copy_(s)
                self.initialized.fill_(1)
        return ops.fake_quant(x, s, self.bits)


class _ChannelFakeQuant(torch.autograd.Function):
    @staticmethod
    def forward(ctx, w, scale, bits):
        qmax = float(2 ** (bits - 1) - 1)
        s = scale.clamp_min(1e-8)
        return (torch.clamp(torch.round(w.float() / s * qmax), -qmax, qmax) * s / qmax).to(w.dtype)

    @staticmethod
    def backward(ctx, dy):
        return dy, None, None


class _ChannelQuantState(nn.Module):
    """``channel_wise_abs_max``: one scale per output channel (``axis``)."""

    def __init__(self, bits, axis=0):
        super().__init__()
        self.bits, self.axis = bits, axis
        self.register_buffer("scale", torch.zeros(1))

    def forward(self, w):
        dims = [d for d in range(w.dim()) if d != self.axis]
        s = w.detach().abs().amax(dim=dims, keepdim=True).float()
        with torch.no_grad():
            if self.scale.shape != s.reshape(-1).shape:
                self.scale = torch.zeros_like(s.reshape(-1))
            self.scale.copy_(s.reshape(-1))
        return _ChannelFakeQuant.apply(w, s, self.bits)


def _out_axis(inner):
    # ConvTranspose weights are [in, out / groups, kh, kw]
    return 1 if isinstance(inner, nn.ConvTranspose2d) else 0


class QuantizedLayer(nn.Module):
    """Wraps a Linear / parallel linear / Conv2D / Conv2DTranspose module:
    fake-quantises its input activation and its weight, then runs the wrapped
    layer unchanged (tensor-parallel communication included)."""

    def __init__(self, inner, weight_bits=8, activation_bits=8, weight_type="abs_max",
                 act_type="moving_average_abs_max"):
        super().__init__()
        self.inner = inner
        if weight_type == "channel_wise_abs_max":
            self.wq = _ChannelQuantState(weight_bits, _out_axis(inner))
        else:
            self.wq = _QuantState(weight_type, weight_bits)
        self.aq = _QuantState(act_type, activation_bits)

    def forward(self, x, *args, **kwargs):
        w = self.inner.weight
        wq = self.wq(w)
        xq = self.aq(x)
        orig = self.inner.weight
        self.inner._parameters["weight"] = wq
        try:
            return self.inner(xq, *args, **kwargs)
        finally:
            self.inner._parameters["weight"] = orig


QuantizedLinear = QuantizedLayer  # round-1 name

_TYPES = {"Linear": (nn.Linear,), "ColumnParallelLinear": (PL.ColumnParallelLinear,),
          "RowParallelLinear": (PL.RowParallelLinear,), "Conv2D": (nn.Conv2d,),
          "Conv2DTranspose": (nn.ConvTranspose2d,)}


def _quantizable(module, types):
    for t in types:
        if t not in _TYPES:
            raise ValueError("unsupported quantizable_layer_type {!r} (supported: {})".format(
                t, sorted(_TYPES)))
        if isinstance(module, _TYPES[t]):
            return True
    return False


def quantize_model(model, qcfg):
    types = list(qcfg.get("quantizable_layer_type",
                          ["Linear", "ColumnParallelLinear", "RowParallelLinear"]))
    wb, ab = int(qcfg.get("weight_bits", 8)), int(qcfg.get("activation_bits", 8))
    wt = qcfg.get("weight_quantize_type", "abs_max")
    at = qcfg.get("activation_quantize_type", "moving_average_abs_max")
    if wt not in ("abs_max", "channel_wise_abs_max"):
        raise ValueError("weight_quantize_type {!r} not supported".format(wt))
    if at not in ("abs_max", "moving_average_abs_max"):
        raise ValueError("activation_quantize_type {!r} not supported".format(at))

    def _swap(parent):
        for name, child in list(parent.named_children()):
            if isinstance(child, QuantizedLayer):
                continue
            if _quantizable(child, types):
                setattr(parent, name, QuantizedLayer(child, wb, ab, wt, at))
            else:
                _swap(child)
    _swap(model)
    return model

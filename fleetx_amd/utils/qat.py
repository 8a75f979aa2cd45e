"""Quantization-aware training (int8 fake quant with straight-through grads).

Parity: reference P11 (``paddleslim.dygraph.quant.QAT(config).quantize(model)``
at ``language_module.py:97-100,142-144``; config keys of
``pretrain_gpt_345M_mp8_qat.yaml:35-44``): ``weight_quantize_type:
abs_max`` (per-tensor scale = max|W| each step), ``activation_quantize_type:
moving_average_abs_max`` (EMA of max|x|, rate 0.9), ``weight_bits`` /
``activation_bits``, ``quantizable_layer_type`` (Linear / Column / Row
parallel linears).

The quantise-dequantise runs in the HIP ``fake_quant`` kernel (K23); the
abs-max reduction is a HIP kernel too, and the moving-average update stays on
the device (no host sync per step).
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


class QuantizedLinear(nn.Module):
    """Wraps a linear module: fake-quantises its input activation and weight."""

    def __init__(self, inner, weight_bits=8, activation_bits=8, weight_type="abs_max",
                 act_type="moving_average_abs_max"):
        super().__init__()
        self.inner = inner
        self.wq = _QuantState(weight_type, weight_bits)
        self.aq = _QuantState(act_type, activation_bits)

    def forward(self, x):
        w = self.inner.weight
        wq = self.wq(w)
        xq = self.aq(x)
        orig = self.inner.weight
        # run the wrapped layer (TP comm etc.) with the quantised weight
        self.inner._parameters["weight"] = wq
        try:
            return self.inner(xq)
        finally:
            self.inner._parameters["weight"] = orig


def _quantizable(module, types):
    names = {"Linear": nn.Linear, "ColumnParallelLinear": PL.ColumnParallelLinear,
             "RowParallelLinear": PL.RowParallelLinear}
    return any(isinstance(module, names[t]) for t in types if t in names)


def quantize_model(model, qcfg):
    types = list(qcfg.get("quantizable_layer_type",
                          ["Linear", "ColumnParallelLinear", "RowParallelLinear"]))
    wb, ab = int(qcfg.get("weight_bits", 8)), int(qcfg.get("activation_bits", 8))
    wt = qcfg.get("weight_quantize_type", "abs_max")
    at = qcfg.get("activation_quantize_type", "moving_average_abs_max")

    def _swap(parent):
        for name, child in list(parent.named_children()):
            if _quantizable(child, types):
                setattr(parent, name, QuantizedLinear(child, wb, ab, wt, at))
            else:
                _swap(child)
    _swap(model)
    return model

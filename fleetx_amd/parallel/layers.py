"""Tensor-parallel (Megatron 1-D) and sequence-parallel layers.

Parity: Fleet ``ColumnParallelLinear`` / ``RowParallelLinear`` /
``VocabParallelEmbedding`` / ``ParallelCrossEntropy`` (reference
``hybrid_model.py:111-163,497-511,590-594,799``) and the sequence-parallel
``Column/RowSequenceParallelLinear`` (``sequence_parallel_utils.py:150-326``).

MI355X notes:
* weights are stored ``[out, in]`` so ``F.linear`` maps straight onto a
  hipBLASLt TN GEMM; no transposed copies;
* ``skip_bias_add`` returns the bias so the caller fuses it into the next
  HIP epilogue (bias+GeLU, bias+dropout+residual) instead of a separate
  broadcast-add kernel;
* parameters are initialised as the FULL matrix from a per-parameter seed and
  then sliced, so every (dp, mp, pp) layout starts from bit-identical weights
  (this is what the layout-equivalence tests rely on);
* parameters replicated across the mp group under sequence parallelism are
  tagged ``sequence_parallel = True``; the gradient synchroniser all-reduces
  them in ONE coalesced mp bucket (N09) instead of per-tensor hooks.
"""
import hashlib
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import mappings as M
from . import topology as topo
from .. import ops
from .linear import linear, column_tp_linear, row_tp_linear
from .sp_overlap import column_sp_linear, row_sp_linear


# Tensor-parallel comm/compute overlap switches (Distributed.comm.tp_overlap*)
TP_OVERLAP = {"enabled": True, "row_chunks": 2}


def _param_seed(base_seed, name):
    h = hashlib.sha256("{}:{}".format(base_seed, name).encode()).hexdigest()
    return int(h[:15], 16)


_INIT_STATE = {"seed": 1234, "device": None}


def set_init_seed(seed, device=None):
    _INIT_STATE["seed"] = seed
    _INIT_STATE["device"] = device


def init_full_then_slice(shape, std, name, dim=None, mean=0.0, dtype=None, device=None,
                         init="normal"):
    """Initialise the full tensor deterministically, return this mp rank's slice."""
    device = device if device is not None else _INIT_STATE["device"]
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
            else torch.device("cpu")
    g = torch.Generator(device=device)
    g.manual_seed(_param_seed(_INIT_STATE["seed"], name))
    full = torch.empty(shape, dtype=torch.float32, device=device)
    if init == "normal":
        full.normal_(mean, std, generator=g)
    elif init == "xavier":
        fan_out, fan_in = shape[0], shape[1] if len(shape) > 1 else shape[0]
        a = math.sqrt(6.0 / (fan_in + fan_out))
        full.uniform_(-a, a, generator=g)
    elif init == "zeros":
        full.zero_()
    elif init == "ones":
        full.fill_(1.0)
    else:
        raise ValueError(init)
    if dim is not None:
        n, r = topo.mp_world_size(), topo.mp_rank()
        if n > 1:
            full = full.chunk(n, dim=dim)[r]
    return full.contiguous().to(dtype or torch.float32)


class ColumnParallelLinear(nn.Module):
    """y = x W^T (+ b); W: [out/t, in].  Input replicated (or seq-sharded under SP)."""

    def __init__(self, in_features, out_features, bias=True, gather_output=False,
                 skip_bias_add=False, sequence_parallel=False, std=0.02, name="col",
                 dtype=None, device=None):
        super().__init__()
        t = topo.mp_world_size()
        assert out_features % t == 0, "out_features {} not divisible by mp {}".format(out_features, t)
        self.in_features, self.out_features = in_features, out_features
        self.out_per_rank = out_features // t
        self.gather_output = gather_output
        self.skip_bias_add = skip_bias_add
        self.sequence_parallel = sequence_parallel and t > 1
        self.weight = nn.Parameter(init_full_then_slice((out_features, in_features), std,
                                                        name + ".weight", dim=0, dtype=dtype,
                                                        device=device))
        self.weight.tp_split = t > 1
        self.weight.tp_dim = 0
        self.weight._fx_fused_wgrad_ok = True
        self.weight._fx_gemm_wgrad = True  # gradient from the wgrad GEMM (fused-norm partials)
        # the SP-overlapped backward writes the gradient in sequence chunks
        # (several GEMM writes): never 16-bit storage (grad16_eligible)
        self.weight._fx_grad_chunked = self.sequence_parallel
        if bias:
            self.bias = nn.Parameter(init_full_then_slice((out_features,), 0.0, name + ".bias",
                                                          dim=0, dtype=dtype, device=device,
                                                          init="zeros"))
            self.bias.tp_split = t > 1
            self.bias.tp_dim = 0
            # a bias applied inside linear() gets its fp32 grad from the wgrad pass
            self.bias._fx_fused_wgrad_ok = not skip_bias_add
        else:
            self.register_parameter("bias", None)

    def forward(self, x):
        b = None if self.skip_bias_add else self.bias
        if self.sequence_parallel:
            if TP_OVERLAP["enabled"] and x.dim() == 3:
                y = column_sp_linear(x, self.weight, b, topo.mp_group(),
                                     chunk_major=getattr(self, "sp_chunk_major", False))
            else:
                x = M.all_gather_seq(x)
                y = linear(x, self.weight, b)
        elif topo.mp_world_size() > 1 and TP_OVERLAP["enabled"]:
            y = column_tp_linear(x, self.weight, b, topo.mp_group())
        else:
            x = M.copy_to_mp(x)
            y = linear(x, self.weight, b)
        if self.gather_output:
            y = M.gather_from_mp(y)
        if self.skip_bias_add:
            return y, self.bias
        return y


class RowParallelLinear(nn.Module):
    """y = x W^T + b; W: [out, in/t].  Output all-reduced (reduce-scattered under SP)."""

    def __init__(self, in_features, out_features, bias=True, input_is_parallel=True,
                 skip_bias_add=False, sequence_parallel=False, std=0.02, name="row",
                 dtype=None, device=None):
        super().__init__()
        t = topo.mp_world_size()
        assert in_features % t == 0
        self.in_features, self.out_features = in_features, out_features
        self.input_is_parallel = input_is_parallel
        self.skip_bias_add = skip_bias_add
        self.sequence_parallel = sequence_parallel and t > 1
        self.weight = nn.Parameter(init_full_then_slice((out_features, in_features), std,
                                                        name + ".weight", dim=1, dtype=dtype,
                                                        device=device))
        self.weight.tp_split = t > 1
        self.weight.tp_dim = 1
        self.weight._fx_fused_wgrad_ok = True
        self.weight._fx_gemm_wgrad = True  # gradient from the wgrad GEMM (fused-norm partials)
        self.weight._fx_grad_chunked = self.sequence_parallel  # (as the column layer)
        if bias:
            self.bias = nn.Parameter(init_full_then_slice((out_features,), 0.0, name + ".bias",
                                                          dtype=dtype, device=device,
                                                          init="zeros"))
            self.bias.sequence_parallel = self.sequence_parallel
            # with skip_bias_add its gradient is reduced by the fused residual
            # kernels straight into main_grad
            self.bias._fx_fused_wgrad_ok = skip_bias_add
        else:
            self.register_parameter("bias", None)

    def forward(self, x):
        if not self.input_is_parallel:
            x = M.scatter_to_mp(x)
        if self.sequence_parallel:
            # chunk-major input exactly when the paired column-SP linear took
            # its overlapped path (same TP_OVERLAP / rank-3 conditions)
            overlap = TP_OVERLAP["enabled"] and x.dim() == 3
            cm = overlap and getattr(self, "sp_chunk_major", False)
            if overlap and x.shape[0] % topo.mp_world_size() == 0:
                y = row_sp_linear(x, self.weight, topo.mp_group(), chunk_major=cm)
            else:
                assert not cm, "a chunk-major input needs the overlapped row-SP path"
                y = M.reduce_scatter_seq(linear(x, self.weight))
        elif topo.mp_world_size() > 1 and TP_OVERLAP["enabled"]:
            y = row_tp_linear(x, self.weight, topo.mp_group(), TP_OVERLAP["row_chunks"])
        else:
            y = M.reduce_from_mp(linear(x, self.weight))
        if self.skip_bias_add:
            return y, self.bias
        return y + self.bias if self.bias is not None else y


class VocabParallelEmbedding(nn.Module):
    """Rows [V/t * r, V/t * (r+1)) live on mp rank r; other ids give zero rows."""

    def __init__(self, vocab_size, hidden, std=0.02, name="word_embeddings", dtype=None,
                 device=None):
        super().__init__()
        t, r = topo.mp_world_size(), topo.mp_rank()
        assert vocab_size % t == 0, "vocab {} not divisible by mp {}".format(vocab_size, t)
        self.vocab_size = vocab_size
        self.per_rank = vocab_size // t
        self.vocab_start = r * self.per_rank
        self.weight = nn.Parameter(init_full_then_slice((vocab_size, hidden), std, name + ".weight",
                                                        dim=0, dtype=dtype, device=device))
        self.weight.tp_split = t > 1
        self.weight.tp_dim = 0

    def forward(self, ids, pos_ids=None, pos_weight=None, reduce=True):
        out = ops.embedding(ids, self.weight, pos_ids, pos_weight, self.vocab_start)
        return out


def parallel_lm_logits(h, weight, parallel_output=True, sequence_parallel=False):
    """logits = h W_emb^T on the local vocab shard (reference ``parallel_matmul``,
    ``hybrid_model.py:45-66``)."""
    if sequence_parallel:
        h = M.all_gather_seq(h)
    else:
        h = M.copy_to_mp(h)
    logits = linear(h, weight)  # fused fp32 wgrad into the tied weight's main_grad
    if not parallel_output:
        logits = M.gather_from_mp(logits)
    return logits


class HeadInput:
    """What the GPT model hands its criterion when the LM head and the
    cross-entropy run fused and chunked (``ops/lm_head_ce.py``): the hidden
    states after the mp copy / sequence gather as ``[tokens, h]`` (token
    order = the logits' row order), and the tied vocab-shard weight."""
    __slots__ = ("h2", "weight")

    def __init__(self, h2, weight):
        self.h2, self.weight = h2, weight


def parallel_lm_head_input(h, weight, sequence_parallel=False):
    """The input half of :func:`parallel_lm_logits`: ``h`` prepared exactly as
    for the head GEMM, which the criterion then runs chunk by chunk."""
    if sequence_parallel:
        h = M.all_gather_seq(h)
    else:
        h = M.copy_to_mp(h)
    return HeadInput(h.reshape(-1, h.shape[-1]), weight)


def mark_sequence_parallel(module):
    """Tag replicated params (LN, row-bias) whose grads need an mp all-reduce."""
    for p in module.parameters():
        p.sequence_parallel = True

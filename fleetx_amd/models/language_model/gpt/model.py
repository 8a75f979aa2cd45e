"""GPT-2/3 decoder (pre-LN) for single-device, tensor/sequence-parallel and
pipeline-stage execution -- one implementation.

Parity: reference ``gpt/dygraph/single_model.py:43-653`` (C26) and
``hybrid_model.py:45-832`` (C28): word + learned position embeddings with
dropout; per layer LN1 -> fused QKV -> causal attention (+ prob dropout) ->
out-proj -> dropout + residual -> LN2 -> FFN (tanh-GeLU) -> dropout +
residual; final LN; LM head tied to the word embedding; loss
``sum(ce * mask) / sum(mask)``.  Recompute granularities ``full`` /
``full_attn`` / ``core_attn``.

MI355X mapping:
* QKV / out-proj / FFN / LM-head GEMMs: the hand-written MFMA GEMM
  (``ops.gemm``) in native layouts; FC1 bias+GeLU and FC2's dgrad*gelu' are
  fused into GEMM epilogues (``parallel.linear.fused_mlp``), the QKV bias too;
* bias+dropout+residual, residual+LN2: HIP epilogue kernels;
* attention: the fused flash kernel reading the packed ``[.., heads, 3, d]``
  QKV output in place;
* embedding gather and vocab-parallel CE: HIP kernels; logits gradient is
  written over the logits buffer.
Activations use ``[b, s, h]``, or ``[s, b, h]`` under sequence parallelism
(so the sequence shard is the leading dim, as in the reference).
"""
import math

import torch
import torch.nn as nn

from .... import ops
from ....parallel import layers as L
from ....parallel import mappings as M
from ....parallel import topology as topo
from ....parallel.linear import fused_mlp
from ....parallel.recompute import recompute
from ....parallel.rng import get_rng_state_tracker


class GPTConfig:
    def __init__(self, vocab_size=50304, hidden_size=1024, num_layers=24, num_attention_heads=16,
                 ffn_hidden_size=None, hidden_dropout_prob=0.1, attention_probs_dropout_prob=0.1,
                 max_position_embeddings=1024, type_vocab_size=16, initializer_range=0.02,
                 use_recompute=False, recompute_granularity=None, sequence_parallel=False,
                 layer_norm_eps=1e-5, fused_linear=False, no_recompute_layers=None,
                 fused_lm_head_ce=False, dtype=torch.float32, **unused):
        self.vocab_size = vocab_size
        self.hidden_size = hidden_size
        self.num_layers = num_layers
        self.num_attention_heads = num_attention_heads
        self.ffn_hidden_size = ffn_hidden_size or 4 * hidden_size
        self.hidden_dropout_prob = hidden_dropout_prob
        self.attention_probs_dropout_prob = attention_probs_dropout_prob
        self.max_position_embeddings = max_position_embeddings
        self.type_vocab_size = type_vocab_size
        self.initializer_range = initializer_range
        self.use_recompute = use_recompute
        self.recompute_granularity = recompute_granularity or ("full" if use_recompute else None)
        self.sequence_parallel = sequence_parallel and topo.mp_world_size() > 1
        self.layer_norm_eps = layer_norm_eps
        self.no_recompute_layers = set(no_recompute_layers or [])
        self.dtype = dtype
        self.head_dim = hidden_size // num_attention_heads
        # training: LM head + CE chunked over tokens, logits never whole (ops/lm_head_ce.py)
        self.fused_lm_head_ce = bool(fused_lm_head_ce)

    @classmethod
    def from_model_config(cls, cfg, dtype=torch.float32):
        keys = ["vocab_size", "hidden_size", "num_layers", "num_attention_heads", "ffn_hidden_size",
                "hidden_dropout_prob", "attention_probs_dropout_prob", "max_position_embeddings",
                "type_vocab_size", "initializer_range", "use_recompute", "recompute_granularity",
                "sequence_parallel", "no_recompute_layers", "layer_norm_eps", "fused_lm_head_ce"]
        kw = {k: cfg[k] for k in keys if k in cfg and cfg[k] is not None}
        return cls(dtype=dtype, **kw)


def _key(stream):
    return get_rng_state_tracker().next_key(stream)


class GPTEmbeddings(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self.word_embeddings = L.VocabParallelEmbedding(cfg.vocab_size, cfg.hidden_size,
                                                        std=cfg.initializer_range,
                                                        name="embeddings.word", dtype=cfg.dtype)
        self.position_embeddings = nn.Parameter(L.init_full_then_slice(
            (cfg.max_position_embeddings, cfg.hidden_size), cfg.initializer_range,
            "embeddings.position", dtype=cfg.dtype))
        # under SP each mp rank only sees its sequence slice -> grads need an mp all-reduce
        self.position_embeddings.sequence_parallel = cfg.sequence_parallel

    def forward(self, input_ids, position_ids=None):
        b, s = input_ids.shape
        if position_ids is None:
            position_ids = torch.arange(s, device=input_ids.device).unsqueeze(0).expand(b, s)
        sp = self.cfg.sequence_parallel
        if sp:  # [s, b] order so the sequence shard is the leading dim
            input_ids = input_ids.t()
            position_ids = position_ids.t()
        if topo.mp_world_size() == 1:
            x = ops.embedding(input_ids, self.word_embeddings.weight, position_ids,
                              self.position_embeddings, 0)
        else:
            x = self.word_embeddings(input_ids)
            if sp:
                x = M.reduce_scatter_seq(x)
                pos = ops.embedding(M._split(position_ids, topo.mp_group(), 0),
                                    self.position_embeddings)
            else:
                x = M.reduce_from_mp(x)
                pos = ops.embedding(position_ids, self.position_embeddings)
            x = x + pos
        p = self.cfg.hidden_dropout_prob if self.training else 0.0
        if p > 0:
            x = ops.dropout(x, p, _key("local_seed" if sp else "global_seed"))
        return x


class GPTAttention(nn.Module):
    def __init__(self, cfg, idx):
        super().__init__()
        self.cfg = cfg
        t = topo.mp_world_size()
        assert cfg.num_attention_heads % t == 0
        self.heads = cfg.num_attention_heads // t
        self.head_dim = cfg.head_dim
        std = cfg.initializer_range
        self.qkv_proj = L.ColumnParallelLinear(cfg.hidden_size, 3 * cfg.hidden_size, bias=True,
                                               sequence_parallel=cfg.sequence_parallel, std=std,
                                               name="layers.%d.attn.qkv" % idx, dtype=cfg.dtype)
        self.out_proj = L.RowParallelLinear(cfg.hidden_size, cfg.hidden_size, bias=True,
                                            skip_bias_add=True,
                                            sequence_parallel=cfg.sequence_parallel, std=std,
                                            name="layers.%d.attn.out" % idx, dtype=cfg.dtype)

    def core_attn(self, qkv, key):
        cfg = self.cfg
        p = cfg.attention_probs_dropout_prob if self.training else 0.0
        if cfg.sequence_parallel:
            s, b = qkv.shape[0], qkv.shape[1]
            qkv5 = qkv.view(s, b, self.heads, 3, self.head_dim).transpose(0, 1)
        else:
            b, s = qkv.shape[0], qkv.shape[1]
            qkv5 = qkv.view(b, s, self.heads, 3, self.head_dim)
        o = ops.flash_attention_qkvpacked(qkv5, causal=True, dropout_p=p, key=key)
        if cfg.sequence_parallel:
            return o.transpose(0, 1).reshape(s, b, self.heads * self.head_dim)
        return o.reshape(b, s, self.heads * self.head_dim)

    def forward(self, x):
        qkv = self.qkv_proj(x)
        key = _key("local_seed") if (self.training and self.cfg.attention_probs_dropout_prob > 0) else 0
        if self.cfg.recompute_granularity == "core_attn" and self.training:
            o = recompute(self.core_attn, qkv, key)
        else:
            o = self.core_attn(qkv, key)
        return self.out_proj(o)


class GPTMLP(nn.Module):
    def __init__(self, cfg, idx):
        super().__init__()
        std = cfg.initializer_range
        self.fc1 = L.ColumnParallelLinear(cfg.hidden_size, cfg.ffn_hidden_size, bias=True,
                                          skip_bias_add=True,
                                          sequence_parallel=cfg.sequence_parallel, std=std,
                                          name="layers.%d.mlp.fc1" % idx, dtype=cfg.dtype)
        self.fc2 = L.RowParallelLinear(cfg.ffn_hidden_size, cfg.hidden_size, bias=True,
                                       skip_bias_add=True, sequence_parallel=cfg.sequence_parallel,
                                       std=std, name="layers.%d.mlp.fc2" % idx, dtype=cfg.dtype)
        # FC1 -> bias+GeLU -> FC2 is row-wise in between: under overlapped
        # SP the intermediate stays in chunk-major row order (one GEMM per
        # chunk instead of one per rank per chunk; parallel/sp_overlap.py)
        self.fc1.sp_chunk_major = self.fc2.sp_chunk_major = bool(cfg.sequence_parallel)

    def forward(self, x):
        if topo.mp_world_size() == 1 and type(self.fc1) is L.ColumnParallelLinear \
                and type(self.fc2) is L.RowParallelLinear:
            # one autograd node: FC1 GEMM+bias+GeLU epilogue, FC2 GEMM; backward
            # fuses gelu' into FC2's data-gradient GEMM (parallel/linear.py)
            return fused_mlp(x, self.fc1.weight, self.fc1.bias, self.fc2.weight), self.fc2.bias
        y, b = self.fc1(x)
        y = ops.bias_gelu(y, b, approximate=True)
        return self.fc2(y)


class GPTDecoderLayer(nn.Module):
    """x -> x + drop(attn(LN1 x)) -> (+) drop(mlp(LN2 .))   (pre-LN)."""

    def __init__(self, cfg, idx):
        super().__init__()
        self.cfg = cfg
        self.idx = idx
        self.ln1 = ops.FusedLayerNorm(cfg.hidden_size, cfg.layer_norm_eps, dtype=cfg.dtype)
        self.attn = GPTAttention(cfg, idx)
        self.ln2 = ops.FusedLayerNorm(cfg.hidden_size, cfg.layer_norm_eps, dtype=cfg.dtype)
        self.mlp = GPTMLP(cfg, idx)
        if cfg.sequence_parallel:
            L.mark_sequence_parallel(self.ln1)
            L.mark_sequence_parallel(self.ln2)

    def _attn_block(self, x):
        return self.attn(self.ln1(x))

    def _attn_block_out(self, x):
        return self._attn_block(x)[0]

    def _forward(self, x):
        cfg = self.cfg
        p = cfg.hidden_dropout_prob if self.training else 0.0
        stream = "local_seed" if cfg.sequence_parallel else "global_seed"
        if cfg.recompute_granularity == "full_attn" and self.training:
            # the out-proj bias is a leaf: pass it around the checkpoint, not through it
            a, ab = recompute(self._attn_block_out, x), self.attn.out_proj.bias
        else:
            # LN1 hands back x as the residual alias: the residual branch's
            # gradient joins the LN1 backward kernel (no separate add pass)
            x, h1 = ops.layer_norm_keep_input(x, self.ln1.weight, self.ln1.bias, self.ln1.eps)
            a, ab = self.attn(h1)
        k1 = _key(stream) if p > 0 else 0
        x2, h2 = ops.add_layer_norm(a, ab, x, self.ln2.weight, self.ln2.bias, self.ln2.eps, p, k1)
        m, mb = self.mlp(h2)
        k2 = _key(stream) if p > 0 else 0
        return ops.bias_dropout_add(m, mb, x2, p, k2)

    def forward(self, x):
        if (self.cfg.recompute_granularity == "full" and self.training
                and self.idx not in self.cfg.no_recompute_layers):
            return recompute(self._forward, x)
        return self._forward(x)


class GPTModel(nn.Module):
    """Embeddings (first stage) + decoder layers [start, end) + final LN (last stage)."""

    def __init__(self, cfg, layer_range=None, has_embedding=True, has_final_ln=True):
        super().__init__()
        self.cfg = cfg
        start, end = layer_range if layer_range is not None else (0, cfg.num_layers)
        self.embeddings = GPTEmbeddings(cfg) if has_embedding else None
        self.layers = nn.ModuleList([GPTDecoderLayer(cfg, i) for i in range(start, end)])
        self.final_ln = ops.FusedLayerNorm(cfg.hidden_size, cfg.layer_norm_eps,
                                           dtype=cfg.dtype) if has_final_ln else None
        if has_final_ln and cfg.sequence_parallel:
            L.mark_sequence_parallel(self.final_ln)

    def forward(self, input_ids=None, position_ids=None, hidden=None):
        x = self.embeddings(input_ids, position_ids) if self.embeddings is not None else hidden
        for layer in self.layers:
            x = layer(x)
        if self.final_ln is not None:
            x = self.final_ln(x)
        return x


class GPTForPretraining(nn.Module):
    """Decoder + tied LM head producing vocab-parallel logits."""

    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self.gpt = GPTModel(cfg)
        emb = self.gpt.embeddings
        if emb is not None:
            # the tied word embedding gets two fused fp32 grad contributions per
            # step (lookup backward + LM-head wgrad), both straight into main_grad
            emb.word_embeddings.weight._fx_fused_wgrad_ok = True
            emb.word_embeddings.weight._fx_grad_parts = 2
            emb.position_embeddings._fx_fused_wgrad_ok = True

    def forward(self, input_ids, position_ids=None):
        h = self.gpt(input_ids, position_ids)
        w = self.gpt.embeddings.word_embeddings.weight
        if self.cfg.fused_lm_head_ce and self.training:
            # the criterion runs head + CE chunk by chunk (ops/lm_head_ce.py)
            return L.parallel_lm_head_input(h, w, sequence_parallel=self.cfg.sequence_parallel)
        logits = L.parallel_lm_logits(h, w, parallel_output=True,
                                      sequence_parallel=self.cfg.sequence_parallel)
        return logits  # [b, s, V/t], or [s, b, V/t] under sequence parallelism


class GPTPretrainingCriterion(nn.Module):
    """``sum(ce * loss_mask) / sum(loss_mask)`` with vocab-parallel CE (K11)."""

    def __init__(self, cfg=None):
        super().__init__()
        self.seq_first = bool(cfg is not None and cfg.sequence_parallel)

    def forward(self, logits, labels, loss_mask):
        if self.seq_first:
            labels, loss_mask = labels.t(), loss_mask.t()
        g = topo.get_hcg().get_model_parallel_group()
        if isinstance(logits, L.HeadInput):
            from ....parallel.linear import linear
            from ....ops import lm_head_ce
            hi = logits
            vocab_start = topo.mp_rank() * hi.weight.shape[0]
            if lm_head_ce.supported(hi.h2, hi.weight):
                return lm_head_ce.lm_head_cross_entropy(
                    hi.h2, hi.weight, labels.reshape(-1), loss_mask.reshape(-1),
                    group=g if g.nranks > 1 else None, vocab_start=vocab_start)
            logits = linear(hi.h2, hi.weight)  # no flat grad buffer: the plain head
        vocab_start = topo.mp_rank() * logits.shape[-1]
        ce = ops.softmax_cross_entropy(logits, labels, group=g if g.nranks > 1 else None,
                                       vocab_start=vocab_start)
        mask = loss_mask.reshape(-1).float()
        return (ce.reshape(-1) * mask).sum() / mask.sum()


def num_params(cfg):
    """Reference model-size estimate (``language_module.py:102-105``)."""
    l, h, V, s = cfg.num_layers, cfg.hidden_size, cfg.vocab_size, cfg.max_position_embeddings
    return 12 * l * h * h * (1 + 13.0 / (12 * h) + (V + s) / (12.0 * l * h))


def flops_per_token(cfg, seq_len):
    """Model FLOPs/token (fwd+bwd, no recompute): 72 L h^2 (1 + s/6h + V/12hL)."""
    l, h, V = cfg.num_layers, cfg.hidden_size, cfg.vocab_size
    return 72.0 * l * h * h * (1 + seq_len / (6.0 * h) + V / (12.0 * h * l))

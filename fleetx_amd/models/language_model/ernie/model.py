"""ERNIE / BERT-style post-LN encoder with MLM + sentence-order heads.

Parity: reference ``models/language_model/ernie/single_model.py:37-978``
(C33, K22):

* ``ErnieEmbeddings`` word + position + token-type (+ optional task-type)
  embeddings -> LayerNorm(eps 1e-12) -> dropout.  The reference returns early
  with the word embeddings only (``single_model.py:88``, a defect recorded in
  SURVEY.md §5); the full sum is computed here.
* ``ErnieModel`` = embeddings -> N x post-LN encoder layers (Paddle
  ``TransformerEncoderLayer(normalize_before=False)``:
  ``x = LN1(x + drop(attn(x))); x = LN2(x + drop(fc2(act(fc1(x)))))``) ->
  tanh pooler on token 0.  Default attention mask: additive ``-1e4`` on keys
  whose id is ``pad_token_id`` (``single_model.py:339-346``); a 2-D ``[B, S]``
  0/1 mask becomes ``(1 - m) * -1e4``.
* Heads: ``ErnieLMPredictionHead`` (transform -> act -> LN -> decoder tied to
  the word embeddings + bias, optional ``masked_positions`` gather),
  ``ErniePretrainingHeads`` (+ 2-way seq-relationship), ``ErnieForPretraining``,
  ``ErnieForMaskedLM``, ``ErnieForMultipleChoice``; ``ErniePretrainingCriterion``
  (CE with ``ignore_index=-1``; mean MLM loss, optional NSP loss).

MI355X mapping: QKV is one fused column-parallel GEMM laid out
``[b, s, heads, 3, d]`` and consumed by the non-causal flash kernel with an
additive per-key bias (the padding mask) evaluated inside the kernel; the two
residual-add + dropout + LayerNorm steps of every post-LN layer are each one
``add_layer_norm`` HIP kernel; bias + exact GeLU is one kernel; the MLM head
runs only on the gathered masked positions, and its vocab projection uses the
vocab-parallel cross entropy (no full-vocab softmax tensor).  Linear layers are
the Megatron column/row-parallel ones, so ``mp_degree > 1`` works unchanged.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .... import ops
from ....parallel import layers as L
from ....parallel import mappings as M
from ....parallel import topology as topo
from ....parallel.recompute import recompute
from ....parallel.rng import get_rng_state_tracker

LN_EPS = 1e-12


def _key(p, training):
    return get_rng_state_tracker().next_key("global_seed") if (training and p > 0) else 0


def _act(name):
    name = (name or "gelu").lower()
    if name in ("gelu", "gelu_erf"):
        return lambda y, b: ops.bias_gelu(y, b, approximate=False)
    if name in ("gelu_new", "gelu_tanh", "gelu_approx"):
        return lambda y, b: ops.bias_gelu(y, b, approximate=True)
    if name == "relu":
        return lambda y, b: F.relu(y + b)
    raise ValueError("unsupported hidden_act {}".format(name))


class ErnieEmbeddings(nn.Module):
    def __init__(self, vocab_size, hidden_size=768, hidden_dropout_prob=0.1,
                 max_position_embeddings=512, type_vocab_size=2, pad_token_id=0, std=0.02,
                 task_type_vocab_size=3, task_id=0, use_task_id=False, dtype=None):
        super().__init__()
        self.word_embeddings = L.VocabParallelEmbedding(vocab_size, hidden_size, std=std,
                                                        name="ernie.word", dtype=dtype)
        self.position_embeddings = nn.Parameter(L.init_full_then_slice(
            (max_position_embeddings, hidden_size), std, "ernie.position", dtype=dtype))
        self.type_vocab_size = type_vocab_size
        if type_vocab_size > 0:
            self.token_type_embeddings = nn.Parameter(L.init_full_then_slice(
                (type_vocab_size, hidden_size), std, "ernie.token_type", dtype=dtype))
        self.use_task_id, self.task_id = use_task_id, task_id
        if use_task_id:
            self.task_type_embeddings = nn.Parameter(L.init_full_then_slice(
                (task_type_vocab_size, hidden_size), std, "ernie.task_type", dtype=dtype))
        self.layer_norm = ops.FusedLayerNorm(hidden_size, LN_EPS, dtype=dtype)
        self.p = hidden_dropout_prob

    def forward(self, input_ids, token_type_ids=None, position_ids=None, task_type_ids=None):
        b, s = input_ids.shape
        if position_ids is None:
            position_ids = torch.arange(s, device=input_ids.device).unsqueeze(0).expand(b, s)
        if topo.mp_world_size() == 1:
            x = ops.embedding(input_ids, self.word_embeddings.weight, position_ids,
                              self.position_embeddings, 0)
        else:
            x = M.reduce_from_mp(self.word_embeddings(input_ids))
            x = x + ops.embedding(position_ids, self.position_embeddings)
        extra = None
        if self.type_vocab_size > 0:
            if token_type_ids is None:
                token_type_ids = torch.zeros_like(input_ids)
            extra = ops.embedding(token_type_ids, self.token_type_embeddings)
        if self.use_task_id:
            if task_type_ids is None:
                task_type_ids = torch.full_like(input_ids, self.task_id)
            t = ops.embedding(task_type_ids, self.task_type_embeddings)
            extra = t if extra is None else extra + t
        if extra is not None:
            x = x + extra
        y = self.layer_norm(x)
        p = self.p if self.training else 0.0
        return ops.dropout(y, p, _key(p, True)) if p > 0 else y


class ErnieEncoderLayer(nn.Module):
    def __init__(self, hidden_size, num_heads, intermediate_size, hidden_dropout_prob,
                 attention_probs_dropout_prob, hidden_act, std, idx, dtype=None):
        super().__init__()
        t = topo.mp_world_size()
        assert num_heads % t == 0
        self.heads, self.head_dim = num_heads // t, hidden_size // num_heads
        self.p, self.pa = hidden_dropout_prob, attention_probs_dropout_prob
        nm = "ernie.layers.%d." % idx
        self.qkv = L.ColumnParallelLinear(hidden_size, 3 * hidden_size, std=std, name=nm + "qkv",
                                          dtype=dtype)
        self.out_proj = L.RowParallelLinear(hidden_size, hidden_size, skip_bias_add=True, std=std,
                                            name=nm + "out", dtype=dtype)
        self.norm1 = ops.FusedLayerNorm(hidden_size, LN_EPS, dtype=dtype)
        self.linear1 = L.ColumnParallelLinear(hidden_size, intermediate_size, skip_bias_add=True,
                                              std=std, name=nm + "fc1", dtype=dtype)
        self.linear2 = L.RowParallelLinear(intermediate_size, hidden_size, skip_bias_add=True,
                                           std=std, name=nm + "fc2", dtype=dtype)
        self.norm2 = ops.FusedLayerNorm(hidden_size, LN_EPS, dtype=dtype)
        self.act = _act(hidden_act)

    def forward(self, x, key_bias):
        b, s, _ = x.shape
        qkv = self.qkv(x).view(b, s, self.heads, 3, self.head_dim)
        pa = self.pa if self.training else 0.0
        o = ops.flash_attention_qkvpacked(qkv, causal=False, dropout_p=pa,
                                          key=_key(pa, self.training), key_bias=key_bias)
        a, ab = self.out_proj(o.reshape(b, s, self.heads * self.head_dim))
        p = self.p if self.training else 0.0
        _, h = ops.add_layer_norm(a, ab, x, self.norm1.weight, self.norm1.bias, LN_EPS, p,
                                  _key(p, self.training))
        y, yb = self.linear1(h)
        m, mb = self.linear2(self.act(y, yb))
        _, out = ops.add_layer_norm(m, mb, h, self.norm2.weight, self.norm2.bias, LN_EPS, p,
                                    _key(p, self.training))
        return out


class ErniePooler(nn.Module):
    def __init__(self, hidden_size, std, dtype=None):
        super().__init__()
        self.dense = nn.Linear(hidden_size, hidden_size, dtype=dtype)
        nn.init.normal_(self.dense.weight, 0.0, std)
        nn.init.zeros_(self.dense.bias)

    def forward(self, hidden_states):
        return torch.tanh(self.dense(hidden_states[:, 0]))


class ErnieModel(nn.Module):
    def __init__(self, vocab_size, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                 intermediate_size=3072, hidden_act="gelu", hidden_dropout_prob=0.1,
                 attention_probs_dropout_prob=0.1, max_position_embeddings=512, type_vocab_size=2,
                 initializer_range=0.02, pad_token_id=0, task_type_vocab_size=3, task_id=0,
                 use_task_id=False, use_recompute=False, dtype=None, **kwargs):
        super().__init__()
        self.pad_token_id = pad_token_id
        self.initializer_range = initializer_range
        self.hidden_size, self.vocab_size, self.hidden_act = hidden_size, vocab_size, hidden_act
        self.hidden_dropout_prob = hidden_dropout_prob
        self.use_recompute = use_recompute
        self.embeddings = ErnieEmbeddings(vocab_size, hidden_size, hidden_dropout_prob,
                                          max_position_embeddings, type_vocab_size, pad_token_id,
                                          initializer_range, task_type_vocab_size, task_id,
                                          use_task_id, dtype)
        self.encoder = nn.ModuleList([
            ErnieEncoderLayer(hidden_size, num_attention_heads, intermediate_size,
                              hidden_dropout_prob, attention_probs_dropout_prob, hidden_act,
                              initializer_range, i, dtype) for i in range(num_hidden_layers)])
        self.pooler = ErniePooler(hidden_size, initializer_range, dtype)

    def key_bias(self, input_ids, attention_mask):
        if attention_mask is None:
            return (input_ids == self.pad_token_id).float() * -1e4
        m = attention_mask
        if m.dim() == 4 and m.shape[1] == 1 and m.shape[2] == 1:
            return m.reshape(m.shape[0], -1).float()  # already additive [B,1,1,S]
        if m.dim() == 2:
            if m.dtype == torch.bool:
                return (~m).float() * -1e4
            if m.is_floating_point() and (m < 0).any():
                return m.float()  # additive
            return (1.0 - m.float()) * -1e4
        raise ValueError("attention_mask must be [B, S] or [B, 1, 1, S] (key padding masks)")

    def forward(self, input_ids, token_type_ids=None, position_ids=None, attention_mask=None,
                task_type_ids=None, output_hidden_states=False):
        kb = self.key_bias(input_ids, attention_mask)
        x = self.embeddings(input_ids, token_type_ids, position_ids, task_type_ids)
        hidden = [x] if output_hidden_states else None
        for layer in self.encoder:
            if self.use_recompute and self.training:
                x = recompute(layer, x, kb)
            else:
                x = layer(x, kb)
            if hidden is not None:
                hidden.append(x)
        pooled = self.pooler(x)
        if output_hidden_states:
            return x, pooled, hidden
        return x, pooled


class ErnieLMPredictionHead(nn.Module):
    def __init__(self, hidden_size, vocab_size, activation, embedding_weights=None, std=0.02,
                 dtype=None):
        super().__init__()
        self.transform = nn.Linear(hidden_size, hidden_size, dtype=dtype)
        nn.init.normal_(self.transform.weight, 0.0, std)
        nn.init.zeros_(self.transform.bias)
        self.act = _act(activation)
        self.layer_norm = ops.FusedLayerNorm(hidden_size, LN_EPS, dtype=dtype)
        t = topo.mp_world_size()
        if embedding_weights is None:
            self.decoder_weight = nn.Parameter(L.init_full_then_slice(
                (vocab_size, hidden_size), std, "ernie.lm_decoder", dim=0, dtype=dtype))
            self.decoder_weight.tp_split = t > 1
            self.decoder_weight.tp_dim = 0
        else:
            self.decoder_weight = embedding_weights
        self.decoder_bias = nn.Parameter(torch.zeros(vocab_size // t, dtype=dtype or torch.float32))
        self.decoder_bias.tp_split = t > 1
        self.decoder_bias.tp_dim = 0

    def forward(self, hidden_states, masked_positions=None):
        if masked_positions is not None:
            hidden_states = hidden_states.reshape(-1, hidden_states.shape[-1])[masked_positions]
        h = self.act(F.linear(hidden_states, self.transform.weight), self.transform.bias)
        h = self.layer_norm(h)
        # vocab-parallel logits (local shard) + shard bias
        return L.parallel_lm_logits(h, self.decoder_weight) + self.decoder_bias


class ErniePretrainingHeads(nn.Module):
    def __init__(self, hidden_size, vocab_size, activation, embedding_weights=None, std=0.02,
                 dtype=None):
        super().__init__()
        self.predictions = ErnieLMPredictionHead(hidden_size, vocab_size, activation,
                                                 embedding_weights, std, dtype)
        self.seq_relationship = nn.Linear(hidden_size, 2, dtype=dtype)
        nn.init.normal_(self.seq_relationship.weight, 0.0, std)
        nn.init.zeros_(self.seq_relationship.bias)

    def forward(self, sequence_output, pooled_output, masked_positions=None):
        return (self.predictions(sequence_output, masked_positions),
                self.seq_relationship(pooled_output))


def _vocab_ce(logits, labels, ignore_index=-1):
    g = topo.get_hcg().get_model_parallel_group() if topo.mp_world_size() > 1 else None
    vs = topo.mp_rank() * logits.shape[-1]
    return ops.softmax_cross_entropy(logits, labels, group=g, vocab_start=vs,
                                     ignore_index=ignore_index)


class ErnieForPretraining(nn.Module):
    def __init__(self, ernie):
        super().__init__()
        self.ernie = ernie
        dt = ernie.pooler.dense.weight.dtype
        self.cls = ErniePretrainingHeads(ernie.hidden_size, ernie.vocab_size, ernie.hidden_act,
                                         ernie.embeddings.word_embeddings.weight,
                                         ernie.initializer_range, dt)

    def forward(self, input_ids, token_type_ids=None, position_ids=None, attention_mask=None,
                masked_positions=None, labels=None, next_sentence_label=None):
        seq, pooled = self.ernie(input_ids, token_type_ids, position_ids, attention_mask)
        scores, rel = self.cls(seq, pooled, masked_positions)
        if labels is not None and next_sentence_label is not None:
            mlm = _vocab_ce(scores.reshape(-1, scores.shape[-1]), labels.reshape(-1), -100)
            valid = (labels.reshape(-1) != -100).float()
            mlm = (mlm.reshape(-1) * valid).sum() / valid.sum().clamp_min(1.0)
            nsp = F.cross_entropy(rel.float().reshape(-1, 2), next_sentence_label.reshape(-1))
            return mlm + nsp, scores, rel
        return scores, rel


class ErniePretrainingCriterion(nn.Module):
    """Mean MLM CE over non-ignored (``-1``) labels (+ mean NSP CE)."""

    def __init__(self, with_nsp_loss=True):
        super().__init__()
        self.with_nsp_loss = with_nsp_loss

    def forward(self, prediction_scores, seq_relationship_score, masked_lm_labels,
                next_sentence_labels=None):
        lab = masked_lm_labels.reshape(-1)
        ce = _vocab_ce(prediction_scores.reshape(-1, prediction_scores.shape[-1]), lab, -1)
        valid = (lab != -1).float()
        mlm = (ce.reshape(-1) * valid).sum() / valid.sum().clamp_min(1.0)
        if not self.with_nsp_loss:
            return mlm
        nsp = F.cross_entropy(seq_relationship_score.float().reshape(-1, 2),
                              next_sentence_labels.reshape(-1).long())
        return mlm, nsp


class ErnieForMaskedLM(nn.Module):
    def __init__(self, ernie):
        super().__init__()
        self.ernie = ernie
        dt = ernie.pooler.dense.weight.dtype
        self.cls = ErnieLMPredictionHead(ernie.hidden_size, ernie.vocab_size, ernie.hidden_act,
                                         ernie.embeddings.word_embeddings.weight,
                                         ernie.initializer_range, dt)

    def forward(self, input_ids, token_type_ids=None, position_ids=None, attention_mask=None,
                masked_positions=None, labels=None):
        seq, _ = self.ernie(input_ids, token_type_ids, position_ids, attention_mask)
        scores = self.cls(seq, masked_positions)
        if labels is None:
            return scores
        ce = _vocab_ce(scores.reshape(-1, scores.shape[-1]), labels.reshape(-1), -100)
        valid = (labels.reshape(-1) != -100).float()
        return (ce.reshape(-1) * valid).sum() / valid.sum().clamp_min(1.0), scores


class ErnieForMultipleChoice(nn.Module):
    def __init__(self, ernie, num_choices=2, dropout=None):
        super().__init__()
        self.ernie, self.num_choices = ernie, num_choices
        self.p = dropout if dropout is not None else ernie.hidden_dropout_prob
        dt = ernie.pooler.dense.weight.dtype
        self.classifier = nn.Linear(ernie.hidden_size, 1, dtype=dt)
        nn.init.normal_(self.classifier.weight, 0.0, ernie.initializer_range)
        nn.init.zeros_(self.classifier.bias)

    def forward(self, input_ids, token_type_ids=None, position_ids=None, attention_mask=None,
                labels=None):
        flat = lambda t: None if t is None else t.reshape(-1, t.shape[-1])  # noqa: E731
        _, pooled = self.ernie(flat(input_ids), flat(token_type_ids), flat(position_ids),
                               flat(attention_mask))
        p = self.p if self.training else 0.0
        if p > 0:
            pooled = ops.dropout(pooled, p, _key(p, True))
        logits = self.classifier(pooled).reshape(-1, self.num_choices)
        if labels is None:
            return logits
        return F.cross_entropy(logits.float(), labels.reshape(-1).long()), logits


def mlm_mask(tokens, vocab_size, mask_token_id, mask_prob=0.15, special_ids=(), generator=None):
    """Dynamic BERT masking on device: of the selected ``mask_prob`` positions
    80% -> ``[MASK]``, 10% -> random token, 10% unchanged.  Returns
    ``(inputs, labels)`` with ``labels = -1`` at unselected positions."""
    dev = tokens.device
    r = torch.rand(tokens.shape, device=dev, generator=generator)
    sel = r < mask_prob
    for s in special_ids:
        sel &= tokens != s
    labels = torch.where(sel, tokens, torch.full_like(tokens, -1))
    r2 = torch.rand(tokens.shape, device=dev, generator=generator)
    rnd = torch.randint(0, vocab_size, tokens.shape, device=dev, generator=generator)
    inputs = torch.where(sel & (r2 < 0.8), torch.full_like(tokens, mask_token_id), tokens)
    inputs = torch.where(sel & (r2 >= 0.8) & (r2 < 0.9), rnd, inputs)
    return inputs, labels

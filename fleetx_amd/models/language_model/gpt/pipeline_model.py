"""GPT as a pipeline of stage chunks (1F1B / interleaved).

Parity: reference ``GPTForPretrainingPipe`` (``hybrid_model.py:838-962``,
C29): ``EmbeddingPipe`` on the first stage, ``num_layers`` decoder layers cut
uniformly ("layer:TransformerDecoderLayer"), final LN + LM head on the last
stage with the head weight shared with the first stage's word embedding
(``SharedLayerDesc``), loss per micro-batch averaged over the step,
``num_virtual_pipeline_stages = virtual_pp_degree``.  Sequence parallelism is
not combined with PP (as in the reference, ``hybrid_model.py:892-893``).

The tied weight exists on both end stages; both copies start identical
(same per-name init seed), carry ``shared_embedding=True`` so the grad buffer
all-reduces their gradients over the first/last-stage group, and the
last-stage copy is excluded from the global grad-norm (counted once).
"""
import torch
import torch.nn as nn

from ....parallel import layers as L
from ....parallel.pipeline import PipelineSchedule
from .model import GPTModel, GPTPretrainingCriterion


class GPTForPretrainingPipe(nn.Module):
    def __init__(self, cfg, hcg, virtual_pp_degree=1):
        super().__init__()
        assert not cfg.sequence_parallel, "sequence parallel is not supported with pipeline parallel"
        self.cfg = cfg
        self.hcg = hcg
        P, r, V = hcg.pp_degree, hcg.pp_rank, virtual_pp_degree
        self.P, self.V = P, V
        assert cfg.num_layers % (P * V) == 0
        per = cfg.num_layers // (P * V)
        chunks = []
        for c in range(V):
            v = c * P + r
            chunks.append(GPTModel(cfg, layer_range=(v * per, (v + 1) * per),
                                   has_embedding=(v == 0), has_final_ln=(v == P * V - 1)))
        self.chunks = nn.ModuleList(chunks)
        self.is_first = r == 0
        self.is_last = r == P - 1
        if self.is_first:
            self.chunks[0].embeddings.word_embeddings.weight.shared_embedding = True
        if self.is_last:
            w = L.init_full_then_slice((cfg.vocab_size, cfg.hidden_size), cfg.initializer_range,
                                       "embeddings.word.weight", dim=0, dtype=cfg.dtype)
            self.shared_word_embeddings = nn.Parameter(w)
            self.shared_word_embeddings.tp_split = hcg.mp_degree > 1
            self.shared_word_embeddings.tp_dim = 0
            self.shared_word_embeddings.shared_embedding = True
            self.shared_word_embeddings.norm_exclude = True
        self.criterion = GPTPretrainingCriterion(cfg)
        self.engine = None
        self._schedule = None

    def attach(self, engine):
        self.engine = engine

    def _head_weight(self):
        if self.is_first and self.is_last:
            return self.chunks[0].embeddings.word_embeddings.weight
        return self.shared_word_embeddings

    def _schedule_for(self, micro_shape):
        p = next(self.parameters())
        if self._schedule is None:
            self._schedule = PipelineSchedule(self.hcg, lambda: self._act_shape, p.dtype, p.device,
                                              num_chunks=self.V)
        self._act_shape = micro_shape
        return self._schedule

    def _stage_fn(self, m, tokens, pos, labels, mask):
        def fn(c, k, x):
            chunk = self.chunks[c]
            if chunk.embeddings is not None:
                x = chunk(input_ids=tokens[k], position_ids=pos[k])
            else:
                x = chunk(hidden=x)
            if chunk.final_ln is not None:
                logits = L.parallel_lm_logits(x, self._head_weight(), parallel_output=True)
                return self.criterion(logits, labels[k], mask[k]) / m
            return x
        return fn

    def _split(self, data, m):
        (tokens, pos), (labels, mask) = data
        return (tokens.chunk(m), pos.chunk(m), labels.chunk(m), mask.chunk(m))

    def train_batch(self, data, accumulate_steps):
        m = accumulate_steps
        tokens, pos, labels, mask = self._split(data, m)
        mb, s = tokens[0].shape
        sched = self._schedule_for((mb, s, self.cfg.hidden_size))
        buf = self.engine.buffer if self.engine is not None else None
        if buf is not None:
            buf.set_last_micro_batch(False)
        last_cb = (lambda: buf.set_last_micro_batch(True)) if buf is not None else None
        fn = self._stage_fn(m, tokens, pos, labels, mask)
        if self.V > 1:
            return sched.train_interleaved(m, fn, last_cb)
        return sched.train_1f1b(m, fn, last_cb)

    @torch.no_grad()
    def eval_batch(self, data, compute_loss=True):
        m = max(1, self.engine._accumulate_steps if self.engine is not None else 1)
        tokens, pos, labels, mask = self._split(data, m)
        mb, s = tokens[0].shape
        sched = self._schedule_for((mb, s, self.cfg.hidden_size))
        fn = self._stage_fn(m, tokens, pos, labels, mask)
        if self.V > 1:
            return sched.forward_only_interleaved(m, fn)
        return sched.forward_only(m, fn)

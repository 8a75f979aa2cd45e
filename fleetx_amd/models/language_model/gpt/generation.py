"""Autoregressive generation for GPT with a preallocated KV cache.

Parity: reference ``GPTForGeneration`` (``single_model.py:656-1122``, C27)
and its logits processors (``gpt/dygraph/processor.py:22-200``): min-length,
repetition penalty, Hamming diversity, forced BOS/EOS; sampling with
temperature / top-k / top-p + multinomial, and greedy search; per-token score
bookkeeping; stop when every sequence has produced EOS.  The hybrid (TP)
variant works here (reference defect §2.12 #1): logits are gathered over the
mp group before sampling.

MI355X design (K18/K19):
* prompts are RIGHT-padded and carried with per-sample lengths; the prefill
  runs the fused flash-attention kernel with ``kv_lens``, so no additive
  mask tensor is built;
* the KV cache is allocated once, ``[layers][B, max_len, heads, d]``, and each
  step writes one row per sample in place (no concat / re-allocation as in the
  reference ``_forward_`` path);
* per-token attention uses the split-free decode kernel
  (``ops.decode_attention``) that streams the cache once.
"""
import os
import torch
import torch.nn.functional as F

from .... import ops
from ....parallel import mappings as M
from ....parallel import topology as topo


# ----------------------------------------------------------------------------
# logits processors
# ----------------------------------------------------------------------------
class LogitsProcessor:
    def __call__(self, input_ids, logits):
        raise NotImplementedError


class LogitsProcessorList(list):
    def __call__(self, input_ids, logits, **kw):
        for p in self:
            logits = p(input_ids, logits)
        return logits


class MinLengthLogitsProcessor(LogitsProcessor):
    def __init__(self, min_length, eos_token_id):
        self.min_length, self.eos = min_length, eos_token_id
        self.cur_len = None

    def __call__(self, input_ids, logits):
        if self.cur_len is not None and self.cur_len < self.min_length:
            logits[:, self.eos] = -1e9
        return logits


class RepetitionPenaltyLogitsProcessor(LogitsProcessor):
    def __init__(self, penalty):
        assert penalty > 0
        self.penalty = penalty

    def __call__(self, input_ids, logits):
        score = torch.gather(logits, 1, input_ids)
        score = torch.where(score < 0, score * self.penalty, score / self.penalty)
        logits.scatter_(1, input_ids, score)
        return logits


class HammingDiversityLogitsProcessor(LogitsProcessor):
    """Penalise tokens chosen by earlier groups at this step (beam groups)."""

    def __init__(self, diversity_rate, num_beams, num_beam_groups):
        self.rate = diversity_rate
        self.group_size = num_beams // num_beam_groups
        self.num_beam_groups = num_beam_groups
        self.previous_tokens = None

    def __call__(self, input_ids, logits):
        if self.previous_tokens is None or self.rate == 0:
            return logits
        freq = torch.zeros_like(logits)
        freq.scatter_add_(1, self.previous_tokens, torch.ones_like(self.previous_tokens, dtype=logits.dtype))
        return logits - self.rate * freq


class ForcedBOSTokenLogitsProcessor(LogitsProcessor):
    def __init__(self, bos_token_id):
        self.bos = bos_token_id
        self.step = 0

    def __call__(self, input_ids, logits):
        if self.step == 0:
            logits[:] = -1e9
            logits[:, self.bos] = 0
        self.step += 1
        return logits


class ForcedEOSTokenLogitsProcessor(LogitsProcessor):
    def __init__(self, max_length, eos_token_id):
        self.max_length, self.eos = max_length, eos_token_id
        self.cur_len = None

    def __call__(self, input_ids, logits):
        if self.cur_len is not None and self.cur_len == self.max_length - 1:
            logits[:] = -1e9
            logits[:, self.eos] = 0
        return logits


def top_k_filter(probs, k, min_keep=1):
    k = min(max(k, min_keep), probs.shape[-1])
    kth = torch.topk(probs, k, dim=-1).values[:, -1:]
    return torch.where(probs >= kth, probs, torch.zeros_like(probs))


def top_p_filter(probs, p, min_keep=1):
    sp, si = torch.sort(probs, descending=True, dim=-1)
    cum = torch.cumsum(sp, dim=-1)
    remove = cum > p
    if min_keep > 1:
        remove[:, :min_keep - 1] = False
    remove[:, 1:] = remove[:, :-1].clone()
    remove[:, 0] = False
    mask = torch.zeros_like(remove).scatter(1, si, remove)
    return torch.where(mask, torch.zeros_like(probs), probs)


# ----------------------------------------------------------------------------
# cached decoding
# ----------------------------------------------------------------------------
class KVCache:
    def __init__(self, num_layers, batch, max_len, heads, head_dim, dtype, device):
        self.k = [torch.zeros(batch, max_len, heads, head_dim, dtype=dtype, device=device)
                  for _ in range(num_layers)]
        self.v = [torch.zeros_like(t) for t in self.k]
        self.max_len = max_len


def _layer_prefill(layer, x, cache, li, lens):
    """Full-prompt pass of one decoder layer that also fills the KV cache."""
    attn = layer.attn
    h = layer.ln1(x)
    qkv = attn.qkv_proj(h)
    b, s = qkv.shape[0], qkv.shape[1]
    qkv5 = qkv.view(b, s, attn.heads, 3, attn.head_dim)
    cache.k[li][:, :s] = qkv5[:, :, :, 1]
    cache.v[li][:, :s] = qkv5[:, :, :, 2]
    o = ops.flash_attention(qkv5[:, :, :, 0], qkv5[:, :, :, 1], qkv5[:, :, :, 2], causal=True,
                            kv_lens=lens).reshape(b, s, -1)
    a, ab = attn.out_proj(o)
    x2, h2 = ops.add_layer_norm(a, ab, x, layer.ln2.weight, layer.ln2.bias, layer.ln2.eps)
    m, mb = layer.mlp(h2)
    return ops.bias_dropout_add(m, mb, x2)


def _layer_decode(layer, x, cache, li, pos, lens_after):
    """One-token pass: x [B, 1, h]; writes K/V at ``pos`` [B] and attends."""
    attn = layer.attn
    h = layer.ln1(x)
    qkv = attn.qkv_proj(h)
    b = qkv.shape[0]
    qkv5 = qkv.view(b, attn.heads, 3, attn.head_dim)
    ar = torch.arange(b, device=x.device)
    cache.k[li][ar, pos] = qkv5[:, :, 1]
    cache.v[li][ar, pos] = qkv5[:, :, 2]
    o = ops.decode_attention(qkv5[:, :, 0].contiguous(), cache.k[li], cache.v[li], lens_after)
    a, ab = attn.out_proj(o.reshape(b, 1, -1))
    x2, h2 = ops.add_layer_norm(a, ab, x, layer.ln2.weight, layer.ln2.bias, layer.ln2.eps)
    m, mb = layer.mlp(h2)
    return ops.bias_dropout_add(m, mb, x2)


def _fusable(layer):
    from ....parallel import layers as L
    a, m = layer.attn, layer.mlp
    return (topo.mp_world_size() == 1 and type(a.qkv_proj) is L.ColumnParallelLinear
            and type(a.out_proj) is L.RowParallelLinear and type(m.fc1) is L.ColumnParallelLinear
            and type(m.fc2) is L.RowParallelLinear)


# LayerNorm as a GEMV prologue in the fused decode layer (FLEETX_DECODE_LN_FUSE=0: separate launch)
_LN_FUSE = os.environ.get("FLEETX_DECODE_LN_FUSE", "1") == "1"


def _layer_decode_fused(layer, x, cache, li, pos, lens_after):
    """One-token pass as four GEMV launches and the attention (K19, the
    fused_multi_transformer counterpart): [LN1 + QKV GEMV + bias, K/V appended
    to the cache in the epilogue] -> split-K decode attention -> [out-proj
    GEMV + bias + residual] -> [LN2 + FFN1 GEMV + bias + GeLU] -> [FFN2 GEMV +
    bias + residual].  The LayerNorms run as GEMV prologues (each block
    normalises the few rows into LDS); shapes the fused prologue does not
    cover fall back to a separate LayerNorm launch.  Returns None when a GEMV
    does not cover the shape (batch > 16)."""
    from ....ops import gemm as G
    attn, mlp = layer.attn, layer.mlp
    B, h = x.shape[0], x.shape[-1]
    x2d = x.reshape(B, h)
    kv = (cache.k[li], cache.v[li], pos)
    q = G.decode_linear(x2d, attn.qkv_proj.weight, attn.qkv_proj.bias, G.GV_QKV, qkv_cache=kv,
                        ln=(layer.ln1.weight, layer.ln1.bias, layer.ln1.eps)) if _LN_FUSE else None
    if q is None:
        q = G.decode_linear(layer.ln1(x2d), attn.qkv_proj.weight, attn.qkv_proj.bias, G.GV_QKV,
                            qkv_cache=kv)
    if q is None:
        return None
    o = ops.decode_attention(q.view(B, attn.heads, attn.head_dim), cache.k[li], cache.v[li],
                             lens_after)
    x2 = G.decode_linear(o.view(B, -1), attn.out_proj.weight, attn.out_proj.bias, G.GV_RES,
                         res=x2d)
    f = G.decode_linear(x2, mlp.fc1.weight, mlp.fc1.bias, G.GV_GELU,
                        ln=(layer.ln2.weight, layer.ln2.bias, layer.ln2.eps)) if _LN_FUSE else None
    if f is None:
        f = G.decode_linear(layer.ln2(x2), mlp.fc1.weight, mlp.fc1.bias, G.GV_GELU)
    out = G.decode_linear(f, mlp.fc2.weight, mlp.fc2.bias, G.GV_RES, res=x2)
    return out.view(B, 1, h)


class _GraphedDecodeStep:
    """The per-token decode step (embedding -> L decoder layers against the KV
    cache -> final LN -> logits) captured once into a HIP graph and replayed
    for every following token.

    At decode batch sizes every op is a tiny, launch-bound kernel (~10 per
    layer), so the eager loop is host-bound; a replay issues the whole step as
    one graph launch.  This is the MI355X counterpart of the reference's
    static inference program with ``fused_multi_transformer`` (K19 / N-12):
    the same fused HIP kernels, with the launch overhead removed by the graph
    instead of a tracing compiler.  The first call runs eagerly (it is also
    that token's real work) and captures; inputs live in static tensors.
    """

    def __init__(self, gen, cache, batch):
        self.gen, self.cache = gen, cache
        dev = cache.k[0].device
        self.nxt = torch.zeros(batch, dtype=torch.long, device=dev)
        self.cur = torch.zeros(batch, dtype=torch.long, device=dev)
        self.graph = None
        self.logits = None

    def __call__(self, nxt, cur):
        self.nxt.copy_(nxt)
        self.cur.copy_(cur)
        if self.graph is None:
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):  # warm-up off the capture stream
                out = self.gen._decode_step(self.nxt, self.cur, self.cache)
            torch.cuda.current_stream().wait_stream(side)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.logits = self.gen._decode_step(self.nxt, self.cur, self.cache)
            return out
        self.graph.replay()
        return self.logits


class GPTForGeneration(torch.nn.Module):
    def __init__(self, pretrain_model, configs):
        super().__init__()
        self.model = pretrain_model  # GPTForPretraining
        self.gpt = pretrain_model.gpt
        c = configs or {}
        self.max_length = c.get("max_dec_len", 20)
        self.min_length = c.get("min_dec_len", 0)
        self.decode_strategy = c.get("decode_strategy", "sampling")
        self.temperature = c.get("temperature", 1.0)
        self.top_k = c.get("top_k", 0)
        self.top_p = c.get("top_p", 1.0)
        self.repetition_penalty = c.get("repetition_penalty", 1.0)
        self.num_beams = c.get("num_beams", 1)
        self.num_beam_groups = c.get("num_beam_groups", 1)
        self.diversity_rate = c.get("diversity_rate", 0.0)
        self.bos_token_id = c.get("bos_token_id")
        self.eos_token_id = c.get("eos_token_id")
        self.pad_token_id = c.get("pad_token_id")
        self.forced_bos_token_id = c.get("forced_bos_token_id")
        self.forced_eos_token_id = c.get("forced_eos_token_id")
        self.num_return_sequences = c.get("num_return_sequences", 1)
        self.use_hip_graph = bool(c.get("use_hip_graph", True))
        # decode layers as five fused kernels with weight-streaming GEMVs (K19)
        self.fused_decode = bool(c.get("fused_decode", True))
        if self.decode_strategy not in ("sampling", "greedy_search"):
            raise ValueError("decode_strategy must be sampling or greedy_search")

    def _processors(self, max_len):
        procs = LogitsProcessorList()
        if self.min_length and self.eos_token_id is not None:
            procs.append(MinLengthLogitsProcessor(self.min_length, self.eos_token_id))
        if self.repetition_penalty and self.repetition_penalty != 1.0:
            procs.append(RepetitionPenaltyLogitsProcessor(self.repetition_penalty))
        if self.num_beam_groups > 1 and self.diversity_rate > 0:
            procs.append(HammingDiversityLogitsProcessor(self.diversity_rate, self.num_beams,
                                                         self.num_beam_groups))
        if self.forced_bos_token_id is not None:
            procs.append(ForcedBOSTokenLogitsProcessor(self.forced_bos_token_id))
        if self.forced_eos_token_id is not None:
            procs.append(ForcedEOSTokenLogitsProcessor(max_len, self.forced_eos_token_id))
        return procs

    def _decode_step(self, nxt, cur, cache):
        """Embed token ``nxt`` at position ``cur`` [B], run every layer against
        the KV cache (appending this token), return fp32 logits [B, V]."""
        x = ops.embedding(nxt[:, None], self.gpt.embeddings.word_embeddings.weight,
                          cur[:, None], self.gpt.embeddings.position_embeddings, 0) \
            if topo.mp_world_size() == 1 else self.gpt.embeddings(nxt[:, None], cur[:, None])
        after = (cur + 1).to(torch.int32)
        fused = self.fused_decode and x.is_cuda and x.shape[0] <= 16
        for li, layer in enumerate(self.gpt.layers):
            y = _layer_decode_fused(layer, x, cache, li, cur, after) \
                if fused and _fusable(layer) else None
            x = y if y is not None else _layer_decode(layer, x, cache, li, cur, after)
        x = self.gpt.final_ln(x)
        return self._logits(x[:, 0])

    def _logits(self, h):
        w = self.gpt.embeddings.word_embeddings.weight
        logits = None
        if self.fused_decode and topo.mp_world_size() == 1:
            from ....ops import gemm as G
            logits = G.decode_linear(h.contiguous(), w)
        if logits is None:
            logits = F.linear(h, w)
        if topo.mp_world_size() > 1:
            logits = M.gather_from_mp(logits)
        return logits.float()

    @torch.no_grad()
    def generate(self, input_ids, lens=None, max_length=None, seed=None):
        """input_ids: [B, S] right-padded; lens: [B] prompt lengths.
        Returns (generated ids [B, T], scores [B])."""
        self.eval()
        dev = input_ids.device
        if self.num_return_sequences > 1:
            input_ids = input_ids.repeat_interleave(self.num_return_sequences, 0)
            if lens is not None:
                lens = lens.repeat_interleave(self.num_return_sequences, 0)
        B, S = input_ids.shape
        lens = lens.to(dev) if lens is not None else torch.full((B,), S, device=dev,
                                                                dtype=torch.long)
        max_new = max_length or self.max_length
        cfg = self.gpt.cfg
        total = min(int(lens.max().item()) + max_new, cfg.max_position_embeddings)
        p = next(self.parameters())
        attn0 = self.gpt.layers[0].attn
        cache = KVCache(len(self.gpt.layers), B, total, attn0.heads, attn0.head_dim, p.dtype, dev)
        gen = None
        if seed is not None:
            gen = torch.Generator(device=dev)
            gen.manual_seed(seed)
        # ---- prefill
        pos = torch.arange(S, device=dev).unsqueeze(0).expand(B, S)
        x = self.gpt.embeddings(input_ids, pos)
        for li, layer in enumerate(self.gpt.layers):
            x = _layer_prefill(layer, x, cache, li, lens.to(torch.int32))
        x = self.gpt.final_ln(x)
        last = x[torch.arange(B, device=dev), lens - 1]
        logits = self._logits(last)
        procs = self._processors(max_new)
        eos = self.eos_token_id
        pad = self.pad_token_id if self.pad_token_id is not None else (eos if eos is not None else 0)
        unfinished = torch.ones(B, dtype=torch.bool, device=dev)
        scores = torch.zeros(B, device=dev)
        out_tokens = []
        cur = lens.clone()
        history = input_ids.clone()
        graphed = None
        for step in range(max_new):
            if cur.max().item() >= total:
                break
            for pr in procs:
                if hasattr(pr, "cur_len"):
                    pr.cur_len = step
            logits = procs(history, logits)
            if self.decode_strategy != "greedy_search" and logits.is_cuda:
                # one fused HIP launch: softmax/T, top-k, top-p, draw, logsumexp
                nxt, lse = ops.fused_sample(logits, self.temperature, self.top_k, self.top_p,
                                            generator=gen)
                step_score = logits.gather(1, nxt[:, None]).squeeze(1).float() - lse
            else:
                logp = torch.log_softmax(logits, -1)
                if self.decode_strategy == "greedy_search":
                    nxt = torch.argmax(logits, -1)
                else:
                    lg = logits / self.temperature if self.temperature not in (None, 1.0) \
                        else logits
                    probs = torch.softmax(lg, -1)
                    if self.top_k:
                        probs = top_k_filter(probs, self.top_k)
                    if self.top_p is not None and self.top_p < 1.0:
                        probs = top_p_filter(probs, self.top_p)
                    nxt = torch.multinomial(probs, 1, generator=gen).squeeze(1)
                step_score = logp.gather(1, nxt[:, None]).squeeze(1)
            nxt = torch.where(unfinished, nxt, torch.full_like(nxt, pad))
            scores = torch.where(unfinished, scores + step_score, scores)
            out_tokens.append(nxt)
            history = torch.cat([history, nxt[:, None]], 1)
            if eos is not None:
                unfinished = unfinished & (nxt != eos)
                if not bool(unfinished.any()):
                    break
            # ---- one decode step (replayed from a HIP graph after the first token)
            if graphed is None and self.use_hip_graph and dev.type == "cuda" \
                    and topo.mp_world_size() == 1:
                graphed = _GraphedDecodeStep(self, cache, B)
            logits = graphed(nxt, cur) if graphed is not None else \
                self._decode_step(nxt, cur, cache)
            cur = cur + 1
        if not out_tokens:
            return torch.zeros(B, 0, dtype=torch.long, device=dev), scores
        return torch.stack(out_tokens, 1), scores

    def forward(self, input_ids, lens=None):
        return self.generate(input_ids, lens)

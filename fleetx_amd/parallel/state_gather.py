"""Gather the distributed fp32 training state into the single-rank layout.

The fp32 master weights of a hybrid job live in pieces: each ZeRO rank owns
a slice of the flat buffer (``grad_buffer.owned_ranges``), tensor-parallel
weights are split along their ``tp_dim`` (column-parallel rows, row-parallel
columns, vocab-parallel rows), and pipeline stages hold disjoint layers under
stage-local names (``chunks.<c>.layers.<i>``).  :func:`gather_master_state`
undoes all three and returns ``{name: fp32 CPU tensor}`` named as the
single-rank model names them (``gpt.layers.<global i>...``) -- what a
checkpoint merge or a layout-equivalence test compares tensor by tensor.

Reference parity: the merged-parameter view Paddle's ``save_for_auto`` /
dist-checkpoint merge produce (reference ``eager_engine.py:581-660`` saves
per-rank shards; merging them is a new capability here).
Collective: every rank of the job must call it.
"""
import re

import torch
import torch.distributed as dist

_CHUNK = re.compile(r"^chunks\.(\d+)\.(.*)$")
_LAYER = re.compile(r"^layers\.(\d+)\.(.*)$")


def canonical_name(name, hcg=None, model=None):
    """Single-rank name of a parameter of a pipeline stage model (identity
    for non-pipeline models).  The last stage's copy of the tied word
    embedding maps to ``<embedding>#tied``."""
    if name == "shared_word_embeddings":
        return "gpt.embeddings.word_embeddings.weight#tied"
    m = _CHUNK.match(name)
    if m is None:
        return name
    c, rest = int(m.group(1)), m.group(2)
    lm = _LAYER.match(rest)
    if lm is not None:
        P = hcg.pp_degree if hcg is not None else 1
        r = hcg.pp_rank if hcg is not None else 0
        V = len(model.chunks) if model is not None else 1
        per = model.cfg.num_layers // (P * V) if model is not None else 0
        g = (c * P + r) * per + int(lm.group(1))
        return "gpt.layers.%d.%s" % (g, lm.group(2))
    return "gpt." + rest


def _owned_flat(opt):
    buf = opt.buffer
    flat = torch.zeros(buf.numel, dtype=torch.float32, device=buf.device)
    for (s, e, _), m in zip(opt.ranges, opt.master):
        flat[s:e].copy_(m.to(flat.device, non_blocking=False))
    return flat


def _flat_params(opt):
    """[(name, param, fp32 full local value)] for a FlatParamGradBuffer:
    owned ranges are disjoint across the ZeRO group, so a sum assembles the
    flat buffer."""
    buf = opt.buffer
    flat = _owned_flat(opt)
    if buf.shard_stage >= 1 and buf.shard_group is not None:
        dist.all_reduce(flat, group=buf.shard_group.group)
    out = []
    for n, p in buf.params:
        o, k = buf.offsets[id(p)]
        out.append((n, p, flat[o:o + k].view(p.shape)))
    return out


def _unit_params(opt):
    """Same for the per-layer-unit buffer of ZeRO-2/3 (``sharding.py``): rank
    r holds piece r of every unit segment; all-gather each segment."""
    buf = opt.buffer
    flat = _owned_flat(opt)
    g = buf.shard_group
    out = []
    for u in buf.all_units:
        for seg in u.segments:
            piece = flat[seg.sstart:seg.send].contiguous()
            parts = [torch.empty_like(piece) for _ in range(g.nranks)]
            dist.all_gather(parts, piece, group=g.group)
            full = torch.cat(parts)
            for n, p, o in seg.params:
                a = o - seg.fstart
                out.append((n, p, full[a:a + p.numel()].view(p.shape)))
    return out


def gather_master_state(engine):
    """``{single-rank name: fp32 CPU tensor}`` of the full master weights."""
    opt, buf, hcg = engine.optimizer, engine.buffer, engine.hcg
    if hasattr(opt, "sync_state"):
        opt.sync_state()
    triples = _unit_params(opt) if hasattr(buf, "all_units") else _flat_params(opt)
    model = getattr(engine._module, "model", None)
    mp = hcg.get_model_parallel_group() if hcg is not None else None
    out = {}
    for n, p, t in triples:
        if getattr(p, "tp_split", False) and mp is not None and mp.nranks > 1:
            parts = [torch.empty_like(t) for _ in range(mp.nranks)]
            dist.all_gather(parts, t.contiguous(), group=mp.group)
            t = torch.cat(parts, dim=getattr(p, "tp_dim", 0))
        out[canonical_name(n, hcg, model)] = t.cpu()
    if dist.is_initialized() and dist.get_world_size() > 1:
        mine = out if (hcg is None or (hcg.mp_rank == 0 and hcg.dp_rank == 0
                                       and hcg.sharding_rank == 0)) else {}
        allp = [None] * dist.get_world_size()
        dist.all_gather_object(allp, mine)
        out = {}
        for d in allp:
            out.update(d)
    return out

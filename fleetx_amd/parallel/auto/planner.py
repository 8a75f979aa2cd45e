"""Parallel-layout planner for GPT-style models on one MI355X node.

This is the "full" auto mode behind :class:`~fleetx_amd.core.engine.auto_engine.AutoEngine`
(reference P10/C11 leave layout choice to Paddle's auto-parallel completion;
here the search is explicit and hardware-specific).  It enumerates
``(dp, tp, pp, sharding stage, micro batch, recompute)`` for a world size and
scores each by an analytic step-time model under the 288 GB HBM budget:

* compute: model FLOPs / (n * sustained bf16 rate), x4/3 with full recompute;
* tensor parallel: 4 activation all-reduces (or RS+AG under SP) of
  ``b*s*h`` bf16 per layer per micro-batch.  xGMI is point-to-point — one
  link (~``LINK_GBPS`` per direction) per GPU pair — so a ring over ``t`` GPUs
  can drive at most ``t - 1`` links: TP-2 sees one link, TP-8 seven.  Half of
  it is hidden by the overlapped TP linears;
* pipeline: 1F1B bubble ``(pp-1)/(m+pp-1)`` plus boundary p2p;
* data parallel / ZeRO: bucketed gradient reduce(-scatter) overlapped with the
  backward (the last bucket is exposed) and, for ZeRO, the parameter
  all-gather after the optimizer step;
* memory: bf16 params + fp32 main grads + fp32 master/m/v (sharded per
  stage), activations ~``34*s*b*h/t`` bytes per layer with the flash kernel
  (``2*s*b*h`` with full recompute), plus the logits.

The constants are calibrated from measured single-GPU runs (profiles/).
"""
import itertools
import math
from dataclasses import asdict, dataclass

HBM_BYTES = 288e9
USABLE = 0.85            # leave room for the caching allocator / workspace
SUSTAINED_FLOPS = 1.16e15  # measured: 6.7B 1-GPU step, 293.7 ms (profiles/r4_full3)
# effective per-direction xGMI bandwidth per link: ~153 GB/s nominal x ~65 % RCCL
# efficiency (an assumption -- the development box has one GPU; recalibrate from
# SCALE_*.json once multi-GPU runs exist)
LINK_GBPS = 100e9
MAX_LINKS = 7            # each GPU has 7 links, one to every peer


@dataclass
class Plan:
    dp: int
    mp: int
    pp: int
    sharding: int
    sharding_stage: int
    micro_batch: int
    recompute: bool
    sequence_parallel: bool
    est_step_s: float
    est_mem_gb: float
    est_tokens_per_s: float

    def parallelism(self):
        parts = []
        if self.dp > 1:
            parts.append("dp%d" % self.dp)
        if self.sharding > 1:
            parts.append("sharding%d_stage%d" % (self.sharding, self.sharding_stage))
        if self.mp > 1:
            parts.append("tp%d" % self.mp)
        if self.pp > 1:
            parts.append("pp%d" % self.pp)
        return "_".join(parts) or "dp1"

    def as_dict(self):
        d = asdict(self)
        d["parallelism"] = self.parallelism()
        return d


def _ring_bw(n):
    return LINK_GBPS * min(max(n - 1, 1), MAX_LINKS)


def _allreduce_s(nbytes, n):
    return 0.0 if n <= 1 else 2.0 * (n - 1) / n * nbytes / _ring_bw(n)


def _rs_or_ag_s(nbytes, n):
    return 0.0 if n <= 1 else (n - 1) / n * nbytes / _ring_bw(n)


def model_params(h, L, V, s, ffn=None):
    ffn = ffn or 4 * h
    return L * (4 * h * h + 2 * h * ffn + 9 * h + ffn) + V * h + s * h + 2 * h


def flops_per_token(h, L, V, s):
    return 72.0 * L * h * h * (1 + s / (6.0 * h) + V / (12.0 * h * L))


def estimate(h, L, heads, V, s, global_batch, dp, mp, pp, sharding, stage, micro, recompute,
             sp=False):
    """Return (step seconds, peak bytes per GPU) or None when infeasible."""
    n = dp * mp * pp * sharding
    data = dp * sharding
    if global_batch % data or heads % mp or L % pp or V % mp:
        return None
    local = global_batch // data
    if local % micro:
        return None
    m = local // micro
    if pp > 1 and m < pp:
        return None
    P = model_params(h, L, V, s)
    p_local = P / (mp * pp)
    if stage >= 3 and pp > 1:
        return None  # ZeRO-3 does not compose with pipeline stages here
    # ---- memory
    layer = (12.0 * h * h) / mp
    grads = 4.0 * p_local
    if stage >= 2 and pp == 1:
        # owned fp32 shard + two layers of full fp32 grads in flight
        # (parallel/sharding.py); under pp > 1 stage 2 keeps the flat layout
        grads = 4.0 * p_local / sharding + 2 * 4.0 * layer
    opt = 12.0 * p_local / (sharding if stage >= 1 else 1)
    params = 2.0 * p_local
    if stage >= 3:  # shards + two layers of full params in flight
        params = 2.0 * p_local / sharding + 2 * 2.0 * layer
    layers_local = L // pp
    act_layer = (2.0 if recompute else 34.0 / mp) * s * micro * h
    in_flight = min(m, pp) if pp > 1 else 1  # 1F1B keeps <= pp micro-batches alive
    act = act_layer * layers_local * in_flight
    if recompute:
        act += 34.0 / mp * s * micro * h  # the layer being replayed
    logits = 6.0 * s * micro * V / mp  # bf16 logits + fp32 grad workspace
    mem = params + grads + opt + act + logits + 3e9
    if mem > HBM_BYTES * USABLE:
        return None
    # ---- time
    tokens_local = local * s
    # GEMM efficiency falls with the rows per micro-batch (calibrated at 8 x 1024)
    eff = (1.0 + 512.0 / 8192.0) / (1.0 + 512.0 / (micro * s))
    comp = flops_per_token(h, L, V, s) * tokens_local / (mp * pp) / (SUSTAINED_FLOPS * eff)
    if recompute:
        comp *= 4.0 / 3.0
    tp = 0.0
    if mp > 1:
        per = 2.0 * s * micro * h
        tp = 4 * layers_local * m * _allreduce_s(per, mp) * 0.5
    bubble = comp * (pp - 1) / (m + pp - 1) if pp > 1 else 0.0
    p2p = 2 * m * (2.0 * s * micro * h / mp) / LINK_GBPS if pp > 1 else 0.0
    gbytes = 4.0 * p_local
    bucket = min(gbytes, 256e6 * 4)
    if sharding > 1:
        # fp32 grad reduce-scatter overlaps backward (~60 % of compute); the bf16
        # parameter all-gather overlaps the next forward (~30 %); stage 3 gathers
        # every layer twice (forward + backward) under the layer compute
        rs = _rs_or_ag_s(gbytes, sharding)
        ag = _rs_or_ag_s(2.0 * p_local, sharding)
        if stage >= 2 and pp == 1:
            rs *= m  # stage 2/3 reduce-scatter every micro-batch's gradient
        grad = _rs_or_ag_s(bucket, sharding) + max(0.0, rs - comp * 0.6)
        grad += max(0.0, ag - comp * 0.3) if stage < 3 else max(0.0, 2 * ag - comp * 0.8)
    else:
        grad = 0.0
    if dp > 1:
        grad += _allreduce_s(bucket, dp) + max(0.0, _allreduce_s(gbytes, dp) - comp * 0.6)
    # optimizer: ~16 bytes read+written per local fp32 element at ~5 TB/s
    optim = 32.0 * p_local / (sharding if stage >= 1 else 1) / 5e12
    return comp + tp + bubble + p2p + grad + optim, mem


def plan(h, L, heads, V, s, global_batch, world, allow_recompute=True, prefer=None):
    """Best layout for ``world`` GPUs; ``prefer`` restricts to a dict of fixed degrees.
    ZeRO-3 is only considered when no stage-1/2 layout fits in HBM."""
    try:
        return _plan(h, L, heads, V, s, global_batch, world, allow_recompute, prefer, (1, 2))
    except ValueError:
        return _plan(h, L, heads, V, s, global_batch, world, allow_recompute, prefer, (1, 2, 3))


def _plan(h, L, heads, V, s, global_batch, world, allow_recompute, prefer, zero_stages):
    divs = [d for d in range(1, world + 1) if world % d == 0]
    cands = []
    for mp, pp in itertools.product(divs, divs):
        if world % (mp * pp):
            continue
        rest = world // (mp * pp)
        for sharding in [d for d in divs if rest % d == 0]:
            dp = rest // sharding
            stages = list(zero_stages) if sharding > 1 else [0]
            for stage, recompute in itertools.product(stages, [False, True]):
                if recompute and not allow_recompute:
                    continue
                cand = dict(dp=dp, mp=mp, pp=pp, sharding=sharding)
                if prefer and any(cand.get(k) != v for k, v in prefer.items() if k in cand):
                    continue
                data = dp * sharding
                if global_batch % data:
                    continue
                local = global_batch // data
                for micro in [d for d in range(1, local + 1) if local % d == 0]:
                    r = estimate(h, L, heads, V, s, global_batch, dp, mp, pp, sharding, stage,
                                 micro, recompute)
                    if r is None:
                        continue
                    t, mem = r
                    cands.append((t, stage, int(recompute), -micro, mem,
                                  Plan(dp, mp, pp, sharding, stage if sharding > 1 else 0,
                                       micro, recompute, False, t, mem / 1e9,
                                       global_batch * s / t)))
    if not cands:
        raise ValueError("no feasible layout for world={} within {:.0f} GB".format(
            world, HBM_BYTES * USABLE / 1e9))
    # layouts within 1 % of the fastest estimate are ties (the model is not
    # that precise): prefer the lower ZeRO stage, no recompute, the larger
    # micro-batch (fewer, larger GEMMs and launches), then less memory
    t_best = min(c[0] for c in cands)
    ties = [c for c in cands if c[0] <= t_best * 1.01]
    return min(ties, key=lambda c: c[1:5])[5]


def plan_from_config(cfg, world):
    m = cfg.Model
    s = cfg.Data.Train.dataset.get("max_seq_len", m.get("max_position_embeddings", 1024))
    gb = cfg.Global.get("global_batch_size") or cfg.Global.local_batch_size * world
    return plan(m.hidden_size, m.num_layers, m.num_attention_heads, m.vocab_size, s, gb, world,
                allow_recompute=True)


def describe(p):
    return ("plan: {par} micro={mb} recompute={rc} est {t:.3f}s/step, {tps:,.0f} tok/s, "
            "{mem:.0f} GB/GPU".format(par=p.parallelism(), mb=p.micro_batch, rc=p.recompute,
                                      t=p.est_step_s, tps=p.est_tokens_per_s, mem=p.est_mem_gb))


__all__ = ["Plan", "plan", "plan_from_config", "estimate", "describe", "model_params",
           "flops_per_token", "math"]

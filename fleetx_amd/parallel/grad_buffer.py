"""Flat parameter / gradient storage with bucketed, backward-overlapped
RCCL gradient reduction (data parallel + ZeRO stage 1/2 sharding).

Capability parity:
* P09 tensor fusion (``tensor_fusion_helper.py:36-127``: 256-byte aligned
  flat ``ParamStorage/GradStorage``, decay / no-decay split);
* P02 data parallel (Paddle ``DataParallel`` reducer: bucketed all-reduce
  overlapped with backward, ``fused_allreduce_gradients``);
* P06 sharding stage 1/2 gradient path (reduce-scatter to the owning rank);
* N09 coalesced mp all-reduce of sequence-parallel replicated grads;
* N11 tied-embedding grad all-reduce between first and last pipeline stage.
* ``reduce_dtype`` (``Distributed.comm.reduce_dtype``: float32 default,
  bfloat16 / float16 like the reference's fp16 gradient all-reduce) puts a
  16-bit copy of each bucket on the wire -- half the xGMI bytes -- and the
  result lands back in the fp32 gradient.

MI355X design:
* every trainable parameter becomes a VIEW into one model-dtype flat buffer
  and owns a ``main_grad`` view into one fp32 flat buffer; autograd's bf16
  ``.grad`` is folded into ``main_grad`` by a post-accumulate hook and freed,
  so gradient accumulation across micro-batches is exact fp32;
* parameters are grouped by category (weight-decay, tensor-parallel
  distributed, sequence-parallel, norm-excluded) so the optimizer, the grad
  norm and the SP all-reduce each see a handful of contiguous ranges (one
  kernel / one RCCL call per range, never per tensor);
* inside a category, parameters are laid out in reverse registration order
  (~ backward order) and cut into buckets of ``bucket_mb`` (default 256 MiB:
  few, large RCCL calls -- on xGMI a ring is per-link bandwidth bound, so a
  bucket must be large enough to amortise the ~10-20 us RCCL launch and
  protocol latency); a bucket's collective is launched asynchronously the
  moment its last gradient lands during the LAST micro-batch's backward, so
  communication overlaps the rest of backward on RCCL's stream.
"""
import math
import os

import torch
import torch.distributed as dist

from .linear import grad_part_done

ALIGN = 128  # elements (256 B in bf16, 512 B in fp32)


def _round_up(n, a):
    return (n + a - 1) // a * a


class Category:
    __slots__ = ("key", "start", "end", "params", "gview")

    def __init__(self, key):
        self.key = key
        self.start = self.end = 0
        self.params = []
        self.gview = None  # 16-bit gradient storage of a grad16 category

    @property
    def decay(self):
        return self.key[0]

    @property
    def distributed(self):
        return self.key[1]

    @property
    def seq_parallel(self):
        return self.key[2]

    @property
    def norm_excluded(self):
        return self.key[3]

    @property
    def grad16(self):
        """Gradient stored in the model's 16-bit dtype (``grad_dtype``)."""
        return len(self.key) > 4 and self.key[4]


class Bucket:
    __slots__ = ("start", "end", "params", "ready", "work", "launched", "shard_ranges",
                 "prescaled")

    def __init__(self, start, end, params):
        self.start, self.end, self.params = start, end, params
        self.ready = 0
        self.work = None
        self.launched = False
        self.prescaled = False  # 16-bit storage averaged before its collective


def _is_gloo(g):
    """gloo stand-ins for the RCCL collective forms; ``FLEETX_GLOO_AS_RCCL=1``
    disables them so CPU tests exercise the exact in-place reduce-scatter /
    all-gather-into-tensor code the GPU path runs."""
    if os.environ.get("FLEETX_GLOO_AS_RCCL", "0") == "1":
        return False
    try:
        return dist.get_backend(g.group) == "gloo"
    except Exception:
        return False


def grad16_eligible(p, fused_wgrad=True):
    """A weight whose whole gradient is ONE write of the weight-gradient GEMM
    (fused into main_grad, not a tied weight with a second part, not a
    sequence-parallel weight whose overlapped backward accumulates it chunk by
    chunk): its gradient can be stored in 16 bits straight from the GEMM's
    fp32 accumulators, rounded once."""
    return (p.dim() == 2 and fused_wgrad and bool(getattr(p, "_fx_fused_wgrad_ok", False))
            and bool(getattr(p, "_fx_gemm_wgrad", False))
            and getattr(p, "_fx_grad_parts", 1) == 1
            and not getattr(p, "_fx_grad_chunked", False))


def default_decay_fn(name, p):
    """Reference rule: no decay for biases and norm params (``optimizer.py:39-43``)."""
    if p.ndim < 2:
        return False
    return not any(nd in name for nd in ("bias", "norm"))


class FlatParamGradBuffer:
    """Owns flat param / fp32 grad storage and the gradient synchronisation."""

    def __init__(self, named_params, dp_group=None, shard_group=None, mp_group=None,
                 embed_group=None, bucket_mb=256, overlap=True, shard_stage=0,
                 decay_fn=default_decay_fn, reduce_dtype=torch.float32, fused_wgrad=True,
                 grad_dtype=torch.float32):
        named = [(n, p) for n, p in named_params if p.requires_grad]
        assert named, "no trainable parameters"
        self.dtype = named[0][1].dtype
        self.device = named[0][1].device
        self.dp_group = dp_group if dp_group is not None and dp_group.nranks > 1 else None
        self.shard_group = shard_group if shard_group is not None and shard_group.nranks > 1 else None
        self.mp_group = mp_group if mp_group is not None and mp_group.nranks > 1 else None
        self.embed_group = embed_group if embed_group is not None and embed_group.nranks > 1 else None
        self.shard_stage = shard_stage if self.shard_group is not None else 0
        self.overlap = overlap
        self.reduce_dtype = reduce_dtype
        # 16-bit gradient storage (Distributed.comm.grad_dtype; reference: the
        # O2 GradStorage in the parameter dtype, tensor_fusion_helper.py:56,72-74)
        # for the GEMM-written weight matrices, in the model dtype only (the
        # GEMM epilogue rounds its fp32 tile once per write); under ZeRO the
        # buckets reduce-scatter in 16 bits and each rank updates its owned
        # 16-bit chunk
        g16 = grad_dtype in (torch.bfloat16, torch.float16) and grad_dtype == self.dtype
        self.grad_dtype = grad_dtype if g16 else torch.float32

        cats = {}
        for n, p in reversed(named):
            key = (bool(decay_fn(n, p)), bool(getattr(p, "tp_split", False)),
                   bool(getattr(p, "sequence_parallel", False)),
                   bool(getattr(p, "norm_exclude", False)),
                   bool(g16 and grad16_eligible(p, fused_wgrad)))
            cats.setdefault(key, Category(key)).params.append((n, p))
        # deterministic category order: big decay/distributed region first
        order = sorted(cats.keys(), key=lambda k: (not k[0], not k[1], k[2], k[3], not k[4]))
        self.categories = [cats[k] for k in order]

        # shard padding: each category region is a multiple of ALIGN * nshard
        nsh = self.shard_group.nranks if self.shard_group is not None else 1
        off = 0
        self.offsets = {}
        for c in self.categories:
            c.start = off
            for n, p in c.params:
                self.offsets[id(p)] = (off, p.numel())
                off += _round_up(p.numel(), ALIGN)
            off = _round_up(off, ALIGN * nsh)
            c.end = off
        self.numel = off
        self.param_flat = torch.zeros(self.numel, dtype=self.dtype, device=self.device)
        self.grad_flat = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        # a grad16 category's gradients live in the first half of its own
        # fp32 region, reinterpreted as 16-bit (no extra memory; nothing reads
        # that region as fp32: every consumer goes through grad_slice)
        for c in self.categories:
            if c.grad16:
                n16 = c.end - c.start
                c.gview = self.grad_flat[c.start:c.end].view(self.grad_dtype)[:n16]
        self._cat_bounds = [(c.start, c.end, c) for c in self.categories]
        self.params = []
        for c in self.categories:
            for n, p in c.params:
                o, k = self.offsets[id(p)]
                view = self.param_flat[o:o + k].view_as(p)
                view.copy_(p.data)
                p.data = view
                p.main_grad = self.grad_slice(o, o + k).view_as(p)
                p.grad = None
                p._fx_fresh = True
                p._fx_fused_wgrad = bool(getattr(p, "_fx_fused_wgrad_ok", False)) and fused_wgrad
                self.params.append((n, p))

        # buckets: contiguous slices inside a category, capped at bucket_mb
        cap = max(ALIGN, int(bucket_mb * 1024 * 1024 // 4))
        self.buckets = []
        self._bucket_of = {}
        for c in self.categories:
            cur, cur_start, fill = [], c.start, 0
            for n, p in c.params:
                o, k = self.offsets[id(p)]
                if cur and fill + k > cap:
                    self._add_bucket(cur_start, o, cur)
                    cur, cur_start, fill = [], o, 0
                cur.append(p)
                fill += _round_up(k, ALIGN)
            if cur:
                self._add_bucket(cur_start, c.end, cur)
        if nsh > 1:
            for b in self.buckets:
                assert (b.end - b.start) % nsh == 0
        self._hooks = []
        self._accumulating = True
        self._last_micro = True
        self._norm_stream = None
        self._fused_norm = None
        self.early_norm = None
        self._install_hooks()

    # ------------------------------------------------------------------ storage
    def category_of(self, start):
        for s, e, c in self._cat_bounds:
            if s <= start < e:
                return c
        raise IndexError(start)

    def grad_slice(self, start, end):
        """Gradient elements [start, end) of the flat layout (inside one
        category) in their storage dtype: fp32 ``grad_flat`` or the 16-bit
        view of a grad16 category."""
        c = self.category_of(start)
        if c.gview is None:
            return self.grad_flat[start:end]
        assert end <= c.end
        return c.gview[start - c.start:end - c.start]

    # ------------------------------------------------------------------ setup
    def _add_bucket(self, start, end, params):
        nsh = self.shard_group.nranks if self.shard_group is not None else 1
        # pad bucket end so it splits evenly over sharding ranks (ranges are ALIGN aligned)
        b = Bucket(start, end, params)
        if nsh > 1 and (end - start) % nsh:
            raise RuntimeError("bucket not divisible by sharding degree")
        self.buckets.append(b)
        for p in params:
            self._bucket_of[id(p)] = b

    def _install_hooks(self):
        for n, p in self.params:
            self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(p)))
            p._fx_grad_ready = self._make_ready(p)

    def _make_ready(self, p):
        def ready():
            b = self._bucket_of[id(p)]
            b.ready += 1
            if b.ready == len(b.params) and self._last_micro and self.overlap:
                self._launch(b)
        return ready

    def _make_hook(self, p):
        def hook(param):
            g = param.grad
            if g is None:
                # fires with no grad when a fused-wgrad Function already wrote
                # main_grad and returned None: readiness was signalled there
                return
            if param._fx_fresh:
                param.main_grad.copy_(g)
            else:
                param.main_grad.add_(g)
            param._fx_fresh = False
            param._fx_sq_ok = False  # this write left no norm partials
            param.grad = None
            grad_part_done(param)
        return hook

    # ------------------------------------------------------------------ control
    def set_last_micro_batch(self, last):
        """Only the last micro-batch's backward launches the reductions."""
        self._last_micro = last
        for b in self.buckets:
            b.ready = 0

    def zero_grad(self):
        # no fill: the first gradient write of a step overwrites (beta = 0)
        for n, p in self.params:
            p._fx_fresh = True
        for b in self.buckets:
            b.ready = 0
            b.work = None
            b.launched = False

    # ------------------------------------------------------------------ early grad norm
    def enable_early_norm(self):
        """Sum of squares of each bucket as soon as it is final, on a side
        stream under the rest of backward (single data rank only: with data
        parallel / ZeRO the norm is over reduced, owned grads).  The optimizer
        reads ``early_norm`` instead of re-reading every gradient after
        backward (~4.6 ms for 6.7B on one MI355X)."""
        if self.device.type != "cuda" or self.dp_group is not None or \
                self.shard_group is not None or not self.overlap or self.embed_group is not None:
            return False
        if self.mp_group is not None and any(c.seq_parallel for c in self.categories):
            return False  # finish() all-reduces those grads over mp after the buckets
        from ..utils.streams import side_stream
        self._norm_stream = side_stream(self.device)
        self._norm_part = torch.zeros(len(self.buckets), dtype=torch.float32, device=self.device)
        self._bucket_index = {id(b): i for i, b in enumerate(self.buckets)}
        cat_of = []
        for b in self.buckets:
            c = next(c for c in self.categories if c.start <= b.start < c.end)
            cat_of.append(c)
        self._norm_dist_idx = torch.tensor(
            [i for i, c in enumerate(cat_of) if c.distributed and not c.norm_excluded],
            dtype=torch.long, device=self.device)
        self._norm_rep_idx = torch.tensor(
            [i for i, c in enumerate(cat_of) if not c.distributed and not c.norm_excluded],
            dtype=torch.long, device=self.device)
        return True

    def _early_norm_bucket(self, b):
        from ..optims.optimizer import _sumsq
        ev = torch.cuda.Event()
        ev.record()
        with torch.cuda.stream(self._norm_stream):
            self._norm_stream.wait_event(ev)
            i = self._bucket_index[id(b)]
            self._norm_part[i:i + 1].copy_(_sumsq(self.grad_slice(b.start, b.end)).reshape(1))

    def _finish_early_norm(self):
        """(distributed_sq, replicated_sq) device scalars, joined to the current stream."""
        torch.cuda.current_stream().wait_stream(self._norm_stream)
        part = self._norm_part
        self.early_norm = (part[self._norm_dist_idx].sum(), part[self._norm_rep_idx].sum())

    # ------------------------------------------------------------------ fused grad norm
    def enable_fused_norm(self):
        """Gradient-norm partials from the weight-gradient GEMM's epilogue.

        Every fused-wgrad matrix gets a region of fp32 slots that the
        hand-written GEMM's fp32 epilogue fills with sums of squares of the
        values it writes into ``main_grad`` (``ops.gemm.linear_wgrad(sq=)``;
        later micro-batches overwrite them with the accumulated values).  At
        ``finish()`` the norm is the sum of those slots plus one sum-of-squares
        pass over whatever they do not cover (embeddings, biases, norms, any
        weight whose gradient took another path this step) -- instead of
        re-reading the whole fp32 gradient (27 GB, 4.7 ms for 6.7B on one
        MI355X).  Single data rank only (with data parallel / ZeRO the norm is
        over reduced gradients); mutually exclusive with ``enable_early_norm``."""
        if self.device.type != "cuda" or self.dp_group is not None or \
                self.shard_group is not None or self._norm_stream is not None:
            return False
        if self.mp_group is not None and any(c.seq_parallel for c in self.categories):
            return False
        from ..ops import gemm as G
        self._fused_norm = {}
        for c in self.categories:
            if c.norm_excluded or c.seq_parallel:
                continue
            elig = [p for n, p in c.params if p.dim() == 2 and p._fx_fused_wgrad
                    and getattr(p, "_fx_gemm_wgrad", False)
                    and getattr(p, "_fx_grad_parts", 1) == 1]
            if not elig:
                continue
            sizes = [G.sq_slots(*p.shape) for p in elig]
            slots = torch.zeros(sum(sizes), dtype=torch.float32, device=self.device)
            o = 0
            for p, k in zip(elig, sizes):
                p._fx_sq = slots[o:o + k]
                p._fx_sq_ok = False
                o += k
            self._fused_norm[id(c)] = (slots, elig)
        return True

    _NORM_CHUNK = 1 << 18  # fp32 elements per block of the segmented sum of squares

    def _fused_norm_plan(self, okey):
        """(addr, len, n_dist) device tensors for one segmented sum-of-squares
        launch: the epilogue slots of covered weights and the gradient ranges
        of everything else, split into chunks, distributed (mp-sharded)
        chunks first."""
        chunks = {True: [], False: []}

        def add(t_addr, n, dist_, squared=False):
            # squared: the values are already sums of squares (epilogue slots)
            for o in range(0, n, self._NORM_CHUNK):
                m = min(self._NORM_CHUNK, n - o)
                chunks[dist_].append((t_addr + 4 * o, -m if squared else m))

        base = self.grad_flat.data_ptr()
        extra = {True: [], False: []}  # uncovered 16-bit gradients: summed by torch
        for c in self.categories:
            if c.norm_excluded:
                continue
            slots, elig = self._fused_norm.get(id(c), (None, ()))
            ok = {id(p) for p in elig if p._fx_sq_ok}
            if slots is not None and len(ok) == len(elig):
                add(slots.data_ptr(), slots.numel(), c.distributed, squared=True)
            else:
                for p in elig:
                    if id(p) in ok:
                        add(p._fx_sq.data_ptr(), p._fx_sq.numel(), c.distributed, squared=True)
            seg = None  # contiguous runs of uncovered parameters (padding is zero)

            def close(seg):
                if c.gview is not None:
                    extra[c.distributed].append(self.grad_slice(seg[0], seg[1]))
                else:
                    add(base + 4 * seg[0], seg[1] - seg[0], c.distributed)

            for n, p in c.params:
                o, k = self.offsets[id(p)]
                if id(p) in ok:
                    if seg is not None:
                        close(seg)
                        seg = None
                elif seg is None:
                    seg = [o, o + k]
                else:
                    seg[1] = o + k
            if seg is not None:
                close(seg)
        allc = chunks[True] + chunks[False]
        # host -> device through PINNED staging kept alive with the plan: a plan
        # first built inside a HIP-graph capture records the H2D copy, and
        # every replay re-reads its source (a freed pageable temporary would
        # feed the replays whatever the allocator put there since)
        host = torch.tensor([[a for a, _ in allc] or [0], [n for _, n in allc] or [0]],
                            dtype=torch.int64)
        if self.device.type == "cuda":
            host = host.pin_memory()
        dev = host.to(self.device, non_blocking=True)
        self._norm_plan_host = getattr(self, "_norm_plan_host", []) + [host]
        return dev[0], dev[1], len(allc), len(chunks[True]), extra

    def _finish_fused_norm(self):
        from ..ops import _lib
        okey = tuple(p._fx_sq_ok for slots, elig in self._fused_norm.values() for p in elig)
        cache = self.__dict__.setdefault("_norm_plans", {})
        plan = cache.get(okey)
        if plan is None:
            plan = cache[okey] = self._fused_norm_plan(okey)
        addr, lens, nch, nd, extra = plan
        part = torch.empty(max(nch, 1), dtype=torch.float32, device=self.device)
        if nch:
            _lib.kernels().sumsq_chunks(addr.data_ptr(), lens.data_ptr(), nch, part.data_ptr(),
                                        _lib.stream())
        zero = torch.zeros((), dtype=torch.float32, device=self.device)
        dist_sq = part[:nd].sum() if nd else zero
        rep_sq = part[nd:nch].sum() if nch > nd else zero
        from ..optims.optimizer import _sumsq  # 16-bit ranges: read in place
        for t in extra[True]:
            dist_sq = dist_sq + _sumsq(t)
        for t in extra[False]:
            rep_sq = rep_sq + _sumsq(t)
        self.early_norm = (dist_sq, rep_sq)

    def _data_groups(self):
        return self.dp_group, self.shard_group

    def _data_world(self):
        n = 1
        if self.dp_group is not None:
            n *= self.dp_group.nranks
        if self.shard_group is not None:
            n *= self.shard_group.nranks
        return n

    def _launch(self, b):
        if b.launched:
            return
        b.launched = True
        from .linear import join_wgrad_stream
        join_wgrad_stream()  # weight gradients computed on the side stream are final
        seg = self.grad_slice(b.start, b.end)
        works = []
        if self._norm_stream is not None:  # _launch only runs on final gradients
            self._early_norm_bucket(b)
        # wire copy in the reduce dtype only for fp32 storage reduced in 16 bits and only
        # when a collective runs; 16-bit gradient storage is reduced in place
        low = (self.reduce_dtype != seg.dtype and seg.dtype == torch.float32
               and (self.dp_group is not None or self.shard_group is not None))
        src = seg.to(self.reduce_dtype) if low else seg
        b.prescaled = False
        if seg.dtype != torch.float32 and self._data_world() > 1:
            # 16-bit gradient storage is reduced in place in 16 bits: average
            # BEFORE the sum (reference all_reduce_parameters scales the
            # fused 16-bit grad by 1/nranks first), so the 16-bit partial
            # sums stay at the gradient's own magnitude
            seg.mul_(1.0 / self._data_world())
            b.prescaled = True
        if self.shard_stage >= 1 and self.shard_group is not None:
            # reduce-scatter to the owner (in place: RCCL's recvbuff = sendbuff + rank*count);
            # dp all-reduce of the owned shard follows in finish()
            n = self.shard_group.nranks
            r = self.shard_group.rank
            chunk = (b.end - b.start) // n
            # the owned chunk in the storage dtype (16-bit buckets reduce-scatter
            # in 16 bits, in place, like the fp32 ones)
            out = self.grad_slice(b.start + r * chunk, b.start + (r + 1) * chunk)
            if _is_gloo(self.shard_group):
                works.append(dist.all_reduce(src, group=self.shard_group.group, async_op=True))
                wire = src[r * chunk:(r + 1) * chunk] if low else None
            elif low:
                wire = torch.empty(chunk, dtype=self.reduce_dtype, device=seg.device)
                works.append(dist.reduce_scatter_tensor(wire, src, group=self.shard_group.group,
                                                        async_op=True))
            else:
                wire = None
                works.append(dist.reduce_scatter_tensor(out, seg, group=self.shard_group.group,
                                                        async_op=True))
            b.work = ("rs", works, out, wire)
        else:
            grp = self.dp_group
            if grp is not None:
                works.append(dist.all_reduce(src, group=grp.group, async_op=True))
            b.work = ("ar", works, seg, src if (low and grp is not None) else None)

    def finish(self):
        """Complete every gradient collective; average over the data world."""
        from .linear import join_wgrad_stream
        join_wgrad_stream()
        for n, p in self.params:
            if p._fx_fresh:  # no gradient this step
                p.main_grad.zero_()
                p._fx_fresh = False
                p._fx_sq_ok = False
        for b in self.buckets:
            if not b.launched:
                self._launch(b)
        data_world = self._data_world()
        for b in self.buckets:
            kind, works, seg, wire = b.work
            for w in works:
                w.wait()
            if wire is not None:  # 16-bit reduction: back into the fp32 gradient
                seg.copy_(wire)
            if kind == "rs" and self.dp_group is not None:
                dist.all_reduce(seg, group=self.dp_group.group)
            if data_world > 1 and not b.prescaled:
                seg.mul_(1.0 / data_world)
        # sequence-parallel replicated params: one coalesced mp all-reduce per range
        if self.mp_group is not None:
            for c in self.categories:
                if c.seq_parallel:
                    dist.all_reduce(self.grad_slice(c.start, c.end), group=self.mp_group.group)
        # tied embedding between first and last pipeline stage
        if self.embed_group is not None:
            for n, p in self.params:
                if getattr(p, "shared_embedding", False):
                    dist.all_reduce(p.main_grad, group=self.embed_group.group)
        if self._norm_stream is not None:
            self._finish_early_norm()
        elif self._fused_norm is not None:
            self._finish_fused_norm()
        for b in self.buckets:
            b.launched = False
            b.work = None
            b.ready = 0

    # ------------------------------------------------------------------ sharding views
    def owned_ranges(self):
        """(start, end, category) ranges whose optimizer state this rank owns."""
        if self.shard_stage < 1 or self.shard_group is None:
            return [(c.start, c.end, c) for c in self.categories]
        n, r = self.shard_group.nranks, self.shard_group.rank
        out = []
        for c in self.categories:
            for b in self.buckets:
                if b.start >= c.start and b.end <= c.end:
                    chunk = (b.end - b.start) // n
                    out.append((b.start + r * chunk, b.start + (r + 1) * chunk, c))
        return out

    # -------------------------------------------------- overlapped parameter gather
    _ag_need = None

    def enable_param_gather_overlap(self, model):
        """ZeRO 1/2: issue the post-update parameter all-gathers asynchronously
        in FORWARD order and let each layer's forward pre-hook wait only for
        the buckets holding its parameters, so the gather (bf16 params, the
        only ZeRO traffic after the reduce-scatter that already overlaps
        backward) hides under the next forward instead of stalling after the
        optimizer step.  Returns False when there is nothing to overlap."""
        if self.shard_stage < 1 or self.shard_group is None:
            return False
        from .sharding import find_layer_units
        units = find_layer_units(model)
        owner = {}
        for i, m in enumerate(units):
            for p in m.parameters():
                owner.setdefault(id(p), i)
        need = {}
        first_use = []
        for bi, b in enumerate(self.buckets):
            us = [owner.get(id(p), -1) for p in b.params]
            for u in us:
                need.setdefault(u, set()).add(bi)
            first_use.append(min(us))
        self._ag_need = need
        self._ag_order = sorted(range(len(self.buckets)), key=lambda bi: first_use[bi])
        self._ag_works = {}
        self._hooks.append(model.register_forward_pre_hook(self._make_ag_wait(-1)))
        for i, m in enumerate(units):
            self._hooks.append(m.register_forward_pre_hook(self._make_ag_wait(i)))
        return True

    def _make_ag_wait(self, unit):
        def hook(module, args):
            if self._ag_works:
                for bi in self._ag_need.get(unit, ()):
                    e = self._ag_works.pop(bi, None)
                    if e is not None:
                        e[0].wait()
        return hook

    def sync_params(self):
        """Complete every outstanding overlapped parameter gather."""
        if self._ag_need is not None:
            for w, _ in self._ag_works.values():
                w.wait()
            self._ag_works = {}

    def gather_bucket_async(self, bi):
        """Issue bucket ``bi``'s parameter all-gather on the current stream
        (ordered after whatever that stream ran before, e.g. the bucket's
        update); the forward pre-hooks of the layers using it wait for it."""
        n, r = self.shard_group.nranks, self.shard_group.rank
        b = self.buckets[bi]
        chunk = (b.end - b.start) // n
        full = self.param_flat[b.start:b.end]
        mine = full[r * chunk:(r + 1) * chunk].clone()
        w = dist.all_gather_into_tensor(full, mine, group=self.shard_group.group, async_op=True)
        self._ag_works[bi] = (w, mine)  # keep the send buffer alive until waited

    def _allgather_async(self):
        self.sync_params()
        for bi in self._ag_order:
            self.gather_bucket_async(bi)

    def allgather_params(self):
        """After a sharded update, every rank gathers the full model-dtype params."""
        if self.shard_stage < 1 or self.shard_group is None:
            return
        if self._ag_need is not None:
            return self._allgather_async()
        n = self.shard_group.nranks
        r = self.shard_group.rank
        gloo = _is_gloo(self.shard_group)
        for b in self.buckets:
            chunk = (b.end - b.start) // n
            full = self.param_flat[b.start:b.end]
            mine = full[r * chunk:(r + 1) * chunk].clone()
            if gloo:
                parts = list(full.view(n, chunk).unbind(0))
                dist.all_gather(parts, mine, group=self.shard_group.group)
                full.copy_(torch.cat(parts))
            else:
                dist.all_gather_into_tensor(full, mine, group=self.shard_group.group)

    def remove_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []

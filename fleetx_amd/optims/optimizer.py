"""Optimizers over flat fp32 master buffers (multi-precision, fused).

Parity: reference ``FusedAdamW`` (``optimizer.py:29-50``: AdamW with
decoupled weight decay skipped for bias/norm params, ``multi_precision``
fp32 master weights, optional tensor fusion), re-exported ``Adam``,
``AdamW``, ``Momentum``; ``ClipGradByGlobalNorm`` (K13) and the GradScaler
path (K14) as used by ``eager_engine.py:425-445``.

MI355X design: the optimizer works on the ranges of a
:class:`~fleetx_amd.parallel.grad_buffer.FlatParamGradBuffer` -- master, m
and v are flat fp32 tensors, one HIP ``adamw_flat`` launch per range (a
handful per step, never one per parameter).  The global grad-norm is a
squared-sum kernel per range + (mp / pp / sharding) all-reduces of ONE float;
the clip coefficient and the fp16 found-inf flag stay on the device, so a
step never synchronises the host.
"""
import math
import os

import torch
import torch.distributed as dist

from ..ops import _lib


class ClipGradByGlobalNorm:
    def __init__(self, clip_norm=1.0, **kw):
        self.clip_norm = float(clip_norm)


class ClipGradByNorm(ClipGradByGlobalNorm):
    pass


def _sumsq(t):
    if t.dtype != torch.float32:  # 16-bit gradient storage (grad_dtype)
        if not t.is_cuda:
            return t.float().square().sum()
        k = _lib.kernels()
        blocks = k.sumsq_blocks(t.numel())
        part = torch.empty(blocks, device=t.device, dtype=torch.float32)
        k.sumsq_16(_lib.dt_code(t.dtype), t.data_ptr(), t.numel(), part.data_ptr(), blocks,
                   _lib.stream())
        return part.sum()
    if t.is_cuda:
        k = _lib.kernels()
        blocks = k.sumsq_blocks(t.numel())
        part = torch.empty(blocks, device=t.device, dtype=torch.float32)
        k.sumsq_f32(t.data_ptr(), t.numel(), part.data_ptr(), blocks, _lib.stream())
        return part.sum()
    return (t.float() * t.float()).sum()


_OFFLOAD_CHUNK = 1 << 25  # fp32 elements per streamed chunk (128 MiB per state tensor)


def _host_copy(src16):
    """fp32 pinned-host copy of a device range, converted chunk by chunk."""
    host = torch.empty(src16.numel(), dtype=torch.float32, pin_memory=True)
    for o in range(0, src16.numel(), _OFFLOAD_CHUNK):
        host[o:o + _OFFLOAD_CHUNK].copy_(src16[o:o + _OFFLOAD_CHUNK].float())
    return host


class FlatOptimizer:
    """Base: owns master/state for the owned ranges of a flat buffer."""

    def __init__(self, learning_rate, buffer, grad_clip=None, weight_decay=0.0,
                 multi_precision=True, check_group=None, pp_group=None, mp_group=None,
                 offload=False):
        self._lr = learning_rate
        self.buffer = buffer
        self.grad_clip = grad_clip
        self.weight_decay = float(weight_decay or 0.0)
        self.ranges = buffer.owned_ranges()
        self.mp_group = mp_group if mp_group is not None and mp_group.nranks > 1 else None
        self.pp_group = pp_group if pp_group is not None and pp_group.nranks > 1 else None
        self.step_count = 0
        dev = buffer.device
        # sharding_offload: fp32 state lives in pinned host memory (GPU runs only)
        self.offload = bool(offload) and dev.type == "cuda"
        if self.offload:
            self.master = [_host_copy(buffer.param_flat[s:e]) for s, e, _ in self.ranges]
        else:
            self.master = [buffer.param_flat[s:e].float().clone() for s, e, _ in self.ranges]
        self.found_inf = torch.zeros(1, dtype=torch.int32, device=dev)
        # number of APPLIED updates (advanced on the device only when found_inf
        # is 0): Adam's bias corrections follow it, so fp16 overflow steps do
        # not age the moments (Paddle's beta_pow semantics)
        self.dev_step = torch.zeros(1, dtype=torch.int32, device=dev)
        self.gscale = torch.ones(1, dtype=torch.float32, device=dev)
        self.last_grad_norm = torch.zeros((), dtype=torch.float32, device=dev)
        self.loss_scale = None  # set by the engine for fp16 (device tensor)

    # ------------------------------------------------------------------ master
    # Packed master (Optimizer.packed_master; bf16 models, device-resident
    # state): the fp32 master of each range is the bf16 parameter itself (its
    # high half, rounded on the low half) plus a 16-bit array of low halves,
    # joined exactly inside the AdamW kernel (loss_optim_embed.hip pk_decode).
    # The update moves 26 instead of 28 B per parameter (bf16 gradients) and
    # the master takes 2 instead of 4 B of HBM.  ``master`` decodes fp32
    # copies for checkpoints, tests and state gathers.
    _lo = None
    _master = None

    @property
    def master(self):
        if self._lo is None:
            return self._master
        return [self._join(ri) for ri in range(len(self.ranges))]

    @master.setter
    def master(self, value):
        self._master = value

    def _maybe_pack_master(self, want):
        pf = getattr(self.buffer, "param_flat", None)
        if not want or self.offload or pf is None or pf.device.type != "cuda" \
                or pf.dtype != torch.bfloat16 or self._master is None:
            return False
        self._lo = [torch.zeros(e - s, dtype=torch.int16, device=pf.device)
                    for s, e, _ in self.ranges]
        for (s, e, _), lo, m in zip(self.ranges, self._lo, self._master):
            _lib.kernels().pk_split(m.data_ptr(), pf[s:e].data_ptr(), lo.data_ptr(), e - s,
                                    _lib.stream())
        self._master = None  # the fp32 copies are gone: hi = the parameters, lo above
        return True

    def _join(self, ri):
        s, e, _ = self.ranges[ri]
        x = torch.empty(e - s, dtype=torch.float32, device=self._lo[ri].device)
        _lib.kernels().pk_join(self.buffer.param_flat[s:e].data_ptr(), self._lo[ri].data_ptr(),
                               x.data_ptr(), e - s, _lib.stream())
        return x

    def _mslice(self, ri, a, b):
        """The master storage of range ``ri`` [a, b) the kernel addresses:
        fp32 values, or (packed) the 16-bit low halves."""
        return (self._lo if self._lo is not None else self._master)[ri][a:b]

    def _set_master(self, ri, src):
        """Overwrite range ``ri``'s master (and, packed, its parameters) with fp32 ``src``."""
        if self._lo is None:
            self._master[ri].copy_(src)
            return
        s, e, _ = self.ranges[ri]
        x = src.to(device=self._lo[ri].device, dtype=torch.float32).contiguous()
        _lib.kernels().pk_split(x.data_ptr(), self.buffer.param_flat[s:e].data_ptr(),
                                self._lo[ri].data_ptr(), e - s, _lib.stream())

    # ------------------------------------------------------------------ lr
    def get_lr(self):
        return self._lr() if callable(self._lr) else float(self._lr)

    @property
    def lr_scheduler(self):
        return self._lr if hasattr(self._lr, "step") else None

    # ------------------------------------------------------------------ grads
    def grad_views(self):
        """Gradient of each owned range in its storage dtype (fp32, or the
        16-bit view of a ``grad_dtype`` category)."""
        gs = getattr(self.buffer, "grad_slice", None)
        if gs is not None:
            return [gs(s, e) for s, e, _ in self.ranges]
        g = self.buffer.grad_flat
        return [g[s:e] for s, e, _ in self.ranges]

    def _adamw_fn(self, g):
        """The fused AdamW launcher for a gradient of this storage dtype (and
        the packed master layout)."""
        k = _lib.kernels()
        if self._lo is not None:
            return k.adamw_flat_pk if g.dtype == torch.float32 else k.adamw_flat_pk_g16
        return k.adamw_flat if g.dtype == torch.float32 else k.adamw_flat_g16

    def compute_grad_norm(self):
        """Global L2 norm over the data/model-parallel world (device scalar)."""
        dev = self.buffer.device
        early = getattr(self.buffer, "early_norm", None)
        if early is not None:
            # per-bucket sums taken on a side stream during backward
            dist_sq, rep_sq = early
            self.buffer.early_norm = None
        else:
            dist_sq = torch.zeros((), dtype=torch.float32, device=dev)
            rep_sq = torch.zeros((), dtype=torch.float32, device=dev)
            for (s, e, c), g in zip(self.ranges, self.grad_views()):
                if c.norm_excluded:
                    continue
                sq = _sumsq(g)
                if c.distributed:
                    dist_sq = dist_sq + sq
                else:
                    rep_sq = rep_sq + sq
        err = getattr(self, "_comm_err", None)
        if err is not None:
            self._comm_err = None
            dist_sq = dist_sq + torch.where(err[0] != 0, float("inf"), 0.0)
        shard = self.buffer.shard_group if self.buffer.shard_stage >= 1 else None
        if shard is not None:
            pair = torch.stack([dist_sq, rep_sq])
            dist.all_reduce(pair, group=shard.group)
            dist_sq, rep_sq = pair[0], pair[1]
        if self.mp_group is not None:
            dist.all_reduce(dist_sq, group=self.mp_group.group)
        total = dist_sq + rep_sq
        if self.pp_group is not None:
            dist.all_reduce(total, group=self.pp_group.group)
        return torch.sqrt(total)

    def _prepare_scale(self):
        """Device-side clip coefficient x loss-scale unscale, and found-inf.

        A timed-out one-shot all-reduce (``parallel/comm.py``) counts as an
        overflow: with a norm, +inf joins the local sum of squares before the
        shard / mp / pp reductions; without one, the flag is the found-inf.
        The flag is MAX-reduced over the world first, so every rank skips."""
        from ..parallel import comm as _comm
        # a timeout is rank-local: shared with EVERY rank (MAX over the world)
        # so all ranks skip the step together instead of the ranks that did
        # not time out applying it alone
        err = _comm.world_error_flag()
        need_norm = self.grad_clip is not None or self.loss_scale is not None
        if not need_norm:
            self.gscale.fill_(1.0)
            if err is None:
                self.found_inf.zero_()
            else:
                self.found_inf.copy_((err != 0).to(torch.int32))
            return
        self._comm_err = err
        norm = self.compute_grad_norm()
        inv_scale = 1.0 / self.loss_scale if self.loss_scale is not None else 1.0
        true_norm = norm * inv_scale
        self.last_grad_norm = true_norm.detach()
        coef = torch.ones((), dtype=torch.float32, device=norm.device)
        if self.grad_clip is not None:
            coef = torch.clamp(self.grad_clip.clip_norm / (true_norm + 1e-6), max=1.0)
        self.gscale.copy_((coef * inv_scale).reshape(1))
        self.found_inf.copy_((~torch.isfinite(norm)).to(torch.int32).reshape(1))

    # ------------------------------------------------------------------ API
    def step(self):
        self._join_overlap()
        sync = getattr(self.buffer, "sync_params", None)
        if sync is not None:  # leftover overlapped parameter gathers of the last step
            sync()
        self._prepare_scale()
        self.step_count += 1
        self.dev_step.add_(1 - self.found_inf)
        if self.defer_update and self._overlap_groups is not None:
            self._pending = self.get_lr()  # launched by the next step (launch_pending)
        else:
            self._update(self.get_lr())
        if not self._overlap_gather:  # (else the overlapped update gathers bucket by bucket)
            self.buffer.allgather_params()

    # Whole-step graph mode (Engine.cuda_graph): the forward-overlapped update
    # of step N is launched at the START of step N+1's captured body, so one
    # replay holds both it and the forward it overlaps (a graph cannot wait
    # on work launched outside it).  Clip scale, found-inf and the Adam step
    # come from step N's device state; the learning rate from the device
    # buffer the engine copies at the end of each body.
    defer_update = False
    _pending = None

    def launch_pending(self, capturing=False):
        """Deferred mode: start the previous step's update on the side stream.

        ``capturing``: the call is being recorded into the whole-step graph,
        whose replays must ALWAYS hold the update launch -- even when a flush
        (``sync_state``: eval / save / predict) cleared ``_pending`` between
        the last eager call and the capture.  The launch reads its learning
        rate from the device buffer of the graph and, after a flush, the
        found-inf flag the flush raised, so the replay right after the capture
        is a no-op update and every later replay applies its step's update."""
        if self._pending is not None:
            lr, self._pending = self._pending, None
            self._update_overlapped(lr)
        elif capturing and self._overlap_groups is not None:
            self._update_overlapped(self.get_lr())

    # ------------------------------------------------------------------ overlap
    _overlap_groups = None
    overlap_grid = 128  # Distributed.comm.overlap_optimizer_grid
    overlap_wide = False  # Distributed.comm.overlap_optimizer_wide: 1024-thread blocks
    overlap_cus = 0  # Distributed.comm.overlap_optimizer_cus: CU-masked stream (0 = grid cap)

    def enable_forward_overlap(self, model):
        """Run the parameter update of step N on a side stream, unit by unit
        in FORWARD order, and let step N+1's forward start immediately: each
        layer's forward pre-hook waits only for ITS parameters' update.

        The update is HBM-bound (~30 B per parameter) while the forward is
        GEMM-bound, so the two share the GPU instead of serialising.  Needs
        device-resident state over an unsharded flat buffer (ZeRO stage 0);
        returns False (and changes nothing) otherwise."""
        from ..parallel.sharding import find_layer_units
        buf = self.buffer
        if not self._overlap_capable:
            # no side-stream update (Momentum): under ZeRO the serial update's
            # step() then issues the parameter all-gather itself
            return False
        if buf.device.type != "cuda" or self.offload or not hasattr(buf, "offsets"):
            return False
        if getattr(buf, "shard_stage", 0) != 0:
            return self._enable_sharded_overlap()
        units = find_layer_units(model)
        if not units:
            return False
        owner = {}
        for i, m in enumerate(units):
            for p in m.parameters():
                owner.setdefault(id(p), i)
        groups = {}
        for ri, (s, e, c) in enumerate(self.ranges):
            items = sorted((buf.offsets[id(p)][0], owner.get(id(p), -1)) for _, p in c.params)
            cur_u, lo = None, s
            for off, u in items:
                if cur_u is None:
                    cur_u = u
                elif u != cur_u:
                    groups.setdefault(cur_u, []).append((ri, lo, off))
                    cur_u, lo = u, off
            if cur_u is not None:
                groups.setdefault(cur_u, []).append((ri, lo, e))
        self._overlap_groups = [(u, groups[u]) for u in sorted(groups)]  # root (-1) first
        from ..utils.streams import cu_masked_stream, side_stream
        self._opt_stream = None
        if self.overlap_cus > 0:
            # pinned to a fixed CU set: the update may then fill those CUs
            # (no grid cap) while every other CU runs the forward undisturbed
            self._opt_stream = cu_masked_stream(buf.device, self.overlap_cus)
            if self._opt_stream is not None:
                self.overlap_grid = 0
        if self._opt_stream is None:
            self._opt_stream = side_stream(buf.device)
        self._unit_events = {}
        self._overlap_hooks = [model.register_forward_pre_hook(self._make_wait(-1))]
        for i, m in enumerate(units):
            self._overlap_hooks.append(m.register_forward_pre_hook(self._make_wait(i)))
        return True

    _overlap_gather = False
    # the subclass implements _update_overlapped (which also issues the ZeRO
    # parameter gathers when _overlap_gather is set)
    _overlap_capable = False

    def _enable_sharded_overlap(self):
        """ZeRO-1 (and stage 2 under pipeline parallelism, which keeps the
        flat buffer): the owned shard of each gradient bucket is updated on the
        side stream in the order the next forward first uses the buckets, and
        the bucket's parameter all-gather is issued on that stream right after
        its update -- so the update AND the gather hide under the next forward,
        whose layers already wait only for the gathers of their own buckets
        (``FlatParamGradBuffer.enable_param_gather_overlap``; reference: the
        stage-1 optimizer step then ``broadcast``/gather of
        ``dygraph_sharding_optimizer``, serial after backward).  Needs the
        overlapped parameter gather (not under pipeline schedules)."""
        buf = self.buffer
        if getattr(buf, "shard_stage", 0) not in (1, 2) or getattr(buf, "_ag_need", None) is None:
            return False
        bucket_of = {}
        for ri, (s, e, c) in enumerate(self.ranges):
            bi = next(i for i, b in enumerate(buf.buckets) if b.start <= s < b.end)
            bucket_of.setdefault(bi, []).append((ri, s, e))
        # every bucket is gathered, also those where this rank owns nothing
        self._overlap_groups = [(bi, [p for p in bucket_of.get(bi, []) if p[2] > p[1]])
                                for bi in buf._ag_order]
        self._overlap_gather = True
        from ..utils.streams import side_stream
        self._opt_stream = side_stream(buf.device)
        self._unit_events = {}
        self._overlap_hooks = []
        return True

    def _make_wait(self, unit):
        def hook(module, args):
            ev = self._unit_events.pop(unit, None)
            if ev is not None:
                torch.cuda.current_stream().wait_event(ev)
        return hook

    def wait_root_update(self):
        """Order the current stream after the overlapped update of the
        parameters outside every layer unit (pipeline schedules, whose model
        forward -- the root unit's hook -- never runs)."""
        if self._overlap_groups is not None:
            ev = self._unit_events.pop(-1, None)
            if ev is not None:
                torch.cuda.current_stream().wait_event(ev)

    def _join_overlap(self):
        """Order the current stream after every pending overlapped update."""
        if self._overlap_groups is not None:
            torch.cuda.current_stream().wait_stream(self._opt_stream)
            self._unit_events.clear()

    def clear_grad(self, set_to_zero=True):
        self.buffer.zero_grad()

    zero_grad = clear_grad

    def _update(self, lr):
        raise NotImplementedError

    def state_dict(self):
        raise NotImplementedError

    def set_state_dict(self, state):
        raise NotImplementedError

    def refresh_master_from_params(self):
        self.sync_state()
        if self._lo is not None:  # master = the parameters exactly: low halves 0
            for lo in self._lo:
                lo.zero_()
            return
        for (s, e, _), m in zip(self.ranges, self.master):
            m.copy_(self.buffer.param_flat[s:e].float())

    def sync_state(self):
        """Wait for the last update: host-offloaded D2H copies, or the
        forward-overlapped update stream (a deferred one is applied now)."""
        flushed = self._pending is not None
        if flushed:
            self.launch_pending()
        self._join_overlap()
        if self._overlap_gather:  # ZeRO: the gathers the overlapped update issued
            self.buffer.sync_params()
        if flushed:
            # a captured step launches this update again at its start: with
            # the skip flag set it leaves the applied update alone (the step's
            # own found-inf is recomputed after its backward).  Set only after
            # the join: the update itself reads the flag
            self.found_inf.fill_(1)
        cs = getattr(self, "_copy_stream", None)
        if cs is not None:
            cs.synchronize()


class FusedAdamW(FlatOptimizer):
    """AdamW (decoupled decay) with fp32 master weights, one launch per range."""

    decoupled = True
    _overlap_capable = True

    def __init__(self, learning_rate, buffer, grad_clip=None, weight_decay=0.01, beta1=0.9,
                 beta2=0.999, epsilon=1e-8, multi_precision=True, **kw):
        tensor_fusion = kw.pop("tensor_fusion", None)  # always fused here
        del tensor_fusion
        super().__init__(learning_rate, buffer, grad_clip, weight_decay, multi_precision,
                         kw.get("check_group"), kw.get("pp_group"), kw.get("mp_group"),
                         offload=kw.get("offload", False))
        self.beta1, self.beta2, self.eps = float(beta1), float(beta2), float(epsilon)
        self._maybe_pack_master(kw.get("packed_master", False))
        if self.offload:
            self.m = [torch.zeros(x.numel(), dtype=torch.float32, pin_memory=True)
                      for x in self.master]
            self.v = [torch.zeros(x.numel(), dtype=torch.float32, pin_memory=True)
                      for x in self.master]
            n = min(_OFFLOAD_CHUNK, max(e - s for s, e, _ in self.ranges))
            dev = buffer.device
            # two staging sets (master, m, v) so chunk j+1 uploads while j computes
            self._stage = [[torch.empty(n, dtype=torch.float32, device=dev) for _ in range(3)]
                           for _ in range(2)]
            self._copy_stream = torch.cuda.Stream(device=dev)
        else:
            dev = buffer.device
            self.m = [torch.zeros(e - s, dtype=torch.float32, device=dev) for s, e, _ in self.ranges]
            self.v = [torch.zeros(e - s, dtype=torch.float32, device=dev) for s, e, _ in self.ranges]

    def _update_overlapped(self, lr):
        """AdamW per unit (root first, then layer 0, 1, ...) on the side
        stream; an event per unit gates that unit's next forward."""
        k = _lib.kernels()
        pf = self.buffer.param_flat
        gf = self.buffer.grad_flat
        dt = _lib.dt_code(pf.dtype)
        os_ = self._opt_stream
        os_.wait_stream(torch.cuda.current_stream())  # grads final, clip scale computed
        # Cap the overlapped update's workgroups: uncapped it fills every CU and
        # the forward GEMMs queue behind it (the overlap then buys nothing);
        # with 128 workgroups it streams at ~2 TB/s beside the GEMMs and ends
        # with the forward (6.7B step -1.5..-1.8 % on two boxes,
        # profiles/r2_final/adamw_overlap_grid.txt).  0 = uncapped.
        grid = int(os.environ.get("FLEETX_ADAMW_OVERLAP_GRID", str(self.overlap_grid)))
        wide = int(os.environ.get("FLEETX_ADAMW_OVERLAP_WIDE", str(int(self.overlap_wide))))
        # non-temporal loads / stores (1, default: each byte is touched once per step)
        nt = int(os.environ.get("FLEETX_ADAMW_NT", "1"))
        # (running the first units -- embeddings, layer 0 -- uncapped because
        # they gate the first forward kernels measured neutral on 6.7B / 1.3B:
        # profiles/r3_adamw/head_ab.txt; every unit is capped)
        head = 0
        if getattr(self, "_overlap_args", None) is None:
            # launch arguments per unit, built once (the flat buffers never
            # move): the per-step host cost is then one bound call per range
            # -- on the 1.3B model slicing every view each step kept the GPU
            # waiting ~1.5 ms per step for the next forward
            units = []
            gviews = self.grad_views()
            for u, pieces in self._overlap_groups:
                args = []
                for ri, lo, hi in pieces:
                    s, e, c = self.ranges[ri]
                    a, b = lo - s, hi - s
                    g = gviews[ri][a:b]
                    wd = float(self.weight_decay if c.decay else 0.0)
                    # AdamW: decoupled decay; Adam: L2 term (as in _update)
                    wd_dec, l2 = (wd, 0.0) if self.decoupled else (0.0, wd)
                    args.append((self._adamw_fn(g), self._mslice(ri, a, b).data_ptr(), g.data_ptr(),
                                 self.m[ri][a:b].data_ptr(), self.v[ri][a:b].data_ptr(),
                                 pf[lo:hi].data_ptr(), hi - lo, wd_dec, l2))
                units.append((u, args))
            self._overlap_args = units
            self._overlap_dev = (self.gscale.data_ptr(), self.found_inf.data_ptr(),
                                 self.dev_step.data_ptr())
        gs, fi, ds = self._overlap_dev
        lr = float(lr)
        b1, b2, eps = self.beta1, self.beta2, self.eps
        with torch.cuda.stream(os_):
            st = _lib.stream()
            for i, (u, args) in enumerate(self._overlap_args):
                if grid and i == head:
                    k.adamw_tune(grid, nt, wide)
                for adamw, mp, gp, m1, v1, pp, n, wd, l2 in args:
                    adamw(dt, mp, gp, m1, v1, pp, n, lr, b1, b2, eps, wd, l2, gs, fi, ds, st)
                if self._overlap_gather:  # ZeRO: this bucket's gather follows its update
                    self.buffer.gather_bucket_async(u)
                    continue
                ev = torch.cuda.Event()
                ev.record(os_)
                self._unit_events[u] = ev
        if grid:
            k.adamw_tune(0, 1, 0)

    def _update_offloaded(self, lr):
        """Stream host-resident master/m/v through the GPU in chunks: the H2D
        copy of chunk j+1 and the D2H copy of chunk j-1 run on a copy stream
        while the fused AdamW kernel updates chunk j (reference
        ``group_sharded_parallel(offload=True)``, ``eager_engine.py:236-242``).
        PCIe traffic: 24 B per parameter per step."""
        k = _lib.kernels()
        cur = torch.cuda.current_stream()
        cs = self._copy_stream
        pf = self.buffer.param_flat
        gviews = self.grad_views()
        jobs = [(ri, o, min(_OFFLOAD_CHUNK, (e - s) - o))
                for ri, (s, e, _) in enumerate(self.ranges) for o in range(0, e - s, _OFFLOAD_CHUNK)]
        if not jobs:
            return
        cs.wait_stream(cur)  # gscale / found_inf / grads are final

        def upload(j):
            ri, o, n = jobs[j]
            with torch.cuda.stream(cs):
                for host, dev in zip((self.master[ri], self.m[ri], self.v[ri]), self._stage[j % 2]):
                    dev[:n].copy_(host[o:o + n], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(cs)
            return ev

        ready = upload(0)
        for j, (ri, o, n) in enumerate(jobs):
            nxt = upload(j + 1) if j + 1 < len(jobs) else None
            s, e, c = self.ranges[ri]
            wd = self.weight_decay if c.decay else 0.0
            st = self._stage[j % 2]
            cur.wait_event(ready)
            self._adamw_fn(gviews[ri])(_lib.dt_code(pf.dtype), st[0].data_ptr(),
                                       gviews[ri][o:o + n].data_ptr(),
                         st[1].data_ptr(), st[2].data_ptr(), pf[s + o:s + o + n].data_ptr(), n,
                         float(lr), self.beta1, self.beta2, self.eps, float(wd), 0.0,
                         self.gscale.data_ptr(), self.found_inf.data_ptr(),
                         self.dev_step.data_ptr(), _lib.stream())
            done = torch.cuda.Event()
            done.record(cur)
            with torch.cuda.stream(cs):
                cs.wait_event(done)
                for host, dev in zip((self.master[ri], self.m[ri], self.v[ri]), st):
                    host[o:o + n].copy_(dev[:n], non_blocking=True)
            ready = nxt

    def _update(self, lr):
        if self.offload:
            if not self.decoupled:
                raise NotImplementedError("sharding_offload supports the decoupled AdamW family")
            return self._update_offloaded(lr)
        if self._overlap_groups is not None:
            return self._update_overlapped(lr)
        pf = self.buffer.param_flat
        masters = [self._mslice(ri, 0, e - s) for ri, (s, e, _) in enumerate(self.ranges)]
        for (s, e, c), g, p, m, v in zip(self.ranges, self.grad_views(), masters, self.m,
                                         self.v):
            wd = self.weight_decay if c.decay else 0.0
            # AdamW: decoupled decay on the weights; Adam: L2 term added to the
            # gradient AFTER clipping / loss-scale unscaling
            wd_dec, l2 = (wd, 0.0) if self.decoupled else (0.0, wd)
            out16 = pf[s:e]
            if p.is_cuda:
                self._adamw_fn(g)(_lib.dt_code(pf.dtype), p.data_ptr(), g.data_ptr(),
                                          m.data_ptr(), v.data_ptr(), out16.data_ptr(), e - s,
                                          float(lr), self.beta1, self.beta2, self.eps,
                                          float(wd_dec), float(l2), self.gscale.data_ptr(),
                                          self.found_inf.data_ptr(), self.dev_step.data_ptr(),
                                          _lib.stream())
            else:
                if int(self.found_inf.item()):
                    continue
                t = int(self.dev_step.item())
                bc1 = 1.0 - self.beta1 ** t
                bc2 = 1.0 - self.beta2 ** t
                gg = g * self.gscale + l2 * p
                m.mul_(self.beta1).add_(gg, alpha=1 - self.beta1)
                v.mul_(self.beta2).addcmul_(gg, gg, value=1 - self.beta2)
                denom = v.sqrt() / math.sqrt(bc2) + self.eps
                p.mul_(1 - lr * wd_dec).addcdiv_(m, denom, value=-lr / bc1)
                out16.copy_(p)

    def state_dict(self):
        self.sync_state()
        cp = (lambda x: x.clone()) if self.offload else (lambda x: x.cpu())
        return {"step": self.step_count, "applied_step": int(self.dev_step.item()),
                "master": [cp(x) for x in self.master],
                "m": [cp(x) for x in self.m], "v": [cp(x) for x in self.v],
                "lr": self._lr.state_dict() if hasattr(self._lr, "state_dict") else self._lr}

    def set_state_dict(self, state):
        self.sync_state()
        self.step_count = state["step"]
        self.dev_step.fill_(int(state.get("applied_step", state["step"])))
        for ri, src in enumerate(state["master"]):
            self._set_master(ri, src)
        for dst, src in zip(self.m, state["m"]):
            dst.copy_(src)
        for dst, src in zip(self.v, state["v"]):
            dst.copy_(src)
        if hasattr(self._lr, "set_state_dict") and isinstance(state.get("lr"), dict):
            self._lr.set_state_dict(state["lr"])
        if self._lo is None:  # (packed: _set_master wrote the parameters)
            pf = self.buffer.param_flat
            for (s, e, _), p in zip(self.ranges, self.master):
                pf[s:e].copy_(p)


class AdamW(FusedAdamW):
    pass


class Adam(FusedAdamW):
    """Adam with classic (L2) weight decay added to the gradient."""
    decoupled = False


class Momentum(FlatOptimizer):
    def __init__(self, learning_rate, buffer, grad_clip=None, momentum=0.9, weight_decay=0.0,
                 use_nesterov=False, multi_precision=True, **kw):
        super().__init__(learning_rate, buffer, grad_clip, weight_decay, multi_precision,
                         kw.get("check_group"), kw.get("pp_group"), kw.get("mp_group"))
        self.momentum = float(momentum)
        self.nesterov = use_nesterov
        self.vel = [torch.zeros_like(x) for x in self.master]

    def _update(self, lr):
        skip = bool(self.found_inf.item()) if self.loss_scale is not None else False
        if skip:
            return
        pf = self.buffer.param_flat
        for (s, e, c), g, p, vel in zip(self.ranges, self.grad_views(), self.master, self.vel):
            gg = g * self.gscale
            if c.decay and self.weight_decay:
                gg = gg + self.weight_decay * p
            vel.mul_(self.momentum).add_(gg)
            upd = gg + self.momentum * vel if self.nesterov else vel
            p.add_(upd, alpha=-lr)
            pf[s:e].copy_(p)

    def state_dict(self):
        return {"step": self.step_count, "master": [x.cpu() for x in self.master],
                "vel": [x.cpu() for x in self.vel]}

    def set_state_dict(self, state):
        self.step_count = state["step"]
        for dst, src in zip(self.master, state["master"]):
            dst.copy_(src)
        for dst, src in zip(self.vel, state["vel"]):
            dst.copy_(src)
        pf = self.buffer.param_flat
        for (s, e, _), p in zip(self.ranges, self.master):
            pf[s:e].copy_(p)


OPTIMIZERS = {"FusedAdamW": FusedAdamW, "AdamW": AdamW, "Adam": Adam, "Momentum": Momentum}
CLIPS = {"ClipGradByGlobalNorm": ClipGradByGlobalNorm, "ClipGradByNorm": ClipGradByNorm}

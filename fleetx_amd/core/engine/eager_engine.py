"""EagerEngine: the train / eval / predict / save / load / export loop.

Parity: reference ``core/engine/eager_engine.py:41-738`` (C15).  Config keys
read: ``Engine.{run_mode, max_steps, num_train_epochs, eval_freq, eval_iters,
test_iters, logging_freq, accumulate_steps, mix_precision.*, save_load.*}``,
``Distributed.*``, ``Profiler.*``, ``Inference.*``.

MI355X-first differences:
* model parameters live in one flat bf16 buffer with fp32 ``main_grad``
  views (:mod:`fleetx_amd.parallel.grad_buffer`); DP / ZeRO gradient
  collectives are bucketed and launched from backward hooks, so they overlap
  with the rest of backward instead of the reference's post-backward
  ``fused_allreduce_gradients``;
* gradient accumulation (``local_batch_size / micro_batch_size``) works for
  every layout (the reference only accumulated under pipeline parallelism,
  SURVEY §2.12 #3);
* the host only synchronises at ``logging_freq`` (the reference synced and
  copied the loss every step, §2.12 #12);
* bf16 by default (no loss scaling); the fp16 path keeps a device-side
  dynamic loss scaler (init 32768, x2 every 1000 good steps, /2 on overflow);
* resume seeks the batch sampler via ``consumed_samples`` instead of reading
  and discarding batches (§2.12 #10), and restores the dropout RNG streams.
"""
import contextlib
import os
import sys
import time
import weakref

import numpy as np
import torch
import torch.distributed as dist

from .basic_engine import BasicEngine
from ...ops import _lib
from ...optims import build_optimizer, build_lr_scheduler
from ...parallel import comm as _comm
from ...parallel import topology as topo
from ...parallel.grad_buffer import FlatParamGradBuffer
from ...parallel.rng import get_rng_state_tracker
from ...utils import checkpoint as ckpt
from ...utils import env
from ...utils.log import logger
from ...utils.profiler import phase

_END = object()
_GRAPH_PTR_OWNER = [None]  # id of the engine whose device salt / lr pointers are registered


def _release_graph_ptrs(owner):
    if _GRAPH_PTR_OWNER[0] != owner:
        return
    _GRAPH_PTR_OWNER[0] = None
    try:
        k = _lib.kernels()
        k.set_dropout_salt(0)
        k.set_adamw_lr_ptr(0)
    except Exception:  # interpreter shutdown / library gone
        pass


class DynamicLossScaler:
    """Device-resident GradScaler (reference K14; ``eager_engine.py:157-167``).

    Paddle ``GradScaler`` semantics: the scale is multiplied by ``decr_ratio``
    only after ``decr_every_n_nan_or_inf`` CONSECUTIVE overflowing steps, and by
    ``incr_ratio`` after ``incr_every_n_steps`` consecutive finite ones."""

    def __init__(self, init_scale=32768.0, incr_every=1000, incr_ratio=2.0, decr_ratio=0.5,
                 decr_every=2, device="cpu"):
        self.scale = torch.full((), float(init_scale), dtype=torch.float32, device=device)
        self.good = torch.zeros((), dtype=torch.int32, device=device)
        self.bad = torch.zeros((), dtype=torch.int32, device=device)
        self.incr_every, self.incr_ratio, self.decr_ratio = incr_every, incr_ratio, decr_ratio
        self.decr_every = int(decr_every)

    def update(self, found_inf):
        """In place on the three device tensors (no host sync, no rebinding):
        the whole-step HIP graph captures this update and every replay must
        advance the SAME scale the next replay's backward multiplies by."""
        inf = found_inf.reshape(()).bool()
        zero = torch.zeros_like(self.good)
        good = torch.where(inf, zero, self.good + 1)
        bad = torch.where(inf, self.bad + 1, zero)
        grow = good >= self.incr_every
        shrink = bad >= self.decr_every
        self.scale.copy_(torch.where(shrink, self.scale * self.decr_ratio,
                                     torch.where(grow, self.scale * self.incr_ratio, self.scale)))
        self.good.copy_(torch.where(grow, zero, good))
        self.bad.copy_(torch.where(shrink, zero, bad))

    def state_dict(self):
        return {"scale": self.scale.cpu(), "good": self.good.cpu(), "bad": self.bad.cpu()}

    def load_state_dict(self, s):
        self.scale.copy_(s["scale"])
        self.good.copy_(s["good"])
        if "bad" in s:
            self.bad.copy_(s["bad"])


def _to_device(batch, device):
    if torch.is_tensor(batch):
        return batch.to(device, non_blocking=True)
    if isinstance(batch, (list, tuple)):
        return type(batch)(_to_device(b, device) for b in batch)
    if isinstance(batch, dict):
        return {k: _to_device(v, device) for k, v in batch.items()}
    return batch


def _split_micro(batch, n):
    if n == 1:
        return [batch]
    if torch.is_tensor(batch):
        assert batch.shape[0] % n == 0, "batch {} not divisible into {} micro-batches".format(
            batch.shape[0], n)
        return list(batch.chunk(n, dim=0))
    if isinstance(batch, (list, tuple)):
        parts = [_split_micro(b, n) for b in batch]
        return [type(batch)(p[i] for p in parts) for i in range(n)]
    return [batch] * n


def _safe_len(loader):
    try:
        return len(loader)
    except TypeError:
        return -1


class EagerEngine(BasicEngine):
    def __init__(self, configs, module, optimizer=None, lr=None, mode="train"):
        super().__init__()
        self.mode = mode
        self._configs = configs
        self._module = module
        e = configs.Engine
        self._run_mode = e.get("run_mode", "step")
        assert self._run_mode in ("epoch", "step"), "run_mode must be epoch or step"
        self._max_steps = e.get("max_steps", 1)
        self._eval_freq = e.get("eval_freq", 1) or 1
        self._eval_iters = e.get("eval_iters", 10)
        self._test_iters = e.get("test_iters", 100)
        self._logging_freq = e.get("logging_freq", 1) or 1
        self._num_train_epochs = e.get("num_train_epochs", 1)
        self._accumulate_steps = e.get("accumulate_steps", 1) or 1
        amp = e.get("mix_precision", {}) or {}
        self._use_pure_fp16 = bool(amp.get("use_pure_fp16", False))
        sl = e.get("save_load", {}) or {}
        self._save_steps = sl.get("save_steps", sys.maxsize)
        self._save_epoch = sl.get("save_epoch", 1)
        self._output_dir = sl.get("output_dir", "./output")
        self._ckpt_dir = sl.get("ckpt_dir")
        self._nan_guard = e.get("nan_guard", "off")
        self._metrics_file = e.get("metrics_file") or os.environ.get("FLEETX_METRICS_FILE")
        self._fault = os.environ.get("FLEETX_FAULT_INJECT")  # "rank:step" -> os._exit(17)
        # GEMM kinds on the MFMA kernel under FLEETX_GEMM=auto, per model
        # (the env var FLEETX_GEMM_AUTO wins): e.g. ViT-g's data gradients.
        # Always (re)set, so an engine without the key does not inherit the
        # routing of an earlier engine in the same process.
        from ...ops import gemm as _gemm
        routing = e.get("gemm_routing")
        _gemm.set_auto_kinds(routing if routing and "FLEETX_GEMM_AUTO" not in os.environ
                             else _gemm.default_auto_kinds())

        self.hcg = topo.get_hcg()
        self._dp_rank = self.hcg.dp_rank
        self._mp_rank, self._pp_rank = self.hcg.mp_rank, self.hcg.pp_rank
        self._sharding_rank = self.hcg.sharding_rank
        self._distributed = self.hcg.topo.world_size > 1
        sh = configs.Distributed.sharding
        self._sharding_stage = sh.get("sharding_stage", 1) if sh.get("sharding_degree", 1) > 1 else 0
        self.device = env.device()

        model = module.model
        from ...models.language_model.language_module import compute_dtype
        self._dtype = compute_dtype(configs)
        model.to(self.device)
        if mode == "export":
            self._dtype = torch.float32  # reference: pure fp16 disabled for export
        model.to(self._dtype)
        self._pipeline = hasattr(model, "train_batch")
        self._fused_head = bool(getattr(getattr(model, "cfg", None), "fused_lm_head_ce", False)) \
            and not self._pipeline

        self.buffer, self.optimizer, self.lr_scheduler = None, optimizer, lr
        self.scaler = None
        comm = configs.Distributed.get("comm", {}) or {}
        # TP / SP communication-compute overlap (parallel/linear.py, sp_overlap.py)
        from ...parallel import layers as _layers, sp_overlap as _spo
        _layers.TP_OVERLAP["enabled"] = bool(comm.get("tp_overlap", True))
        _layers.TP_OVERLAP["row_chunks"] = int(comm.get("tp_row_chunks", 2))
        _spo.SP_CHUNKS["chunks"] = int(comm.get("sp_chunks", 2))
        if mode == "train":
            sh_grp = self.hcg.get_sharding_parallel_group() if self._sharding_stage >= 1 else None
            red = {"float32": torch.float32, "bfloat16": torch.bfloat16,
                   "float16": torch.float16}[str(comm.get("reduce_dtype", "float32"))]
            if self._sharding_stage == 3 or (self._sharding_stage == 2 and self.hcg.pp_degree == 1):
                # reference: group_sharded_parallel(level='p_g_os' / 'os_g')
                # (eager_engine.py:228-242); stage 2 keeps whole parameters
                # but only the owned fp32 gradient shard
                from ...parallel.sharding import Stage3ParamGradBuffer
                assert self.hcg.pp_degree == 1, \
                    "sharding stage 3 does not compose with pipeline parallelism"
                self.buffer = Stage3ParamGradBuffer(
                    model, shard_group=sh_grp, dp_group=self.hcg.get_data_parallel_group(),
                    mp_group=self.hcg.get_model_parallel_group(),
                    prefetch=comm.get("stage3_prefetch", True), stage=self._sharding_stage,
                    reduce_dtype=red)
            else:
                # 16-bit gradient storage for the GEMM-written weight matrices
                # (reference O2: GradStorage in the parameter dtype,
                # tensor_fusion_helper.py:56,72-74): the weight-gradient GEMM
                # rounds its fp32 tile once per write and the update reads 2 B
                # instead of 4 per parameter; the data-parallel reduction then
                # runs in 16 bits, averaged first (grad_buffer._launch).
                # "auto": 16-bit models (bf16; fp16 O2, where the epilogue's
                # norm partials are of the stored fp16 values so an overflow
                # makes the norm non-finite and the scaler skips the step)
                # without ZeRO sharding; micro-batch accumulation and pipeline
                # schedules add each micro-batch into the 16-bit storage (one
                # fp32 add + one rounding per write, as the reference's 16-bit
                # GradStorage accumulates); under ZeRO-1 (and stage 2 with a
                # pipeline, which keeps this flat buffer) the buckets
                # reduce-scatter in 16 bits.  6.7B step on one MI355X: -4.4 ms
                # (profiles/r5_grad16/)
                gd = str(comm.get("grad_dtype", "auto"))
                if gd == "auto":
                    g16 = {torch.bfloat16: "bfloat16", torch.float16: "float16"}.get(self._dtype)
                    gd = g16 if g16 is not None else "float32"
                gdt = {"float32": torch.float32, "bfloat16": torch.bfloat16,
                       "float16": torch.float16}[gd]
                # stage 1 (and stage 2 under pipeline parallelism, where the
                # tied-embedding reduction needs the flat layout)
                self.buffer = FlatParamGradBuffer(
                    model.named_parameters(), dp_group=self.hcg.get_data_parallel_group(),
                    shard_group=sh_grp if sh_grp is not None
                    else self.hcg.get_sharding_parallel_group(),
                    mp_group=self.hcg.get_model_parallel_group(),
                    embed_group=self.hcg.get_embedding_group() if self.hcg.pp_degree > 1 else None,
                    bucket_mb=comm.get("dp_bucket_mb", 256),
                    overlap=comm.get("overlap_grad_reduce", True),
                    shard_stage=self._sharding_stage, reduce_dtype=red, grad_dtype=gdt)
            if self.lr_scheduler is None and "lr" in configs.Optimizer:
                self.lr_scheduler = build_lr_scheduler(configs.Optimizer.lr)
            self.optimizer = build_optimizer(configs.Optimizer, self.buffer, self.lr_scheduler,
                                             mp_group=self.hcg.get_model_parallel_group(),
                                             pp_group=self.hcg.get_pipe_parallel_group(),
                                             offload=bool(sh.get("sharding_offload", False)))
            if self._use_pure_fp16 and self._dtype == torch.float16:
                self.scaler = DynamicLossScaler(
                    amp.get("scale_loss", 32768.0),
                    incr_every=int(amp.get("incr_every_n_steps", 1000)),
                    incr_ratio=float(amp.get("incr_ratio", 2.0)),
                    decr_ratio=float(amp.get("decr_ratio", 0.5)),
                    decr_every=int(amp.get("decr_every_n_nan_or_inf", 2)),
                    device=self.device)
                self.optimizer.loss_scale = self.scaler.scale
            # weight-gradient GEMMs beside the data-gradient chain (parallel/linear.py;
            # only gemm5 launches go there: two library stream-K GEMMs in flight
            # on two streams can deadlock).  "auto" (default): models whose GEMMs
            # under-fill the chip (hidden <= 2048) outside whole-step graph mode
            # -- 1.3B 71.7 -> 70.3 ms; 345M in its graph 30.1 -> 30.6 ms, so off
            # there; profiles/r4_wgs/
            ws = comm.get("wgrad_stream", "auto")
            if ws == "auto":
                ws = configs.Model.get("hidden_size", 0) <= 2048 and \
                    not bool(e.get("cuda_graph", False))
            from ...parallel import linear as _lin
            _lin.WGRAD_STREAM["enabled"] = bool(ws) and self.device.type == "cuda" \
                and type(self.buffer) is FlatParamGradBuffer
            # whole-step HIP graph (Engine.cuda_graph): one replay per step
            self._cuda_graph = bool(e.get("cuda_graph", False)) and self._graph_ok(comm)
            self._graph = None
            self._graph_calls = 0
            # step N's AdamW runs on a side stream under step N+1's forward (also
            # with the fp16 loss scaler: its found-inf / scale live on the device
            # and the next step() joins the side stream before rewriting them)
            # (in whole-step graph mode the update is deferred into the next
            # step's captured body: FlatOptimizer.launch_pending)
            # (under pipeline parallelism too: the stage's decoder layers wait
            # for their own units in their forward pre-hooks, the rest of the
            # stage -- embedding, final LN, head -- before the schedule starts,
            # _fit_impl)
            # ZeRO-1/2: the post-update parameter all-gather hides under the next forward
            # (and, with overlap_optimizer, the owned shard's update before it)
            if comm.get("overlap_param_gather", True) and not self._pipeline \
                    and hasattr(self.buffer, "enable_param_gather_overlap"):
                self.buffer.enable_param_gather_overlap(model)
            if comm.get("overlap_optimizer", True) \
                    and hasattr(self.optimizer, "enable_forward_overlap"):
                self.optimizer.overlap_grid = int(comm.get("overlap_optimizer_grid", 128))
                self.optimizer.overlap_cus = int(comm.get("overlap_optimizer_cus", 0) or 0)
                if self.optimizer.enable_forward_overlap(model) and self._cuda_graph:
                    self.optimizer.defer_update = True
                    # uncapped in the graph for hidden <= 1024 (345M: 29.07-29.28
                    # ms vs 29.20-29.58 at the 128-workgroup cap, serial
                    # 29.27-29.32; profiles/r4_defer/); larger models keep the
                    # cap (6.7B 293.7-294.4 ms at 128 vs 297.0-298.7 uncapped,
                    # 64: 306.8, 192: 297.3-298.7; 1.3B 70.4-70.5 vs 71.4;
                    # profiles/r4_g67/)
                    small = configs.Model.get("hidden_size", 0) <= 1024
                    self.optimizer.overlap_grid = int(comm.get("overlap_optimizer_grid",
                                                               0 if small else 128))
            # single data rank: gradient sum-of-squares per bucket under backward
            # (opt-in: measured neutral on 6.7B, the GEMMs leave no CU slots free)
            if comm.get("early_grad_norm", False) and not self._pipeline and not self._cuda_graph \
                    and hasattr(self.buffer, "enable_early_norm"):
                self.buffer.enable_early_norm()
            # otherwise the weight-gradient GEMMs hand the norm their sums of
            # squares (no second pass over the gradient at step end); under the
            # fp16 loss scaler the partials are of the stored fp16 values, so
            # an overflow makes the norm non-finite (tests/test_fp16_gpu.py:
            # graph replay bitwise the eager step across an overflowed step)
            elif comm.get("fused_grad_norm", True) \
                    and hasattr(self.buffer, "enable_fused_norm") \
                    and getattr(self.optimizer, "grad_clip", None) is not None:
                self.buffer.enable_fused_norm()
            if self._pipeline:
                model.attach(self)
            if self.device.type == "cuda":
                from ...utils.streams import log_inventory
                log_inventory(self.hcg, self.optimizer, self.buffer,
                              _lin.WGRAD_STREAM["enabled"])
        self._profiler = self._build_profiler(configs.get("Profiler"))
        self._inference_engine = None
        self.consumed_samples = 0
        if mode == "inference":
            inf = configs.get("Inference", {}) or {}
            self._inference_model_dir = inf.get("model_dir", self._output_dir)

    # ------------------------------------------------------------------ profiler
    def _build_profiler(self, pcfg):
        if not pcfg or not pcfg.get("enable", False):
            return None
        from ...utils.profiler import Profiler
        return Profiler(pcfg)

    # ------------------------------------------------------------------ train
    def _fault_check(self, step):
        # only the first launch attempt faults, so a launcher restart can finish
        if self._fault and os.environ.get("FLEETX_RESTART_COUNT", "0") == "0":
            r, s = self._fault.split(":")
            if int(r) == env.get_rank() and int(s) == step:
                logger.error("fault injection: rank %s exits at step %s" % (r, s))
                os._exit(17)

    # ------------------------------------------------------------------ HIP graph
    def _graph_ok(self, comm):
        """Whole-step capture needs a single-rank, non-pipelined step with
        device-resident optimizer state (no host syncs).  The fp16 dynamic
        loss scaler qualifies: scale, counters and found-inf stay on the
        device and are updated in place (DynamicLossScaler.update)."""
        why = None
        if not torch.cuda.is_available() or self.device.type != "cuda":
            why = "no GPU"
        elif self._distributed:
            why = "multi-rank runs keep eager collectives"
        elif self._pipeline:
            why = "pipeline schedules run eagerly"
        elif self.scaler is not None and not hasattr(self.optimizer, "_update_overlapped"):
            why = "%s reads found-inf on the host" % type(self.optimizer).__name__
        elif getattr(self.optimizer, "offload", False):
            why = "offloaded optimizer state"
        if why is not None:
            logger.warning("Engine.cuda_graph disabled: %s" % why)
            return False
        return True

    def _graph_setup(self):
        k = _lib.kernels()
        self._graph_salt = torch.full((1,), getattr(self, "_graph_salt_resume", 0),
                                      dtype=torch.int64, device=self.device)
        self._graph_lr = torch.zeros(1, dtype=torch.float32, device=self.device)
        # deferred update (optimizer.defer_update): it runs one step later and
        # reads the learning rate of its own step, copied here by each body
        self._graph_lr_pending = torch.zeros(1, dtype=torch.float32, device=self.device)
        k.set_dropout_salt(self._graph_salt.data_ptr())
        k.set_adamw_lr_ptr((self._graph_lr_pending if self._defer_update() else
                            self._graph_lr).data_ptr())
        # the kernels read these process-global device pointers: clear them when
        # this engine goes away (unless a newer engine has taken them over), so
        # a later engine / optimizer never reads freed memory
        _GRAPH_PTR_OWNER[0] = id(self)
        weakref.finalize(self, _release_graph_ptrs, id(self))

    def _defer_update(self):
        return bool(getattr(self.optimizer, "defer_update", False))

    def _graph_body(self, batch):
        """The device work of one step: fresh dropout salt, forward, backward,
        gradient finish, clip + AdamW, gradient reset.  With the deferred
        overlapped update the previous step's AdamW starts first, on the side
        stream, under this step's forward."""
        defer = self._defer_update()
        if defer:
            self.optimizer.launch_pending(capturing=torch.cuda.is_current_stream_capturing())
        self._graph_salt.add_(1)
        model = self._module.model
        model.train()
        micro = _split_micro(batch, self._accumulate_steps)
        loss = None
        for i, mb in enumerate(micro):
            self.buffer.set_last_micro_batch(i == len(micro) - 1)
            self._declare_head_grad()
            l = self._module.training_step(mb)
            if self._accumulate_steps > 1:
                l = l / self._accumulate_steps
            self._module.backward(l * self.scaler.scale if self.scaler is not None else l)
            loss = l.detach() if loss is None else loss + l.detach()
        self.buffer.finish()
        self.optimizer.step()
        if self.scaler is not None:
            # device-side GradScaler step (in place: the captured graph advances
            # the same scale / counters every replay)
            self.scaler.update(self.optimizer.found_inf)
        self.optimizer.clear_grad()
        if defer:
            self._graph_lr_pending.copy_(self._graph_lr)
        return loss

    def _graph_batch_matches(self, batch):
        if len(batch) != len(self._graph_static):
            return False
        for a, b in zip(self._graph_static, batch):
            if torch.is_tensor(a) != torch.is_tensor(b):
                return False
            if torch.is_tensor(a) and (a.shape != b.shape or a.dtype != b.dtype):
                return False
        return True

    def _fit_graphed(self, batch, warmup=2):
        """Capture the whole training step into one HIP graph after ``warmup``
        eager steps (same kernels, same device-side salt / lr), then replay it.
        Dropout draws new masks every replay (device salt); the learning rate
        is written to the device before each replay; host bookkeeping
        (scheduler, step counter) runs outside the graph."""
        if self._graph_calls == 0:
            self._graph_setup()
        self._graph_calls += 1
        self._graph_lr.fill_(float(self.optimizer.get_lr()))
        if self._graph is None and self._graph_calls <= warmup:
            loss = self._graph_body(batch)
        elif self._graph is None:
            torch.cuda.synchronize()
            self._graph_static = [t.clone() if torch.is_tensor(t) else t for t in batch]
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._graph_loss = self._graph_body(self._graph_static)
            self._graph = g
            g.replay()  # the capture itself does not execute the step
            loss = self._graph_loss.clone()
        elif not self._graph_batch_matches(batch):
            # a batch of another shape (e.g. a short last batch): run it eagerly
            # with the same device-side salt / lr; the graph stays for the rest
            loss = self._graph_body(batch)
        else:
            for dst, src in zip(self._graph_static, batch):
                if torch.is_tensor(dst):
                    dst.copy_(src, non_blocking=True)
            self._graph.replay()
            self.optimizer.step_count += 1  # the captured step() ran its host part once
            if self._defer_update():
                self.optimizer._pending = self.optimizer.get_lr()  # this replay's update
            # the captured loss is one static tensor that every replay rewrites:
            # hand out a copy (fit() accumulates it across steps)
            loss = self._graph_loss.clone()
        if self.lr_scheduler is not None and hasattr(self.lr_scheduler, "step"):
            self.lr_scheduler.step()
        return loss

    def _fit_impl(self, batch):
        if getattr(self, "_cuda_graph", False):
            return self._fit_graphed(batch)
        model = self._module.model
        model.train()
        if self._pipeline:
            # the stage's parameters outside its decoder layers (embedding,
            # final LN, LM head) are the update's root unit, launched first:
            # the schedule never calls the model's own forward, whose
            # pre-hook waits for it otherwise
            wait_root = getattr(self.optimizer, "wait_root_update", None)
            if wait_root is not None:
                wait_root()
            loss = model.train_batch(self._module.pretreating_batch(batch), self._accumulate_steps)
        else:
            micro = _split_micro(batch, self._accumulate_steps)
            loss = None
            for i, mb in enumerate(micro):
                self.buffer.set_last_micro_batch(i == len(micro) - 1)
                with phase("Forward"):
                    self._declare_head_grad()
                    l = self._module.training_step(mb)
                    if self._accumulate_steps > 1:
                        l = l / self._accumulate_steps
                with phase("Backward"):
                    self._module.backward(l * self.scaler.scale if self.scaler is not None else l)
                loss = l.detach() if loss is None else loss + l.detach()
        with phase("GradSync"):
            self.buffer.finish()
        with phase("Optimization"):
            self._optim_update()
        return loss

    def _declare_head_grad(self):
        """Fused LM-head cross-entropy (``Model.fused_lm_head_ce``): the head's
        backward runs inside the forward, so the gradient the loss will
        receive -- 1 / accumulation steps x the fp16 loss scale -- is
        declared before each micro-batch (ops/lm_head_ce.py)."""
        if self._fused_head:
            from ...ops import lm_head_ce
            lm_head_ce.declare_grad_scale(self.scaler.scale if self.scaler is not None else None,
                                          self._accumulate_steps)

    def _optim_update(self):
        self.optimizer.step()
        if self.scaler is not None:
            self.scaler.update(self.optimizer.found_inf)
            self.optimizer.loss_scale = self.scaler.scale
        if self.lr_scheduler is not None and hasattr(self.lr_scheduler, "step"):
            self.lr_scheduler.step()
        self.optimizer.clear_grad()

    def _current_lr(self):
        return self.optimizer.get_lr() if self.optimizer is not None else 0.0

    def fit(self, epoch=1, train_data_loader=None, valid_data_loader=None):
        assert self.mode == "train"
        start_epoch = getattr(self, "_load_recovery", {}).get("epoch", 0)
        start_step = getattr(self, "_load_recovery", {}).get("step", 0)
        if self._profiler:
            self._profiler.start()
        global_step = start_step
        for ep in range(start_epoch, epoch if self._run_mode == "epoch" else max(epoch, 1)):
            sampler = getattr(train_data_loader, "batch_sampler", None)
            if sampler is not None and hasattr(sampler, "set_epoch"):
                sampler.set_epoch(ep, self.consumed_samples if ep == start_epoch else 0)
            t_epoch = time.time()
            global_step, done = self._train_one_epoch(ep, train_data_loader, valid_data_loader,
                                                      global_step)
            self._module.training_epoch_end({"epoch": ep, "train_cost": time.time() - t_epoch})
            if self._run_mode == "epoch" and valid_data_loader is not None and \
                    (ep + 1) % self._eval_freq == 0:
                self._evaluate_impl(ep, valid_data_loader, None)
            if self._run_mode == "epoch" and (ep + 1) % self._save_epoch == 0:
                self.save(epoch=ep + 1, step=global_step)
            if done:
                break
        if self._profiler:
            self._profiler.stop()
        if getattr(self.optimizer, "sync_state", None) is not None:
            self.optimizer.sync_state()  # the last (overlapped / deferred) update lands
        if torch.cuda.is_available():
            torch.cuda.synchronize()
            _comm.check_all()
        return global_step

    def _train_one_epoch(self, epoch, loader, valid_loader, global_step):
        gbs = self._configs.Global.global_batch_size
        total = _safe_len(loader)
        loss_acc, n_acc = None, 0
        t0 = time.time()
        it = iter(loader)
        while True:
            with phase("Dataloader"):
                batch = next(it, _END)
                if batch is _END:
                    break
                batch = _to_device(batch, self.device)
            self._fault_check(global_step)
            loss = self._fit_impl(batch)
            global_step += 1
            self.consumed_samples += gbs
            if loss is not None:
                loss_acc = loss if loss_acc is None else loss_acc + loss
                n_acc += 1
            if global_step % self._logging_freq == 0:
                if torch.cuda.is_available():
                    torch.cuda.synchronize()
                    # a one-shot all-reduce that timed out on a peer wrote NaN
                    # and flagged it: stop here, naming the group
                    _comm.check_all()
                if self._fused_head:
                    from ...ops import lm_head_ce
                    lm_head_ce.check()
                cost = (time.time() - t0) / self._logging_freq
                lval = self._reduce_log_loss(loss_acc, n_acc)
                if self._nan_guard != "off" and not np.isfinite(lval):
                    msg = "non-finite loss at step %d" % global_step
                    if self._nan_guard == "abort":
                        raise FloatingPointError(msg)
                    logger.warning(msg)
                self._module.training_step_end({"epoch": epoch, "batch": global_step, "loss": lval,
                                                "train_cost": cost, "lr": self._current_lr(),
                                                "total_batch": total})
                self._write_metrics(epoch, global_step, lval, cost)
                loss_acc, n_acc = None, 0
                t0 = time.time()
            if self._run_mode == "step" and valid_loader is not None and \
                    global_step % self._eval_freq == 0:
                self._evaluate_impl(epoch, valid_loader, self._eval_iters)
                t0 = time.time()
            if self._run_mode == "step" and global_step % self._save_steps == 0:
                self.save(epoch=epoch, step=global_step)
            if self._profiler:
                self._profiler.step()
            if self._run_mode == "step" and global_step >= self._max_steps:
                return global_step, True
        return global_step, False

    def _write_metrics(self, epoch, step, loss, step_time):
        """Optional JSONL metrics sink (``Engine.metrics_file``):
        one record per logging window from global rank 0 (the loss is already
        broadcast from the last pipeline stage)."""
        if not self._metrics_file or env.get_rank() != 0:
            return
        import json
        rec = {"time": round(time.time(), 3), "epoch": epoch, "step": step, "loss": loss,
               "lr": self._current_lr(), "step_time_s": round(step_time, 6),
               "consumed_samples": self.consumed_samples}
        if self.optimizer is not None and getattr(self.optimizer, "last_grad_norm", None) is not None:
            rec["grad_norm"] = float(self.optimizer.last_grad_norm)
        tokens = getattr(self._module, "tokens_per_step", None)
        if callable(tokens):
            rec["tokens_per_s"] = round(tokens() / max(step_time, 1e-9), 1)
        if torch.cuda.is_available():
            rec["max_mem_gb"] = round(torch.cuda.max_memory_allocated() / 2 ** 30, 2)
        d = os.path.dirname(os.path.abspath(self._metrics_file))
        os.makedirs(d, exist_ok=True)
        with open(self._metrics_file, "a") as f:
            f.write(json.dumps(rec) + "\n")

    def _reduce_log_loss(self, loss_acc, n):
        """Loss for the log line: mean over the window; under PP it lives on
        the last stage and is broadcast to all stages."""
        if loss_acc is None:
            v = torch.zeros((), device=self.device)
        else:
            v = (loss_acc / max(n, 1)).float()
        if self.hcg.pp_degree > 1:
            g = self.hcg.get_pipe_parallel_group()
            src = g.ranks[-1]
            v = v.clone()
            dist.broadcast(v, src=src, group=g.group)
        return float(v.item())

    # ------------------------------------------------------------------ eval
    @torch.no_grad()
    def _evaluate_impl(self, epoch, loader, iters):
        self._flush_deferred_update()
        model = self._module.model
        model.eval()
        outs = []
        total = _safe_len(loader)
        t0 = t_start = time.time()
        for i, batch in enumerate(loader):
            if iters is not None and i >= iters:
                break
            batch = _to_device(batch, self.device)
            if self._pipeline:
                loss = model.eval_batch(self._module.pretreating_batch(batch))
            else:
                loss = self._module.validation_step(batch)
            outs.append(loss)
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            cost = time.time() - t0
            if (i + 1) % self._logging_freq == 0:
                if self._pipeline:
                    # the loss lives on the last stage: broadcast it to every stage
                    lval = self._reduce_log_loss(loss, 1)
                else:
                    lval = float(loss.float().item()) if torch.is_tensor(loss) else loss
                self._module.validation_step_end({"epoch": epoch, "batch": i, "loss": lval,
                                                  "eval_cost": cost / self._logging_freq,
                                                  "total_batch": total})
                t0 = time.time()
        self._module.validation_epoch_end({"epoch": epoch, "eval_cost": time.time() - t_start})
        model.train()
        return outs

    def _flush_deferred_update(self):
        if getattr(self, "optimizer", None) is not None and self._defer_update():
            self.optimizer.sync_state()  # the last step's update has not started yet

    def evaluate(self, epoch=1, valid_data_loader=None):
        self._flush_deferred_update()
        model = self._module.model
        model.eval()
        outs = []
        total = _safe_len(valid_data_loader)
        t0 = t_start = time.time()
        with torch.no_grad():
            for i, batch in enumerate(valid_data_loader):
                batch = _to_device(batch, self.device)
                out = self._module.validation_step(batch)
                self._module.validation_step_end({"epoch": epoch, "batch": i, "loss": out,
                                                  "eval_cost": time.time() - t0,
                                                  "total_batch": total})
                outs.append(out)
                t0 = time.time()
        self._module.validation_epoch_end({"epoch": epoch, "eval_cost": time.time() - t_start})
        return outs

    @torch.no_grad()
    def predict(self, epoch=1, test_data_loader=None):
        self._flush_deferred_update()
        model = self._module.model
        model.eval()
        outs = []
        t0 = time.time()
        for i, batch in enumerate(test_data_loader):
            if i >= self._test_iters:
                break
            batch = _to_device(batch, self.device)
            out = self._module.test_step(batch)
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            lval = float(out.float().item()) if torch.is_tensor(out) and out.numel() == 1 else 0.0
            self._module.test_step_end({"epoch": epoch, "batch": i, "loss": lval,
                                        "test_cost": time.time() - t0})
            outs.append(out)
            t0 = time.time()
        return outs

    # ------------------------------------------------------------------ save/load
    def _shard_dir(self, base):
        if self._distributed:
            return os.path.join(base, ckpt.shard_dirname(self._mp_rank, self._sharding_rank,
                                                         self._pp_rank))
        return base

    def _params_gathered(self, writeback=False):
        g = getattr(self.buffer, "gathered", None)
        return g(writeback=writeback) if g is not None else contextlib.nullcontext()

    def save(self, epoch=0, step=0):
        if self._dp_rank != 0:
            return
        if self.optimizer is not None:
            self.optimizer.sync_state()  # an overlapped update may still be in flight
        if hasattr(self.buffer, "sync_params"):
            self.buffer.sync_params()  # and overlapped parameter gathers
        if torch.cuda.is_available():
            # never checkpoint the skipped / diverged state a timed-out one-shot
            # all-reduce leaves behind: raise first, naming the group
            torch.cuda.synchronize()
            _comm.check_all()
        target = self._shard_dir(ckpt.step_dir(self._output_dir, epoch, step))
        # stage 3: gather full parameters first (reference get_all_parameters, :600-601)
        with self._params_gathered():
            model_sd = {k: v.detach().to("cpu", copy=True)
                        for k, v in self._module.model.state_dict().items()}
        payloads = {"model.pdparams": model_sd}
        if self.optimizer is not None:
            payloads["model_state.pdopt"] = self.optimizer.state_dict()
        meta = {"epoch": epoch, "step": step, "consumed_samples": self.consumed_samples,
                "rng_tracker": get_rng_state_tracker().get_states()}
        if self.scaler is not None:
            meta["scaler"] = self.scaler.state_dict()
        if getattr(self, "_graph_salt", None) is not None:
            # graph mode: the device dropout salt continues after a resume
            meta["graph_salt"] = int(self._graph_salt.item())
        if torch.cuda.is_available():
            meta["cuda_rng_state"] = torch.cuda.get_rng_state()
        payloads["meta_state.pdopt"] = meta
        ckpt.save_payloads(target, payloads)
        logger.info("Save model to %s" % target)

    def load(self, ckpt_dir=None):
        ckpt_dir = ckpt_dir or self._ckpt_dir
        if not ckpt_dir:
            return
        if ckpt_dir == "auto":
            shards = None
            if self._distributed:
                h = self.hcg
                shards = [ckpt.shard_dirname(m, s, p) for m in range(h.mp_degree)
                          for s in range(h.sharding_degree) for p in range(h.pp_degree)]
            ckpt_dir = ckpt.latest_checkpoint(self._output_dir, shards)
            if ckpt_dir is None:
                logger.info("no checkpoint to resume from in %s" % self._output_dir)
                return
        d = self._shard_dir(ckpt_dir)
        if not os.path.isdir(d):
            d = ckpt_dir
        mp = os.path.join(d, "model.pdparams")
        if not os.path.isfile(mp):
            raise FileNotFoundError("{} not found".format(mp))
        sd = ckpt.load_payload(mp)
        with self._params_gathered(writeback=True):
            res = self._module.model.load_state_dict(sd, strict=False)
        missing = [k for k in res.missing_keys
                   if dict(self._module.model.named_parameters()).get(k) is not None
                   and dict(self._module.model.named_parameters())[k].requires_grad]
        if missing:
            raise RuntimeError("checkpoint {} lacks {} trainable parameter(s) of this model, e.g. "
                               "{}".format(mp, len(missing), missing[:5]))
        if res.unexpected_keys:
            logger.warning("checkpoint {}: {} unexpected key(s) ignored, e.g. {}".format(
                mp, len(res.unexpected_keys), res.unexpected_keys[:5]))
        if self.mode == "train":
            op, mt = os.path.join(d, "model_state.pdopt"), os.path.join(d, "meta_state.pdopt")
            if not (os.path.isfile(op) and os.path.isfile(mt)):
                raise FileNotFoundError("optimizer/meta state missing in {}".format(d))
            self.optimizer.set_state_dict(ckpt.load_payload(op))
            meta = ckpt.load_payload(mt)
            self._load_recovery = {"epoch": meta.get("epoch", 0), "step": meta.get("step", 0)}
            self.consumed_samples = int(meta.get("consumed_samples", 0))
            if "rng_tracker" in meta:
                get_rng_state_tracker().set_states(meta["rng_tracker"])
            self._graph_salt_resume = int(meta.get("graph_salt", 0))
            if getattr(self, "_graph_salt", None) is not None:
                self._graph_salt.fill_(self._graph_salt_resume)
            if self.scaler is not None and "scaler" in meta:
                self.scaler.load_state_dict(meta["scaler"])
            if "cuda_rng_state" in meta and torch.cuda.is_available():
                torch.cuda.set_rng_state(meta["cuda_rng_state"])
        logger.info("Load checkpoint from %s" % d)

    # ------------------------------------------------------------------ export / inference
    def export(self):
        from ...utils.export import export_inference_model
        # one directory per tensor-parallel shard (rank_{mp_rank}); data-parallel
        # replicas hold identical weights, so only the first replica writes
        if self.hcg.mp_degree > 1:
            if self._dp_rank != 0 or self._sharding_rank != 0:
                return
            out = os.path.join(self._output_dir, "rank_{}".format(self._mp_rank))
        else:
            out = os.path.join(self._output_dir, "rank_{}".format(self._dp_rank))
        with self._params_gathered():
            export_inference_model(self._module, out, mp_degree=self.hcg.mp_degree)
        logger.info("export model to %s" % out)

    def inference(self, data):
        if self._inference_engine is None:
            from .inference_engine import InferenceEngine
            self._inference_engine = InferenceEngine(self._inference_model_dir,
                                                     self.hcg.mp_degree)
        return self._inference_engine.predict(data)

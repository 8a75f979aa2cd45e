"""Native intra-node communicator: one-shot IPC all-reduce for small messages.

SURVEY.md N-11 / §5.8 (reference call sites: the three ParallelCrossEntropy
mp all-reduces, ``hybrid_model.py:799,822-824``; the mp all-reduce of every
decoder layer in an mp>1 ``InferenceEngine``, ``inference_engine.py:103-109``).

RCCL's ring/tree all-reduce is bandwidth-optimal but pays 2(n-1) link hops of
latency, which dominates the 4 KiB - 256 KiB tensor-parallel messages.  The
ranks of an MI355X node are fully connected by point-to-point xGMI links, so
:class:`IpcAllReduce` moves such a message in ONE hop: every rank pushes its
payload straight into every peer's receive area (IPC-mapped device memory,
``hipIpcGetMemHandle``/``hipIpcOpenMemHandle``) and reduces what it received
(``csrc/kernels/comm.hip``: 8-byte {epoch tag, data} granules, bounded spins,
rank-ordered reduction so every rank gets bitwise-identical results, device
side epochs so the call can be captured in a HIP graph).

Failure mode: every wait for a peer is bounded (``FLEETX_ONESHOT_TIMEOUT_S``,
default 120 s, long enough for a peer's checkpoint save or data stall).  A
timed-out call writes NaN into the outputs it could not reduce and raises the
device error flag; :func:`check_all` reads the flags (the engine calls it at
every logging sync and at the end of ``fit``) and raises naming the group, so
a slow or dead peer can never silently feed garbage into training.

:class:`Communicator` routes each call: the one-shot kernel when the group is
one node, the dtype/op are supported and the message fits the receive slot;
``torch.distributed`` (RCCL) otherwise.  Whether the one-shot path is used is
decided collectively (all ranks of the group or none), and with the
collective fingerprint checker enabled its calls are fingerprinted like the
RCCL ones (``parallel/collective_check.py``).
"""
import os
import socket

import torch
import torch.distributed as dist

from ..ops import _lib

# bytes of payload per rank above which RCCL's bandwidth-optimal algorithms win
DEFAULT_MAX_BYTES = int(os.environ.get("FLEETX_ONESHOT_MAX_BYTES", str(256 * 1024)))
# bound on every wait for a peer inside the kernel (seconds)
DEFAULT_TIMEOUT_S = float(os.environ.get("FLEETX_ONESHOT_TIMEOUT_S", "120"))
_TICKS_PER_S = 100_000_000  # s_memrealtime runs at 100 MHz
_DT = {torch.bfloat16: 0, torch.float16: 1, torch.float32: 2}
_OPS = {dist.ReduceOp.SUM: 0, dist.ReduceOp.MAX: 1}


def _group_members(group):
    return list(group.ranks) if group is not None else list(range(dist.get_world_size()))


class OneShotTimeout(RuntimeError):
    pass


def _agree(ok, pg, device):
    """True on every rank iff ``ok`` on every rank of the group."""
    backend = dist.get_backend(pg)
    dev = device if backend == "nccl" else torch.device("cpu")
    f = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(f, op=dist.ReduceOp.MIN, group=pg)
    return bool(int(f.item()))


class IpcAllReduce:
    """One-shot all-reduce over IPC-mapped receive areas of a single-node group.

    All ranks of ``group`` must construct it together (it exchanges IPC
    handles with an all-gather) and then issue the same sequence of calls.
    """

    def __init__(self, group=None, max_bytes=DEFAULT_MAX_BYTES, device=None,
                 timeout_s=DEFAULT_TIMEOUT_S):
        k = _lib.kernels()
        self.k = k
        self.group = group
        self.name = "world" if group is None else str(list(group.ranks))
        pg = group.group if group is not None else None
        members = _group_members(group)
        self.world = len(members)
        self.rank = members.index(dist.get_rank())
        if self.world > k.comm_max_world():
            raise ValueError("one-shot all-reduce supports up to %d ranks" % k.comm_max_world())
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.max_bytes = int(max_bytes)
        self.timeout_ticks = int(max(timeout_s, 1e-3) * _TICKS_PER_S)
        self.slot = (self.max_bytes + 3) // 4  # granules (4 payload bytes each) per source
        self.opened = []
        self.base = 0
        # Every step below is reached by every rank, whatever failed locally,
        # and the outcome is agreed on by all of them: one rank falling back to
        # RCCL while its peers spin in the kernel (or wait in a barrier) would
        # hang the group.
        why = None
        handle = None
        try:
            self.base = k.comm_alloc(self.slot)
            if not self.base:
                why = "hipExtMallocWithFlags(uncached) failed"
            else:
                handle = k.comm_ipc_handle(self.base)
        except RuntimeError as e:  # hipIpcGetMemHandle refused, ...
            why = str(e)
        handles = [None] * self.world
        dist.all_gather_object(handles, (socket.gethostname(), handle), group=pg)
        if why is None and len(set(h for h, _ in handles)) != 1:
            why = "one-shot all-reduce needs every rank of the group on one node"
        if why is None and any(h is None for _, h in handles):
            why = "a peer could not export its receive area"
        peers = []
        if why is None:
            for r, (_, h) in enumerate(handles):
                if r == self.rank:
                    peers.append(self.base)
                    continue
                p = k.comm_ipc_open(h)
                if not p:
                    why = "hipIpcOpenMemHandle failed for rank %d" % r
                    break
                self.opened.append(p)
                peers.append(p)
        ok = _agree(why is None, pg, self.device)
        if not ok:
            self.close()
            raise RuntimeError(why or "a peer could not set up the one-shot all-reduce")
        self.peers = peers
        self.epochs = torch.zeros(k.comm_max_blocks(), dtype=torch.int32, device=self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.calls = 0
        self._last = None  # (stream, event) of the previous call
        # every rank must have mapped every peer before anyone writes into it
        dist.barrier(group=pg)
        self._self_test(pg)

    def _self_test(self, pg, bound_s=5.0):
        """One all-reduce of known values under a short wait bound, agreed by
        every rank: a receive area the peers cannot reach (no peer mapping
        over xGMI, a refused IPC import that still returned a pointer, ...)
        then disables the path at setup instead of stalling the first training
        step for the full timeout and skipping it."""
        n = max(1, min(256, self.max_bytes // 4))
        probe = torch.full((n,), float(self.rank + 1), dtype=torch.float32, device=self.device)
        saved = self.timeout_ticks
        self.timeout_ticks = int(bound_s * _TICKS_PER_S)
        try:
            self.all_reduce(probe)
        finally:
            self.timeout_ticks = saved
        expect = float(self.world * (self.world + 1) // 2)
        ok = int(self.err.item()) == 0 and bool((probe == expect).all())
        self.err.zero_()
        if not _agree(ok, pg, self.device):
            self.close()
            raise RuntimeError("one-shot all-reduce self-test failed on group %s" % self.name)

    def supports(self, t, op=dist.ReduceOp.SUM):
        return (t.is_cuda and t.dtype in _DT and op in _OPS and t.is_contiguous()
                and t.numel() * t.element_size() <= self.max_bytes)

    def all_reduce(self, t, op=dist.ReduceOp.SUM, out=None):
        """Reduce ``t`` across the group on the current stream (in place
        unless ``out`` is given); returns the result tensor."""
        if not self.supports(t, op):
            raise ValueError("tensor not supported by the one-shot path")
        out = t if out is None else out
        self.calls += 1
        # calls must not overlap (shared device epochs): a call from another
        # stream than the previous one first waits for that one
        cur = torch.cuda.current_stream()
        capturing = torch.cuda.is_current_stream_capturing()
        if not capturing and self._last is not None and self._last[0] != cur:
            cur.wait_event(self._last[1])
        self.k.comm_allreduce(_DT[t.dtype], _OPS[op], t.data_ptr(), out.data_ptr(), t.numel(),
                              self.rank, self.world, self.peers, self.epochs.data_ptr(),
                              self.err.data_ptr(), self.slot, self.timeout_ticks, _lib.stream())
        if not capturing:  # a graph orders its own nodes
            ev = self._last[1] if self._last is not None and self._last[0] == cur \
                else torch.cuda.Event()
            ev.record(cur)
            self._last = (cur, ev)
        _lib.maybe_sync()
        return out

    def check(self):
        """Raise if any call timed out waiting for a peer (host sync).  The
        timed-out outputs were written as NaN; the flag stays set."""
        if int(self.err.item()) != 0:
            raise OneShotTimeout(
                "one-shot all-reduce on group %s timed out waiting for a peer (> %.1f s; "
                "FLEETX_ONESHOT_TIMEOUT_S); the affected outputs were written as NaN"
                % (self.name, self.timeout_ticks / _TICKS_PER_S))

    def close(self):
        for p in getattr(self, "opened", []):
            self.k.comm_ipc_close(p)
        self.opened = []
        if getattr(self, "base", 0):
            self.k.comm_free(self.base)
            self.base = 0


class Communicator:
    """Collective front end of one process group (``topology.CommGroup``):
    ``all_reduce`` takes the one-shot IPC kernel for small single-node
    messages and RCCL otherwise (``FLEETX_ONESHOT=0`` disables the kernel).
    Calls run on the caller's stream (no communicator stream of its own: the
    per-rank stream budget is fixed by ``GPU_MAX_HW_QUEUES``, see
    ``utils/streams.py``)."""

    def __init__(self, group, max_bytes=DEFAULT_MAX_BYTES, oneshot=None):
        self.group = group
        self.nranks = 1 if group is None else group.nranks
        self.oneshot = None
        if oneshot is None:
            oneshot = os.environ.get("FLEETX_ONESHOT", "1") == "1"
        # FLEETX_ONESHOT_FORCE=1 also enables it over gloo (GPU tests that put
        # several ranks on one device, where RCCL refuses to run)
        nccl = dist.get_backend(group.group if group is not None else None) == "nccl"
        force = os.environ.get("FLEETX_ONESHOT_FORCE", "0") == "1"
        # (world_error_flag does not key on this: communicators are created
        # lazily and differ between pipeline stages; world_oneshot_possible)
        self.tried_oneshot = bool(oneshot and self.nranks > 1 and torch.cuda.is_available()
                                  and (nccl or force))
        if self.tried_oneshot:
            try:
                self.oneshot = IpcAllReduce(group, max_bytes)
            except (RuntimeError, ValueError) as e:  # multi-node group, IPC refused, ...
                from ..utils.log import logger
                logger.warning("one-shot all-reduce disabled for %s: %s" % (group, e))
                self.oneshot = None

    def all_reduce(self, t, op=dist.ReduceOp.SUM):
        if self.nranks == 1:
            return t
        pg = self.group.group if self.group is not None else None
        if self.oneshot is not None and self.oneshot.supports(t, op):
            from . import collective_check
            collective_check.check_call("all_reduce", pg, t, op)
            return self.oneshot.all_reduce(t, op)
        dist.all_reduce(t, op=op, group=pg)
        return t

    def check(self):
        if self.oneshot is not None:
            self.oneshot.check()


_COMMS = {}


def get_communicator(group):
    """Cached :class:`Communicator` of a ``CommGroup`` (created collectively:
    every member must make its first call for a group at the same point)."""
    key = None if group is None else tuple(group.ranks)
    c = _COMMS.get(key)
    if c is None:
        c = Communicator(group)
        _COMMS[key] = c
    return c


def check_all():
    """Raise :class:`OneShotTimeout` if any one-shot call of this process timed
    out (one device read per communicator; call at host syncs)."""
    for c in _COMMS.values():
        c.check()


def error_flag():
    """Device int32 ``[1]``: non-zero once any one-shot call of this process
    timed out (no host sync), or ``None`` when no one-shot path exists.  The
    optimizer folds it into the step's found-inf so a step whose collectives
    lost a peer is skipped instead of applied."""
    flags = [c.oneshot.err for c in _COMMS.values() if c.oneshot is not None]
    if not flags:
        return None
    out = flags[0]
    for f in flags[1:]:
        out = out + f
    return out


def world_oneshot_possible():
    """Whether ANY rank's communicator may take the one-shot path, decided
    from state that is the same on every rank: the env switches, the world
    backend and the world size.  (Which communicators a rank has created is
    NOT rank-invariant: they are created lazily, and under pipeline
    parallelism the first, middle and last stages reach different
    collectives -- keying a world collective on them hangs the ranks that
    skip it.)"""
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return False
    if os.environ.get("FLEETX_ONESHOT", "1") != "1" or not torch.cuda.is_available():
        return False
    return dist.get_backend() == "nccl" or os.environ.get("FLEETX_ONESHOT_FORCE", "0") == "1"


def world_error_flag():
    """:func:`error_flag` shared by EVERY rank (MAX over the world, 4 bytes),
    or :func:`error_flag` alone when no rank can take the one-shot path.
    Whether the collective runs comes from :func:`world_oneshot_possible`
    (env / backend / world size), so every rank enters it at the same step,
    also ranks that never created a communicator, or whose group's one-shot
    setup failed (they contribute a zero)."""
    err = error_flag()
    if not world_oneshot_possible():
        return err
    dev = torch.device("cuda", torch.cuda.current_device())
    err = torch.zeros(1, dtype=torch.int32, device=dev) if err is None \
        else (err != 0).to(torch.int32)
    dist.all_reduce(err, op=dist.ReduceOp.MAX)
    return err


def reset():
    for c in _COMMS.values():
        if c.oneshot is not None:
            c.oneshot.close()
    _COMMS.clear()

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

:class:`Communicator` routes each call: the one-shot kernel when the group is
one node, the dtype/op are supported and the message fits the receive slot;
``torch.distributed`` (RCCL) otherwise.  It also owns a dedicated HIP stream
for collectives issued asynchronously (:meth:`Communicator.all_reduce_async`).
"""
import os
import socket

import torch
import torch.distributed as dist

from ..ops import _lib

# bytes of payload per rank above which RCCL's bandwidth-optimal algorithms win
DEFAULT_MAX_BYTES = int(os.environ.get("FLEETX_ONESHOT_MAX_BYTES", str(256 * 1024)))
_DT = {torch.bfloat16: 0, torch.float16: 1, torch.float32: 2}
_OPS = {dist.ReduceOp.SUM: 0, dist.ReduceOp.MAX: 1}


def _group_members(group):
    return list(group.ranks) if group is not None else list(range(dist.get_world_size()))


class IpcAllReduce:
    """One-shot all-reduce over IPC-mapped receive areas of a single-node group.

    All ranks of ``group`` must construct it together (it exchanges IPC
    handles with an all-gather) and then issue the same sequence of calls.
    """

    def __init__(self, group=None, max_bytes=DEFAULT_MAX_BYTES, device=None):
        k = _lib.kernels()
        self.k = k
        self.group = group
        pg = group.group if group is not None else None
        members = _group_members(group)
        self.world = len(members)
        self.rank = members.index(dist.get_rank())
        if self.world > k.comm_max_world():
            raise ValueError("one-shot all-reduce supports up to %d ranks" % k.comm_max_world())
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.max_bytes = int(max_bytes)
        self.slot = (self.max_bytes + 3) // 4  # granules (4 payload bytes each) per source
        self.base = k.comm_alloc(self.slot)
        if not self.base:
            raise RuntimeError("hipExtMallocWithFlags(uncached) failed")
        handle = k.comm_ipc_handle(self.base)
        handles = [None] * self.world
        dist.all_gather_object(handles, (socket.gethostname(), handle), group=pg)
        if len(set(h for h, _ in handles)) != 1:
            k.comm_free(self.base)
            raise RuntimeError("one-shot all-reduce needs every rank of the group on one node")
        self.opened = []
        peers = []
        for r, (_, h) in enumerate(handles):
            if r == self.rank:
                peers.append(self.base)
                continue
            p = k.comm_ipc_open(h)
            if not p:
                self.close()
                raise RuntimeError("hipIpcOpenMemHandle failed for rank %d" % r)
            self.opened.append(p)
            peers.append(p)
        self.peers = peers
        self.epochs = torch.zeros(k.comm_max_blocks(), dtype=torch.int32, device=self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.calls = 0
        self._last = None  # (stream, event) of the previous call
        # every rank must have mapped every peer before anyone writes into it
        dist.barrier(group=pg)

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
                              self.err.data_ptr(), self.slot, _lib.stream())
        if not capturing:  # a graph orders its own nodes
            ev = self._last[1] if self._last is not None and self._last[0] == cur \
                else torch.cuda.Event()
            ev.record(cur)
            self._last = (cur, ev)
        _lib.maybe_sync()
        return out

    def check(self):
        """Raise if any call timed out waiting for a peer (host sync)."""
        if int(self.err.item()) != 0:
            raise RuntimeError("one-shot all-reduce timed out waiting for a peer")

    def close(self):
        for p in getattr(self, "opened", []):
            self.k.comm_ipc_close(p)
        self.opened = []
        if getattr(self, "base", 0):
            self.k.comm_free(self.base)
            self.base = 0


class Communicator:
    """Collective front end of one process group (``topology.CommGroup``).

    * ``all_reduce``: one-shot IPC kernel for small single-node messages,
      RCCL otherwise (``FLEETX_ONESHOT=0`` disables the kernel);
    * ``all_reduce_async``: the same on this communicator's own HIP stream,
      ordered after the caller's stream, returning an event to wait on.
    """

    def __init__(self, group, max_bytes=DEFAULT_MAX_BYTES, oneshot=None):
        self.group = group
        self.nranks = 1 if group is None else group.nranks
        self.oneshot = None
        self._stream = None
        if oneshot is None:
            oneshot = os.environ.get("FLEETX_ONESHOT", "1") == "1"
        # FLEETX_ONESHOT_FORCE=1 also enables it over gloo (GPU tests that put
        # several ranks on one device, where RCCL refuses to run)
        nccl = dist.get_backend(group.group if group is not None else None) == "nccl"
        force = os.environ.get("FLEETX_ONESHOT_FORCE", "0") == "1"
        if oneshot and self.nranks > 1 and torch.cuda.is_available() and (nccl or force):
            try:
                self.oneshot = IpcAllReduce(group, max_bytes)
            except (RuntimeError, ValueError) as e:  # multi-node group, IPC refused, ...
                from ..utils.log import logger
                logger.warning("one-shot all-reduce disabled for %s: %s" % (group, e))
                self.oneshot = None

    @property
    def stream(self):
        if self._stream is None:
            self._stream = torch.cuda.Stream()
        return self._stream

    def all_reduce(self, t, op=dist.ReduceOp.SUM):
        if self.nranks == 1:
            return t
        if self.oneshot is not None and self.oneshot.supports(t, op):
            return self.oneshot.all_reduce(t, op)
        dist.all_reduce(t, op=op, group=self.group.group if self.group is not None else None)
        return t

    def all_reduce_async(self, t, op=dist.ReduceOp.SUM):
        """Issue on the communicator stream; returns an event recorded after it."""
        cur = torch.cuda.current_stream()
        s = self.stream
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            self.all_reduce(t, op)
            ev = torch.cuda.Event()
            ev.record(s)
        t.record_stream(s)
        return ev


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


def reset():
    for c in _COMMS.values():
        if c.oneshot is not None:
            c.oneshot.close()
    _COMMS.clear()

"""Per-rank HIP stream budget.

HIP maps a process's streams round-robin onto ``GPU_MAX_HW_QUEUES`` hardware
queues (4 by default), and every RCCL communicator adds a stream of its own.
Two kernels that spin on peers -- RCCL collectives / p2p, the one-shot IPC
all-reduce -- queued in one in-order hardware queue in a different order on
two ranks can deadlock the job, so the framework keeps its own streams few
and names them:

* ``compute``  -- the default stream: forward, backward, the one-shot
  all-reduces (they run on the caller's stream);
* ``side``     -- ONE background stream per device shared by the
  forward-overlapped AdamW (step N's update under step N+1's forward), the
  early per-bucket gradient norm and the opt-in weight-gradient stream
  (they never need to run concurrently with each other); with
  ``Distributed.comm.overlap_optimizer_cus`` the overlapped AdamW instead
  gets a stream pinned to that many CUs (:func:`cu_masked_stream`);
* ``copy``     -- only with ZeRO CPU offload (H2D/D2H staging);
* one RCCL stream per process group in use.  The pipeline uses ONE
  communicator per pipe group by default: both directions of a stage link
  share one in-order stream of grouped ``batch_isend_irecv`` calls, which is
  deadlock-free whatever the queue mapping (``Distributed.comm.
  pp_split_directions`` opts back into two).

:func:`log_inventory` prints the count at engine init and warns when the
streams that may carry peer-waiting kernels outnumber the hardware queues.
:func:`ensure_hw_queues` (launcher / bench, before HIP initialises) raises
``GPU_MAX_HW_QUEUES`` for multi-rank jobs so RCCL communicators do not share
queues (at most 32, the pool's limit).
"""
import os

import torch

_SIDE = {}


def side_stream(device):
    """The shared background stream of ``device``."""
    dev = torch.device(device)
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _SIDE.get(key)
    if s is None:
        s = torch.cuda.Stream(device=torch.device("cuda", key))
        _SIDE[key] = s
    return s


_MASKED = {}


def cu_masked_stream(device, ncu):
    """A stream of ``device`` whose kernels run only on ``ncu`` fixed CUs
    (``csrc/kernels/streams.hip``), as a ``torch.cuda.ExternalStream``;
    ``None`` if the runtime refuses the mask."""
    dev = torch.device(device)
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), int(ncu))
    s = _MASKED.get(key)
    if s is None:
        from ..ops import _lib
        with torch.cuda.device(key[0]):
            handle, got = _lib.kernels().cumask_stream_create(int(ncu))
        if not handle:
            return None
        s = torch.cuda.ExternalStream(handle, device=torch.device("cuda", key[0]))
        s.fx_cus = got
        _MASKED[key] = s
    return s


def hw_queues(env=None):
    env = os.environ if env is None else env
    try:
        return int(env.get("GPU_MAX_HW_QUEUES", "4") or 4)
    except ValueError:
        return 4


def ensure_hw_queues(n=8, limit=32, env=None):
    """Raise ``GPU_MAX_HW_QUEUES`` in ``env`` (default: this process) to ``n``
    (never lower it, never above ``limit``).  Only effective before the HIP
    runtime of that process initialises."""
    env = os.environ if env is None else env
    cur = hw_queues(env)
    want = min(max(cur, n), limit)
    if want != cur or "GPU_MAX_HW_QUEUES" not in env:
        env["GPU_MAX_HW_QUEUES"] = str(want)
    return want


def inventory(hcg=None, optimizer=None, buffer=None, wgrad_stream=False):
    """``[(name, peer_waiting)]`` of the streams this rank uses."""
    out = [("compute", True)]
    side_users = []
    masked = getattr(getattr(optimizer, "_opt_stream", None), "fx_cus", None)
    if optimizer is not None and getattr(optimizer, "_overlap_groups", None) is not None:
        if masked:
            out.append(("adamw-overlap(%d CUs)" % masked, False))
        else:
            side_users.append("adamw-overlap")
    if buffer is not None and getattr(buffer, "_norm_stream", None) is not None:
        side_users.append("early-norm")
    if wgrad_stream:
        side_users.append("wgrad")
    if side_users:
        out.append(("side(%s)" % "+".join(side_users), False))
    if optimizer is not None and getattr(optimizer, "_copy_stream", None) is not None:
        out.append(("copy", False))
    if hcg is not None:
        seen = set()
        for name, g in sorted(getattr(hcg, "_groups", {}).items()):
            if g is None or g.group is None or id(g.group) in seen:
                continue
            seen.add(id(g.group))
            c = hcg.ctas_for(name) if getattr(hcg, "_nccl", False) and hasattr(hcg, "ctas_for") \
                else None
            budget = "" if c is None else "(ctas %s-%s)" % (c[0] or "auto", c[1] or "auto")
            out.append(("rccl:%s%s%s" % (name, list(g.ranks), budget), True))
    return out


def log_inventory(hcg=None, optimizer=None, buffer=None, wgrad_stream=False):
    from .log import logger
    inv = inventory(hcg, optimizer, buffer, wgrad_stream)
    q = hw_queues()
    peer = sum(1 for _, p in inv if p)
    msg = "stream inventory: %d streams (%d may wait on peers) over %d HW queues: %s" % (
        len(inv), peer, q, ", ".join(n for n, _ in inv))
    if peer > q:
        logger.warning(msg + " -- more peer-waiting streams than hardware queues; set "
                       "GPU_MAX_HW_QUEUES >= %d (fleetx_amd.launch / bench.py do for "
                       "multi-rank runs)" % peer)
    else:
        logger.info(msg)
    return inv

"""Collective fingerprint checking (SURVEY §5.2 race / desync detection).

``Distributed.debug: fingerprint`` (or ``FLEETX_COLLECTIVE_CHECK=fingerprint``)
wraps the ``torch.distributed`` collectives the framework issues.  Before a
collective runs on a group, every member contributes a fingerprint of the
call -- op, per-group sequence number, dtype, element count and the leading
four dims -- to an all-gather over a CPU gloo MIRROR of that group, and the
call is refused with a per-rank table when the fingerprints differ.  A rank
that took a different branch (skipped a bucket, changed a shape, swapped the
order of two collectives) is named at the first divergent call instead of
hanging RCCL or silently reducing mismatched buffers.

The mirrors are created eagerly for every group of the hybrid topology
(``new_group`` is collective over the world, so it cannot happen lazily inside
a sub-group call).  Cost: one small gloo all-gather per collective -- a
debugging mode, off by default.  Point-to-point ops are pairwise and are not
fingerprinted.
"""
import zlib

import torch
import torch.distributed as dist

_OPS = ("all_reduce", "all_gather_into_tensor", "reduce_scatter_tensor", "broadcast",
        "all_gather", "reduce_scatter", "reduce", "all_to_all_single")
_DTYPES = [torch.float32, torch.float16, torch.bfloat16, torch.float64, torch.int32,
           torch.int64, torch.uint8, torch.int8, torch.bool]
_state = {"enabled": False, "orig": {}, "mirror": {}, "seq": {}, "world": None}
_P2P_LEN = 9


class CollectiveMismatch(RuntimeError):
    pass


def _first_tensor(args, kwargs):
    for a in list(args) + list(kwargs.values()):
        if torch.is_tensor(a):
            return a
        if isinstance(a, (list, tuple)) and a and torch.is_tensor(a[0]):
            return a[0]
    return None


def _fingerprint(op, seq, t, extra=0):
    shape = list(t.shape) if t is not None else []
    dims = (shape + [0, 0, 0, 0])[:4]
    dt = _DTYPES.index(t.dtype) if t is not None and t.dtype in _DTYPES else -1
    numel = t.numel() if t is not None else 0
    return torch.tensor([_OPS.index(op), seq, dt, numel, len(shape)] + dims + [extra],
                        dtype=torch.int64)


def _describe(row):
    op = _OPS[int(row[0])] if 0 <= int(row[0]) < len(_OPS) else "?"
    dt = _DTYPES[int(row[2])] if 0 <= int(row[2]) < len(_DTYPES) else "?"
    nd = int(row[4])
    return "#%d %s %s %s" % (int(row[1]), op, str(dt).replace("torch.", ""),
                             tuple(int(x) for x in row[5:5 + min(nd, 4)]))


def _check(op, group, t, extra=0):
    key = group if group is not None else "world"
    mirror = _state["mirror"].get(key)
    if mirror is None:
        return
    seq = _state["seq"].get(key, 0)
    _state["seq"][key] = seq + 1
    fp = _fingerprint(op, seq, t, extra)
    n = dist.get_world_size(mirror)
    out = [torch.empty_like(fp) for _ in range(n)]
    _state["orig"]["all_gather"](out, fp, group=mirror)
    if any(not torch.equal(o, out[0]) for o in out[1:]):
        ranks = dist.get_process_group_ranks(mirror) if hasattr(dist, "get_process_group_ranks") \
            else list(range(n))
        rows = "\n".join("  rank %d: %s" % (r, _describe(o)) for r, o in zip(ranks, out))
        raise CollectiveMismatch("collective fingerprint mismatch on group {}:\n{}".format(
            ranks, rows))


def enabled():
    return _state["enabled"]


def _p2p_fp(seq, t):
    shape = list(t.shape)
    dt = _DTYPES.index(t.dtype) if t.dtype in _DTYPES else -1
    return torch.tensor([seq, dt, t.numel(), len(shape)] + (shape + [0, 0, 0, 0])[:4] + [0],
                        dtype=torch.int64)


def _p2p_describe(row):
    dt = _DTYPES[int(row[1])] if 0 <= int(row[1]) < len(_DTYPES) else "?"
    nd = int(row[3])
    return "#%d %s %s" % (int(row[0]), str(dt).replace("torch.", ""),
                          tuple(int(x) for x in row[4:4 + min(nd, 4)]))


def check_p2p(group, ops):
    """Fingerprint one grouped p2p call (``ops = [(kind, tensor, peer)]``,
    peer a global rank) against the matching calls of its peers."""
    mirror = _state["mirror"].get(group)
    if mirror is None:
        return
    works, checks = [], []
    for kind, t, peer in ops:
        key = (mirror, peer, kind)
        seq = _state["seq"].get(key, 0)
        _state["seq"][key] = seq + 1
        fp = _p2p_fp(seq, t)
        if kind == "send":
            works.append(dist.isend(fp, dst=peer, group=mirror))
        else:
            got = torch.empty(_P2P_LEN, dtype=torch.int64)
            works.append(dist.irecv(got, src=peer, group=mirror))
            checks.append((peer, fp, got))
    for w in works:
        w.wait()
    for peer, want, got in checks:
        if not torch.equal(want, got):
            raise CollectiveMismatch(
                "p2p fingerprint mismatch: rank {} expects to receive {} from rank {}, "
                "which sent {}".format(dist.get_rank(), _p2p_describe(want), peer,
                                       _p2p_describe(got)))


def _op_extra(rop):
    return zlib.crc32(str(rop).encode()) & 0xFFFF if rop is not None else 0


def check_call(op, group, t, rop=None):
    """Fingerprint a collective issued outside ``torch.distributed`` (the
    one-shot IPC all-reduce of ``parallel/comm.py``) exactly like the wrapped
    ones, so a rank that routes a call differently is named too."""
    if _state["enabled"]:
        _check(op, group, t, _op_extra(rop))


def _wrap(op):
    orig = getattr(dist, op)

    def wrapped(*args, **kwargs):
        group = kwargs.get("group")
        if group is None:
            # positional group argument (all_reduce(t, op, group, async_op))
            for a in args:
                if isinstance(a, dist.ProcessGroup):
                    group = a
                    break
        t = _first_tensor(args, kwargs)
        _check(op, group, t, _op_extra(kwargs.get("op")))
        return orig(*args, **kwargs)
    wrapped.__wrapped__ = orig
    return wrapped


def enable(hcg=None):
    """Install the wrappers.  Collective: call on every rank after the hybrid
    topology exists (creates the gloo mirrors)."""
    if _state["enabled"] or not dist.is_initialized():
        return False
    mirrors = {}
    world = dist.new_group(backend="gloo")
    mirrors["world"] = world
    if hcg is not None:
        # every group of every axis, created in the same order on every rank
        seen = dict(hcg._groups)
        for name in sorted(seen):
            rank_lists = _rank_lists(hcg, name)
            for ranks in rank_lists:
                if len(ranks) < 2:
                    continue
                gg = dist.new_group(ranks=ranks, backend="gloo")
                mine = seen[name]
                if mine is not None and mine.group is not None and list(mine.ranks) == list(ranks):
                    mirrors[mine.group] = gg
    _state["mirror"] = mirrors
    for op in _OPS:
        if hasattr(dist, op):
            _state["orig"][op] = getattr(dist, op)
    _state["orig"].setdefault("all_gather", dist.all_gather)
    for op in _OPS:
        if hasattr(dist, op):
            setattr(dist, op, _wrap(op))
    _state["enabled"] = True
    return True


def _rank_lists(hcg, name):
    t = hcg.topo
    if name in ("data", "pipe", "sharding", "model", "pipe_bwd"):
        return t.axis_groups("pipe" if name == "pipe_bwd" else name)
    if name == "data_world":
        return hcg._data_world_groups()
    if name == "check":
        return hcg._check_groups()
    if name == "embedding":
        return hcg._embedding_groups()
    return []


def disable():
    if not _state["enabled"]:
        return
    for op, fn in _state["orig"].items():
        setattr(dist, op, fn)
    _state.update(enabled=False, orig={}, mirror={}, seq={})

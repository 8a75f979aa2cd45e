"""Order replay of the pipeline schedules' grouped p2p calls (no devices).

RCCL semantics being modelled: the grouped calls of one communicator run in
order on one stream; a group completes only when every send in it has met
the matching receive (the k-th send rank r -> q on a communicator meets the
k-th receive on q from r) inside the group that is ACTIVE on the peer's
stream, and vice versa (rendezvous -- transfers of ``[micro_b, s, h]`` are far
larger than RCCL's per-channel staging buffer, so a send cannot complete
into an unposted receive).  A group is enqueued on its stream when the rank's
compute stream reaches the post (the comm stream waits for the producer), and
the compute stream blocks where it waits for a receive.

``record(kind, P, m, V, split)`` runs ``PipelineSchedule`` for every stage on
the CPU with tiny tensors and a recording transport, and ``replay(logs)``
plays the logs against the model above (``blocking=True`` additionally waits
for every group right after posting it: the host-blocking matching that
``collective_check.check_p2p`` and gloo impose).  A schedule whose posting
order can deadlock on RCCL raises :class:`Deadlock` naming every blocked
rank's head group.

Reference parity: the schedules replayed are the P05 / N10 paths
(reference ``eager_engine.py:406-410``, ``hybrid_model.py:862-962``).
"""
import itertools
from types import SimpleNamespace

import torch

from .pipeline import P2P, PipelineSchedule


class Deadlock(RuntimeError):
    pass


class _Work:
    def __init__(self, log, gid):
        self.log, self.gid = log, gid

    def wait(self):
        self.log.append(("wait", self.gid))


class _Recorder:
    """Recording transport for one rank: ``issue(group, ops)`` logs the group
    and returns one coalesced Work (RCCL-style)."""

    def __init__(self, names, counter):
        self.log = []
        self.names = names
        self.counter = counter

    def __call__(self, group, ops):
        gid = next(self.counter)
        self.log.append(("post", gid, self.names[id(group)],
                         tuple((kind, peer) for kind, _, peer in ops)))
        return [_Work(self.log, gid)]


def _hcg(P, rank, g, gb):
    return SimpleNamespace(
        pp_rank=rank, pp_degree=P,
        get_pipe_parallel_group=lambda: SimpleNamespace(group=g, ranks=list(range(P))),
        get_pipe_bwd_group=lambda: SimpleNamespace(group=gb, ranks=list(range(P))))


def record(kind, P, m, V=1, split=False):
    """Per-rank event logs of one step of schedule ``kind`` (``"1f1b"``,
    ``"interleaved"``, ``"forward_only"``, ``"forward_only_interleaved"``)."""
    g = object()
    gb = object() if split else g
    names = {id(g): "pipe", id(gb): "pipe_bwd" if split else "pipe"}
    counter = itertools.count()
    logs = []
    shape = (2, 3)
    for rank in range(P):
        rec = _Recorder(names, counter)
        hcg = _hcg(P, rank, g, gb)
        sched = PipelineSchedule(hcg, lambda: shape, torch.float32, "cpu", num_chunks=V,
                                 p2p=P2P(hcg, issue=rec))
        w = torch.nn.Parameter(torch.full(shape, 1.0 + rank))

        def stage_fn(c, k, x, rank=rank, w=w):
            h = w * float(k + 1) if x is None else x.float() * w
            if rank == P - 1 and c == V - 1:
                return h.sum()
            return h

        if kind == "1f1b":
            sched.train_1f1b(m, stage_fn)
        elif kind == "interleaved":
            sched.train_interleaved(m, stage_fn)
        elif kind == "forward_only":
            sched.forward_only(m, stage_fn)
        elif kind == "forward_only_interleaved":
            sched.forward_only_interleaved(m, stage_fn)
        else:
            raise ValueError(kind)
        logs.append(rec.log)
    return logs


def replay(logs, blocking=False):
    """Play per-rank logs against in-order per-(rank, communicator) matching.
    Returns the number of groups completed; raises :class:`Deadlock`."""
    n = len(logs)
    progs = []
    for log in logs:
        ev = []
        for e in log:
            ev.append(e)
            if blocking and e[0] == "post":
                ev.append(("wait", e[1]))
        progs.append(ev)
    pc = [0] * n
    queues = {}                  # (rank, comm) -> [group]
    done = set()
    seq = {}                     # (comm, src, dst, kind) -> count of ops posted
    groups = {}

    def enqueue(rank, gid, comm, ops):
        items = []
        for kind, peer in ops:
            key = (comm, rank, peer, kind) if kind == "send" else (comm, peer, rank, kind)
            k = seq.get(key, 0)
            seq[key] = k + 1
            items.append([kind, peer, k, False])
        grp = {"gid": gid, "rank": rank, "comm": comm, "ops": items}
        groups[gid] = grp
        queues.setdefault((rank, comm), []).append(grp)

    def head(rank, comm):
        q = queues.get((rank, comm))
        return q[0] if q else None

    completed = 0
    while True:
        progress = False
        for r in range(n):                   # advance compute streams
            while pc[r] < len(progs[r]):
                e = progs[r][pc[r]]
                if e[0] == "post":
                    enqueue(r, e[1], e[2], e[3])
                elif e[1] not in done:
                    break
                pc[r] += 1
                progress = True
        for (r, comm), q in list(queues.items()):   # match active heads
            if not q:
                continue
            grp = q[0]
            for op in grp["ops"]:
                if op[3]:
                    continue
                kind, peer, k = op[0], op[1], op[2]
                other = head(peer, comm)
                if other is None:
                    continue
                want = "recv" if kind == "send" else "send"
                for o in other["ops"]:
                    if not o[3] and o[0] == want and o[1] == r and o[2] == k:
                        o[3] = op[3] = True
                        progress = True
                        break
        for (r, comm), q in queues.items():         # retire finished groups
            while q and all(op[3] for op in q[0]["ops"]):
                done.add(q.pop(0)["gid"])
                completed += 1
                progress = True
        if all(pc[r] == len(progs[r]) for r in range(n)) and \
                all(not q for q in queues.values()):
            return completed
        if not progress:
            blocked = []
            for r in range(n):
                heads = ["%s: %s" % (comm, [(o[0], o[1], o[2]) for o in q[0]["ops"] if not o[3]])
                         for (rr, comm), q in sorted(queues.items(), key=lambda kv: kv[0][1])
                         if rr == r and q]
                at = progs[r][pc[r]] if pc[r] < len(progs[r]) else "end"
                blocked.append("  rank %d at %s; heads %s" % (r, at, heads))
            raise Deadlock("p2p schedule deadlocks:\n" + "\n".join(blocked))

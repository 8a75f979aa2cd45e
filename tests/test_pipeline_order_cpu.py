"""RCCL ordering safety of the pipeline schedules (no devices needed).

Every schedule's grouped ``batch_isend_irecv`` calls are recorded per stage
and replayed against in-order per-communicator matching
(``fleetx_amd/parallel/p2p_replay.py``): RCCL runs one communicator's groups
in order on one stream and a group finishes only when all its transfers met
their peers, so a posting order that differs between the two ends of a link
deadlocks on GPUs even though gloo (independent ops) runs it fine.

Reference call sites: ``eager_engine.py:406-410`` (``train_batch``),
``hybrid_model.py:862-962`` (``GPTForPretrainingPipe``).
"""
import pytest

from fleetx_amd.parallel import p2p_replay

CASES = [(P, m) for P in (2, 4, 8) for m in sorted({P, 2 * P, 8, 1, P + 1})]


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("blocking", [False, True])
@pytest.mark.parametrize("P,m", CASES)
def test_1f1b_order(P, m, split, blocking):
    logs = p2p_replay.record("1f1b", P, m, split=split)
    assert p2p_replay.replay(logs, blocking=blocking) > 0


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("blocking", [False, True])
@pytest.mark.parametrize("V", [2, 3])
@pytest.mark.parametrize("P,m", [(P, m) for P in (2, 4, 8) for m in (P, 2 * P) if m <= 8 or P == 8])
def test_interleaved_order(P, m, V, split, blocking):
    logs = p2p_replay.record("interleaved", P, m, V=V, split=split)
    assert p2p_replay.replay(logs, blocking=blocking) > 0


@pytest.mark.parametrize("kind,V", [("forward_only", 1), ("forward_only_interleaved", 2)])
@pytest.mark.parametrize("P,m", [(2, 2), (4, 8), (8, 8)])
def test_forward_only_order(kind, V, P, m):
    for blocking in (False, True):
        assert p2p_replay.replay(p2p_replay.record(kind, P, m, V=V), blocking=blocking) > 0


def test_replay_catches_mismatched_posting_order():
    """The round-3 1F1B posted the activation-direction and gradient-direction
    groups of one exchange separately, in an order that differed between
    neighbouring stages; the replay must call that a deadlock."""
    g = "pipe"
    # stage 0: {send y0} {recv dy0} {send y1} {recv dy1}
    # stage 1: {recv x0} {recv x1} {send dx0} {send dx1}
    logs = [
        [("post", 0, g, (("send", 1),)), ("post", 1, g, (("recv", 1),)), ("wait", 1),
         ("post", 2, g, (("send", 1),)), ("post", 3, g, (("recv", 1),)), ("wait", 3)],
        [("post", 4, g, (("recv", 0),)), ("wait", 4), ("post", 5, g, (("recv", 0),)),
         ("post", 6, g, (("send", 0),)), ("wait", 5), ("post", 7, g, (("send", 0),))],
    ]
    with pytest.raises(p2p_replay.Deadlock):
        p2p_replay.replay(logs)
    # the same transfers with separate communicators per direction complete
    logs[0] = [(e[0], e[1], "bwd" if e[0] == "post" and e[3][0][0] == "recv" else g) + e[3:]
               if e[0] == "post" else e for e in logs[0]]
    logs[1] = [(e[0], e[1], "bwd" if e[0] == "post" and e[3][0][0] == "send" else g) + e[3:]
               if e[0] == "post" else e for e in logs[1]]
    assert p2p_replay.replay(logs) == 8


def test_groups_are_mirror_images_in_steady_state():
    """1F1B on one communicator: stage s's {send y, recv dy} meets stage s+1's
    {send dx, recv x} -- one group per exchange, two ops each."""
    logs = p2p_replay.record("1f1b", 2, 4)
    posts0 = [set(e[3]) for e in logs[0] if e[0] == "post"]
    posts1 = [set(e[3]) for e in logs[1] if e[0] == "post"]
    assert {("send", 1), ("recv", 1)} in posts0
    assert {("send", 0), ("recv", 0)} in posts1
    n_send0 = sum(op[0] == "send" for p in posts0 for op in p)
    n_recv1 = sum(op[0] == "recv" for p in posts1 for op in p)
    assert n_send0 == n_recv1 == 4

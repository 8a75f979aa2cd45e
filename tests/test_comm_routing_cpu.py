"""CPU-side logic of the round-2 runtime pieces: the communicator's RCCL/gloo
fallback (no one-shot kernel off the GPU), the measured GEMM routing table,
and the decode-split rule."""
import torch
import torch.distributed as dist

from tests import dist_utils


def _comm_worker(rank, world):
    from fleetx_amd.parallel.comm import Communicator
    from fleetx_amd.parallel.topology import CommGroup
    g = CommGroup(list(range(world)), None)
    c = Communicator(g)
    assert c.oneshot is None  # gloo / CPU: plain torch.distributed
    x = torch.full((5,), float(rank + 1))
    y = c.all_reduce(x.clone())
    m = c.all_reduce(torch.tensor([float(rank)]), dist.ReduceOp.MAX)
    return y.tolist(), m.item()


def test_communicator_falls_back_to_torch_distributed():
    res = dist_utils.run(_comm_worker, 2)
    for y, m in res:
        assert y == [3.0] * 5 and m == 1.0


def test_gemm_routing_table():
    from types import SimpleNamespace as NS
    from fleetx_amd.ops import gemm as G

    def t(*shape):  # a shape-only stand-in for a bf16 GPU tensor
        return NS(shape=shape, numel=lambda: __import__("math").prod(shape), is_cuda=True,
                  dtype=torch.bfloat16)
    old = G._MODE, G.ROUTE_TUNE
    try:
        G.set_mode("auto")
        G.ROUTE_TUNE = False
        x, w_qkv = t(8192, 4096), t(12288, 4096)
        # 6.7B: weight gradients and the fused-epilogue GEMMs go to the MFMA kernel
        assert G.out_tiles("wgrad", t(8192, 12288), x, 256) == 48 * 16
        assert G.use("wgrad", t(8192, 12288), x) and G.use("wgrad", t(8192, 4096), x)
        assert not G.use("fwd_act", x, t(16384, 4096))          # opt-in (FLEETX_GEMM_AUTO)
        # forward and data-gradient GEMMs are not in the kind table (the
        # per-shape race decides them on GPU; off here)
        assert not G.use("fwd", x, w_qkv) and not G.use("dgrad", t(8192, 12288), w_qkv)
        # hidden 1024-2048 shapes run on 128 x 128 tiles: 1.3B out-proj (256
        # tiles), 345M qkv / fc1 (192 / 256); the 345M out-proj (64 tiles) runs
        # split along K (gemm5.hip g5_split_plan); 32 tiles stay on hipBLASLt
        assert G.use("wgrad", t(8192, 2048), t(8192, 2048))
        assert G.use("wgrad", t(8192, 3072), t(8192, 1024))
        assert G.use("wgrad", t(8192, 1024), t(8192, 1024))
        assert not G.use("wgrad", t(8192, 512), t(8192, 1024))
        G.set_mode("blas")
        assert not G.use("wgrad", t(8192, 12288), x)
    finally:
        G.set_mode(old[0])
        G.ROUTE_TUNE = old[1]


def test_decode_split_rule():
    from fleetx_amd.ops.attention import decode_splits
    assert decode_splits(1, 16, 192) == 1          # short context: one split, no combine
    assert decode_splits(1, 32, 32768) == 64       # long context fills the chip
    assert decode_splits(64, 32, 32768) == 1       # enough (b, h) pairs already


def test_engine_raises_on_oneshot_timeout(monkeypatch):
    """fit() reads the one-shot error flags at every logging sync and stops,
    instead of training on NaN-poisoned all-reduce outputs."""
    import pytest
    from fleetx_amd.parallel import comm
    from fleetx_amd.core.engine import eager_engine

    calls = []

    def boom():
        calls.append(1)
        raise comm.OneShotTimeout("one-shot all-reduce on group [0, 1] timed out")

    monkeypatch.setattr(comm, "check_all", boom)
    monkeypatch.setattr(eager_engine.torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(eager_engine.torch.cuda, "synchronize", lambda *a, **k: None)
    eng = eager_engine.EagerEngine.__new__(eager_engine.EagerEngine)
    eng._logging_freq = 1
    eng._configs = type("C", (), {"Global": type("G", (), {"global_batch_size": 1})()})()
    eng._fit_impl = lambda batch: None
    eng._fault_check = lambda step: None
    eng.device = eager_engine.torch.device("cpu")
    eng.consumed_samples = 0
    with pytest.raises(comm.OneShotTimeout):
        eng._train_one_epoch(0, [[eager_engine.torch.zeros(1)]], None, 0)
    assert calls


def test_stream_inventory_counts_peer_waiting_streams():
    from fleetx_amd.utils import streams

    class G:
        def __init__(self, ranks):
            self.ranks, self.group = ranks, object()

    class H:
        _groups = {"model": G([0, 1]), "pipe": None, "data": G([0, 2])}

    h = H()
    h._groups["pipe_bwd"] = h._groups["model"]   # same communicator: counted once
    inv = streams.inventory(h)
    names = [n for n, _ in inv]
    assert names[0] == "compute"
    assert sum(1 for n in names if n.startswith("rccl:")) == 2
    assert all(p for n, p in inv if n.startswith("rccl:"))


def _world_flag_worker(rank, world):
    # ranks with and without communicators (as pipeline stages have) must
    # agree on whether the world MAX of the one-shot error flag runs
    from types import SimpleNamespace as NS
    from fleetx_amd.parallel import comm
    import os
    comm._COMMS.clear()
    if rank == 0:
        comm._COMMS[(0, 1)] = NS(tried_oneshot=True, oneshot=None)
    res = [comm.world_oneshot_possible()]
    os.environ["FLEETX_ONESHOT_FORCE"] = "1"
    torch.cuda.is_available = lambda: True  # what the GPU box reports
    res.append(comm.world_oneshot_possible())
    os.environ["FLEETX_ONESHOT"] = "0"
    res.append(comm.world_oneshot_possible())
    comm._COMMS.clear()
    return res


def test_world_error_flag_decision_is_rank_invariant():
    res = dist_utils.run(_world_flag_worker, 2)
    assert res[0] == res[1] == [False, True, False], res

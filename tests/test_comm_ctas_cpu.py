"""Per-communicator RCCL CTA budget (``Distributed.comm.ctas``): parsing, and
that the options reach ``new_group`` for every group of the hybrid topology.

Reference collective call sites the groups serve: ``eager_engine.py:386-396``
(DP/sharding reductions), ``tensor_fusion_helper.py:119-127`` (fused buckets),
``sequence_parallel_utils.py:55,69,139`` (TP/SP).
"""
import pytest

from fleetx_amd.parallel import topology as topo
from tests import dist_utils


def test_parse_defaults_and_overrides():
    assert topo.parse_ctas(None) == {} and topo.parse_ctas({}) == {}   # opt-in
    d = topo.parse_ctas("preset")
    assert d == topo.parse_ctas(True)
    assert d["model"] == (32, 64) and d["data"] == (8, 16) and d["check"] == (1, 4)
    assert d["pipe_bwd"] == d["pipe"]
    o = topo.parse_ctas({"dp": "4,8", "mp": 48, "pp": [2, 4], "check": None})
    assert o["data"] == (4, 8) and o["model"] == (None, 48) and o["pipe"] == (2, 4)
    assert "check" not in o and o["pipe_bwd"] == (2, 4)
    assert topo.parse_ctas(False) == {}
    with pytest.raises(ValueError):
        topo.parse_ctas({"bogus": 4})
    with pytest.raises(ValueError):
        topo.parse_ctas({"dp": "16,8"})


def test_nccl_options_carry_budget():
    o = topo.nccl_options((8, 16))
    assert o.config.min_ctas == 8 and o.config.max_ctas == 16
    assert topo.nccl_options(None) is None


def _build(rank, world, ctas):
    import torch.distributed as dist
    seen = []
    real = dist.new_group

    def fake_new_group(ranks=None, pg_options=None, **kw):
        if pg_options is not None:
            lo, hi = pg_options.config.min_ctas, pg_options.config.max_ctas
            seen.append((tuple(ranks), lo if lo > 0 else None, hi if hi > 0 else None))
        elif kw.get("backend") is None:
            seen.append((tuple(ranks), None, None))
        return real(ranks=ranks, **kw)

    topo.dist.new_group = fake_new_group
    topo.dist.get_backend = lambda *a, **k: "nccl"     # pretend RCCL for the options path
    topo.reset_hcg()
    hcg = topo.init_hcg(dp=2, mp=2, pp=2, ctas=ctas)
    from fleetx_amd.utils.streams import inventory
    names = [n for n, _ in inventory(hcg)]
    return {"seen": seen, "inv": names}


def test_options_reach_new_group():
    res = dist_utils.run(_build, 8, {"dp": "4,12"})
    seen = res[0]["seen"]
    # the axis groups are built in order data, pipe, sharding(1: none), model
    by = {}
    for ranks, lo, hi in seen:
        by.setdefault((lo, hi), []).append(ranks)
    assert (4, 12) in by and (0, 4) in by[(4, 12)]          # dp groups: ranks differ by 4
    # mp groups (adjacent ranks): a TP-2 pair is one xGMI link -> small budget
    assert (8, 16) in by and (0, 1) in by[(8, 16)]
    assert (4, 16) in by and (0, 2) in by[(4, 16)]          # pp groups
    assert any("rccl:model[0, 1](ctas 8-16)" == n for n in res[0]["inv"])


def test_model_budget_scales_with_group_size():
    assert topo.model_ctas(2) == (8, 16)
    assert topo.model_ctas(4) == (16, 32)
    assert topo.model_ctas(8) == topo.DEFAULT_CTAS["model"] == (32, 64)


def test_default_topology_sets_no_group_budget():
    """Budgets are opt-in: without ``Distributed.comm.ctas`` no group carries
    options (the process-wide NCCL_MIN_NCHANNELS floor applies)."""
    res = dist_utils.run(_build, 8, None)
    assert all(lo is None and hi is None for _, lo, hi in res[0]["seen"])
    from fleetx_amd.utils import env
    assert env.DEFAULT_RCCL_ENV.get("NCCL_MIN_NCHANNELS") == "32"

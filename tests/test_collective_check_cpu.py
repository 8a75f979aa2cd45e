"""Collective fingerprint checker: matching collectives pass,
a rank that diverges (shape / op order) is reported on every rank instead of
hanging."""
import torch

from tests import dist_utils


def _run(rank, world, diverge):
    import torch.distributed as dist
    from fleetx_amd.parallel import topology as topo
    from fleetx_amd.parallel import collective_check as cc
    topo.reset_hcg()
    hcg = topo.init_hcg(dp=2)
    assert cc.enable(hcg)
    g = hcg.get_data_parallel_group().group
    t = torch.ones(4)
    dist.all_reduce(t, group=g)
    out = {"ok": float(t[0])}
    x = torch.ones(5 if (diverge and rank == 1) else 4)
    try:
        dist.all_reduce(x, group=g)
        out["err"] = None
    except cc.CollectiveMismatch as e:
        out["err"] = str(e)
    cc.disable()
    return out


def test_matching_collectives_pass():
    for r in dist_utils.run(_run, 2, False):
        assert r["ok"] == 2.0 and r["err"] is None


def test_divergent_shape_is_reported_on_every_rank():
    res = dist_utils.run(_run, 2, True)
    for r in res:
        assert r["err"] is not None
        assert "rank 0: #1 all_reduce float32 (4,)" in r["err"]
        assert "rank 1: #1 all_reduce float32 (5,)" in r["err"]

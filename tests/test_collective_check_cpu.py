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


def _run_p2p(rank, world, diverge):
    """A 1F1B step over a pp2 gloo pipe with p2p fingerprinting on; with
    ``diverge`` stage 1 expects a wrong activation shape."""
    from fleetx_amd.parallel import topology as topo
    from fleetx_amd.parallel import collective_check as cc
    from fleetx_amd.parallel.pipeline import PipelineSchedule
    topo.reset_hcg()
    hcg = topo.init_hcg(pp=2)
    assert cc.enable(hcg)
    shape = (2, 3) if not (diverge and rank == 1) else (2, 4)
    w = torch.nn.Parameter(torch.full((2, 3), 2.0))
    sched = PipelineSchedule(hcg, lambda: shape, torch.float32, "cpu")

    def fn(c, k, x):
        if rank == 0:
            return w * float(k + 1)
        return (x * w[:, :1]).sum()

    out = {}
    try:
        loss = sched.train_1f1b(4, fn)
        out["loss"] = None if loss is None else float(loss)
        out["err"] = None
    except (cc.CollectiveMismatch, RuntimeError) as e:   # the peer of a refused rank loses it
        out["err"] = str(e)
    cc.disable()
    return out


def test_p2p_fingerprints_pass_on_matching_pipeline():
    res = dist_utils.run(_run_p2p, 2, False)
    assert all(r["err"] is None for r in res)
    assert res[1]["loss"] == 4.0 * 6 * (1 + 2 + 3 + 4)


def test_p2p_shape_mismatch_is_named():
    res = dist_utils.run(_run_p2p, 2, True)
    assert "rank 1 expects to receive #0 float32 (2, 4) from rank 0, which sent #0 float32 (2, 3)" \
        in res[1]["err"]

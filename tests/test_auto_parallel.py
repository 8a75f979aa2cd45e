"""Auto-parallel front end (reference C05/C11/C16/C22/C32, P10): mesh
construction, annotations, the MI355X layout planner, and tools/auto.py
end-to-end (semi: single process; full: gloo world of 2 with the planner)."""
import os

import pytest
import torch

from fleetx_amd.parallel.auto.mesh import Mesh, ProcessMesh, shard_tensor, shard_op
from fleetx_amd.parallel.auto import planner as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AUTO = os.path.join(ROOT, "fleetx_amd/configs/nlp/gpt/auto")
TINY = ["Model.hidden_size=64", "Model.num_layers=2", "Model.num_attention_heads=4",
        "Model.ffn_hidden_size=256", "Model.vocab_size=128", "Model.max_position_embeddings=64",
        "Global.device=cpu", "Engine.max_steps=3", "Engine.eval_freq=2", "Engine.eval_iters=1",
        "Global.local_batch_size=4", "Global.micro_batch_size=2",
        "Data.Train.dataset.name=SyntheticGPTDataset", "Data.Train.dataset.max_seq_len=32",
        "Data.Train.dataset.vocab_size=128", "Data.Eval.dataset.name=SyntheticGPTDataset",
        "Data.Eval.dataset.max_seq_len=32", "Data.Eval.dataset.vocab_size=128"]


def test_mesh_layouts():
    m = Mesh(dict(pp_degree=2, dp_degree=2, mp_degree=2))
    assert m.process_mesh.dim_names == ["pp", "dp", "mp"] and m.process_mesh.shape == [2, 2, 2]
    assert m[1].process_ids == [4, 5, 6, 7] and m[1].dim_names == ["dp", "mp"]
    assert m.stages(8) == [0, 0, 0, 0, 1, 1, 1, 1]
    m2 = Mesh(dict(pp_degree=1, dp_degree=4, mp_degree=1))
    assert m2.dp == "dp" and m2.mp is None and m2[0] == m2.process_mesh
    serial = Mesh(dict(pp_degree=1, dp_degree=1, mp_degree=1))
    assert serial.process_mesh.process_ids == [0]
    pm = ProcessMesh([[0, 1], [2, 3]], ["dp", "mp"])
    t = shard_tensor(torch.zeros(4, 6), pm, [None, "mp"])
    assert t._fx_dist[1] == [None, "mp"]
    with pytest.raises(AssertionError):
        shard_tensor(torch.zeros(4), pm, ["pp"])
    f = shard_op(lambda a: a * 2, pm, out_specs=[["dp", None]])
    assert f(torch.ones(2, 2))._fx_dist[1] == ["dp", None]


def test_planner_respects_memory_and_links():
    p1 = P.plan(4096, 32, 32, 50304, 1024, 8, 1)
    assert (p1.dp, p1.mp, p1.pp) == (1, 1, 1) and p1.est_mem_gb < 288
    p8 = P.plan(4096, 32, 32, 50304, 1024, 64, 8)
    assert p8.dp * p8.mp * p8.pp * p8.sharding == 8
    # TP-2 over one xGMI link is never better than the chosen plan
    t_tp2 = P.estimate(4096, 32, 32, 50304, 1024, 64, 2, 2, 2, 1, 0, 2, False)[0]
    assert p8.est_step_s <= t_tp2
    # a ~30B model needs its weights/optimizer states split across GPUs
    big = P.plan(7168, 48, 56, 51200, 2048, 64, 8)
    assert big.mp * big.pp > 1 or big.sharding > 1
    assert big.est_mem_gb < 288
    # 175B with fp32 Adam states does not fit one node without offload
    with pytest.raises(ValueError):
        P.plan(12288, 96, 96, 51200, 2048, 8, 8)


def test_auto_semi_single_process(tmp_path):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import auto as auto_tool
    eng = auto_tool.main(["-c", os.path.join(AUTO, "pretrain_gpt_345M_single_card.yaml")] +
                         sum([["-o", o] for o in TINY + ["Engine.save_load.output_dir=%s" % tmp_path]],
                             []))
    eng.save(epoch=0, step=3)
    assert os.path.isdir(tmp_path / "auto")


def _auto_full_worker(rank, world, tmp):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import auto as auto_tool
    ov = TINY + ["Engine.auto_mode=full", "Engine.save_load.output_dir=%s" % tmp]
    eng = auto_tool.main(["-c", os.path.join(AUTO, "pretrain_gpt_1.3B_dp8.yaml")] +
                         sum([["-o", o] for o in ov], []))
    d = eng.engine._configs.Distributed
    assert d.dp_degree * d.mp_degree * d.pp_degree * d.sharding.sharding_degree == world


def test_auto_full_gloo_world2(tmp_path):
    from tests.dist_utils import run
    run(_auto_full_worker, 2, str(tmp_path))


def _lowering_worker(rank, world, mp, pp, bad):
    """Semi-auto lowering: the per-rank model equals the annotated serial
    network split by its specs (gathered shards == serial weights, gathered
    vocab-parallel logits == serial logits); a wrong annotation is refused."""
    import torch.distributed as dist
    from fleetx_amd.utils import config as cfgmod
    from fleetx_amd.utils import env
    from fleetx_amd.models import build_module
    from fleetx_amd.models.language_model.gpt.auto import auto_module as am
    from fleetx_amd.parallel import topology as topo
    topo.reset_hcg()
    ov = TINY + ["Distributed.mp_degree=%d" % mp, "Distributed.pp_degree=%d" % pp,
                 "Distributed.dp_degree=1", "Model.hidden_dropout_prob=0.0",
                 "Model.attention_probs_dropout_prob=0.0", "Global.global_batch_size=4"]
    cfg = cfgmod.get_auto_config(os.path.join(AUTO, "pretrain_gpt_345M_single_card.yaml"),
                                 overrides=ov, show=False)
    env.init_dist_env(cfg)
    env.set_seed(cfg.Global.seed)
    if bad:
        orig = am.annotate_gpt

        def wrong(model, mesh):
            n = orig(model, mesh)
            for name, mod in model.named_modules():
                if name.endswith("fc1"):
                    shard_tensor(mod.weight, mesh.process_mesh, ["mp", None])  # row, not column
            return n
        am.annotate_gpt = wrong
        try:
            build_module(cfg).get_model()
        except ValueError as e:
            return {"refused": str(e)}
        finally:
            am.annotate_gpt = orig
        return {"refused": None}
    module = build_module(cfg)
    model = module.get_model()
    serial = module._serial_model()
    hcg = topo.get_hcg()
    out = {"layout": {k: v for k, v in module.auto_layout.items() if k != "stages"},
           "nstages": len(module.auto_layout["stages"])}
    if mp > 1:
        w = model.gpt.layers[0].mlp.fc1.weight.detach()
        parts = [torch.empty_like(w) for _ in range(mp)]
        dist.all_gather(parts, w.contiguous())
        out["fc1_ok"] = torch.equal(torch.cat(parts, 0), serial.gpt.layers[0].mlp.fc1.weight)
        w2 = model.gpt.layers[1].attn.out_proj.weight.detach()
        parts = [torch.empty_like(w2) for _ in range(mp)]
        dist.all_gather(parts, w2.contiguous())
        out["out_ok"] = torch.equal(torch.cat(parts, 1), serial.gpt.layers[1].attn.out_proj.weight)
        model.eval()
        serial.eval()
        toks = torch.randint(0, 128, (2, 16), generator=torch.Generator().manual_seed(3))
        with torch.no_grad():
            lg = model(toks)
            parts = [torch.empty_like(lg) for _ in range(mp)]
            dist.all_gather(parts, lg.contiguous())
            with topo.serial_scope():
                ref = serial(toks)
        out["logit_err"] = (torch.cat(parts, -1) - ref).abs().max().item()
    else:
        # pipeline: every stage holds exactly its annotated layers' serial weights
        names = [n for n, _ in model.named_parameters()]
        out["n_params"] = len(names)
        out["stage"] = hcg.pp_rank
    return out


@pytest.mark.parametrize("mp,pp", [(2, 1), (1, 2)])
def test_semi_auto_lowering_matches_serial(mp, pp):
    from tests.dist_utils import run
    res = run(_lowering_worker, 2, mp, pp, False)
    for r in res:
        assert r["layout"]["tp_degree"] == mp and r["layout"]["lowered"] > 0
        assert r["nstages"] == 2
        if mp > 1:
            assert r["fc1_ok"] and r["out_ok"]
            assert r["logit_err"] < 1e-4, r["logit_err"]


def test_semi_auto_wrong_annotation_refused():
    from tests.dist_utils import run
    res = run(_lowering_worker, 2, 2, 1, True)
    for r in res:
        assert r["refused"] and "fc1" in r["refused"], r


def test_175B_tp8_zero3_recipe_fits_hbm():
    """BASELINE config 4: the 175B shape with TP8 + ZeRO-3 (+ recompute) is
    sized for 288 GB per GPU on 16 nodes; one node alone cannot hold it."""
    from fleetx_amd.utils import config as C
    cfg = C.get_config(os.path.join(ROOT, "fleetx_amd/configs/nlp/gpt/"
                                    "pretrain_gpt_175B_tp8_sharding16_stage3.yaml"), nranks=128)
    d, m = cfg.Distributed, cfg.Model
    assert d.mp_degree * d.sharding.sharding_degree * d.dp_degree * d.pp_degree == 128
    est = P.estimate(m.hidden_size, m.num_layers, m.num_attention_heads, m.vocab_size,
                     m.max_position_embeddings, cfg.Global.global_batch_size, d.dp_degree,
                     d.mp_degree, d.pp_degree, d.sharding.sharding_degree,
                     d.sharding.sharding_stage, cfg.Global.micro_batch_size, True)
    assert est is not None and est[1] < P.HBM_BYTES * P.USABLE
    assert est[1] < 60e9  # stage 3 keeps ~1/128 of the states per GPU
    with pytest.raises(ValueError):
        P.plan(12288, 96, 96, 51200, 2048, 8, 8)

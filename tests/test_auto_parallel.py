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

"""Layout equivalence on CPU/gloo: DP, TP, SP, PP (1F1B, interleaved), ZeRO
and hybrids must reproduce the single-process loss curve (dropout off, fp32).

Reference behaviour being matched: SURVEY.md §7.2 phase 4/5/6 exit checks
("mp, dp, +/-SP give the same loss curve as 1 GPU for a fixed seed").
"""
import os

import pytest
import torch

from tests import dist_utils

CFG = os.path.join(os.path.dirname(__file__), "..", "fleetx_amd", "configs", "nlp", "gpt",
                   "pretrain_gpt_345M_single_card.yaml")
GBS, SEQ, VOCAB = 8, 32, 512


def _global_batch():
    g = torch.Generator().manual_seed(7)
    toks = torch.randint(0, VOCAB, (3, GBS, SEQ + 1), generator=g)
    return toks


def _train(rank, world, layout, steps=3, extra=()):
    from fleetx_amd.utils import config as C
    from fleetx_amd.utils import env
    from fleetx_amd.models import build_module
    from fleetx_amd.core.engine.eager_engine import EagerEngine
    from fleetx_amd.parallel import topology as topo
    dp, mp, pp, sd, stage, micro, sp, vpp = layout
    topo.reset_hcg()
    local = GBS // (dp * sd)
    ov = ["Model.hidden_size=64", "Model.num_layers=4", "Model.num_attention_heads=4",
          "Model.vocab_size=%d" % VOCAB, "Model.hidden_dropout_prob=0.0",
          "Model.attention_probs_dropout_prob=0.0", "Model.max_position_embeddings=64",
          "Model.sequence_parallel=%s" % sp, "Global.device=cpu",
          "Global.local_batch_size=%d" % local, "Global.micro_batch_size=%d" % micro,
          "Distributed.dp_degree=%d" % dp, "Distributed.mp_degree=%d" % mp,
          "Distributed.pp_degree=%d" % pp, "Distributed.sharding.sharding_degree=%d" % sd,
          "Distributed.sharding.sharding_stage=%d" % stage,
          "Optimizer.lr.name=ConstantLR", "Optimizer.lr.learning_rate=0.01",
          "Engine.max_steps=10", "Engine.mix_precision.use_pure_fp16=False",
          "Data.Train.dataset.name=SyntheticGPTDataset"] + list(extra)
    if vpp > 1:
        ov.append("Model.virtual_pp_degree=%d" % vpp)
    for k in ("decay_steps", "warmup_rate", "max_lr", "min_lr"):
        pass
    cfg = C.get_config(CFG, overrides=ov, nranks=world)
    cfg.Optimizer.lr = {"name": "ConstantLR", "learning_rate": 0.01}
    env.init_dist_env(cfg, backend="gloo")
    env.set_seed(cfg.Global.seed)
    module = build_module(cfg)
    eng = EagerEngine(configs=cfg, module=module, mode="train")
    hcg = eng.hcg
    drank = hcg.dp_rank * hcg.sharding_degree + hcg.sharding_rank
    toks = _global_batch()
    losses, norms = [], []
    for s in range(steps):
        t = toks[0, drank * local:(drank + 1) * local]
        batch = [t[:, :-1].contiguous(), torch.arange(SEQ).expand(local, SEQ).contiguous(),
                 t[:, 1:].contiguous(), torch.ones(local, SEQ)]
        loss = eng._fit_impl(batch)
        losses.append(eng._reduce_log_loss(loss, 1))
        norms.append(float(eng.optimizer.last_grad_norm))
    return {"losses": losses, "norms": norms, "drank": drank, "mp": hcg.mp_rank, "pp": hcg.pp_rank}


def _single(extra=()):
    r = dist_utils.run(_train, 1, (1, 1, 1, 1, 0, GBS, False, 1), 3, tuple(extra))
    return r[0]["losses"]


@pytest.fixture(scope="module")
def ref_losses():
    return _single()


def _avg_over_data(results):
    by = {}
    for r in results:
        by.setdefault(r["drank"], r["losses"])
    n = len(by)
    return [sum(v[i] for v in by.values()) / n for i in range(len(next(iter(by.values()))))]


def _check(results, ref, tol=2e-4):
    got = _avg_over_data(results)
    for a, b in zip(got, ref):
        assert abs(a - b) < tol * max(1.0, abs(b)), (got, ref)


def test_single_process_loss_decreases(ref_losses):
    assert ref_losses[2] < ref_losses[0]


def test_data_parallel(ref_losses):
    _check(dist_utils.run(_train, 2, (2, 1, 1, 1, 0, 4, False, 1)), ref_losses)


def test_grad_accumulation(ref_losses):
    _check(dist_utils.run(_train, 1, (1, 1, 1, 1, 0, 2, False, 1)), ref_losses)


def test_tensor_parallel(ref_losses):
    _check(dist_utils.run(_train, 2, (1, 2, 1, 1, 0, GBS, False, 1)), ref_losses)


def test_sequence_parallel(ref_losses):
    _check(dist_utils.run(_train, 2, (1, 2, 1, 1, 0, GBS, True, 1)), ref_losses)


def test_pipeline_1f1b(ref_losses):
    _check(dist_utils.run(_train, 2, (1, 1, 2, 1, 0, 2, False, 1)), ref_losses)


def test_pipeline_interleaved(ref_losses):
    _check(dist_utils.run(_train, 2, (1, 1, 2, 1, 0, 2, False, 2)), ref_losses)


def test_sharding_stage1(ref_losses):
    _check(dist_utils.run(_train, 2, (1, 1, 1, 2, 1, 4, False, 1)), ref_losses)


def test_sharding_stage2(ref_losses):
    _check(dist_utils.run(_train, 2, (1, 1, 1, 2, 2, 4, False, 1)), ref_losses)


def test_hybrid_tp_pp_dp(ref_losses):
    _check(dist_utils.run(_train, 8, (2, 2, 2, 1, 0, 2, False, 1)), ref_losses)

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
    from fleetx_amd.parallel.state_gather import gather_master_state
    master0 = gather_master_state(eng)
    for s in range(steps):
        t = toks[0, drank * local:(drank + 1) * local]
        batch = [t[:, :-1].contiguous(), torch.arange(SEQ).expand(local, SEQ).contiguous(),
                 t[:, 1:].contiguous(), torch.ones(local, SEQ)]
        loss = eng._fit_impl(batch)
        losses.append(eng._reduce_log_loss(loss, 1))
        norms.append(float(eng.optimizer.last_grad_norm))
    return {"losses": losses, "norms": norms, "drank": drank, "mp": hcg.mp_rank, "pp": hcg.pp_rank,
            "master": gather_master_state(eng), "master0": master0 if rank == 0 else None}


def _single(extra=()):
    r = dist_utils.run(_train, 1, (1, 1, 1, 1, 0, GBS, False, 1), 3, tuple(extra))
    return r[0]


class _Ref(list):
    """Reference loss curve (a list) carrying the single-process master
    weights before (``master0``) and after (``master``) the steps."""


@pytest.fixture(scope="module")
def ref_losses():
    r = _single()
    ref = _Ref(r["losses"])
    ref.master, ref.master0 = r["master"], r["master0"]
    return ref


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
    if isinstance(ref, _Ref):
        check_master_per_tensor(results[0]["master"], ref.master, ref.master0, rel=20 * tol)


def _drop_key_bias(t, heads):
    """The key third of a packed [heads][3][head_dim] qkv bias, zeroed: its
    exact gradient is 0 (a per-row constant under the softmax), so what Adam
    makes of the rounding noise there differs between any two runs."""
    t = t.clone()
    t.view(heads, 3, -1)[:, 1] = 0
    return t


def check_master_per_tensor(got, ref, ref0, rel, heads=4):
    """Every fp32 master tensor, gathered into the single-rank layout
    (TP shards concatenated along their split dim, ZeRO slices assembled,
    pipeline stage names mapped to global layers), against the single-rank
    run: ||w - w_ref|| <= rel * ||w_ref - w_init|| + 1e-3 ||w_ref|| per
    tensor, so a permuted or misplaced shard (same norm, wrong place: error
    ~ ||w||) fails."""
    names = set(k.replace("#tied", "") for k in got)
    assert names == set(ref), (sorted(names ^ set(ref)))
    for k, w in got.items():
        base = k.replace("#tied", "")
        r, r0 = ref[base], ref0[base]
        if "qkv" in base and base.endswith("bias"):
            w, r, r0 = (_drop_key_bias(x, heads) for x in (w, r, r0))
        assert w.shape == r.shape, (k, w.shape, r.shape)
        upd = float((r - r0).norm())
        err = float((w - r).norm())
        assert err <= rel * upd + 1e-3 * float(r.norm()), (k, err, upd)


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


@pytest.mark.parametrize("extra", [("Distributed.comm.sp_chunks=4",),
                                   ("Distributed.comm.tp_overlap=False",)])
def test_sequence_parallel_overlap_variants(ref_losses, extra):
    """Chunked overlapped SP linears (4 chunks) and the plain gather/scatter path."""
    _check(dist_utils.run(_train, 2, (1, 2, 1, 1, 0, GBS, True, 1), 3, extra), ref_losses)


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


def test_sharding_stage1_dp_accumulation(ref_losses):
    # dp2 x sharding2 ZeRO-1, two micro-batches per rank, overlapped param gather
    _check(dist_utils.run(_train, 4, (2, 1, 1, 2, 1, 1, False, 1)), ref_losses)


# ---------------------------------------------------------------- ZeRO stage 3
def test_sharding_stage3(ref_losses):
    _check(dist_utils.run(_train, 2, (1, 1, 1, 2, 3, 4, False, 1)), ref_losses)


def test_sharding_stage3_dp_and_accumulation(ref_losses):
    # dp2 x sharding2, micro 1 -> 2 accumulation steps per rank
    _check(dist_utils.run(_train, 4, (2, 1, 1, 2, 3, 1, False, 1)), ref_losses)


def test_sharding_stage3_recompute(ref_losses):
    _check(dist_utils.run(_train, 2, (1, 1, 1, 2, 3, 4, False, 1), 3,
                          ("Model.use_recompute=True",)), ref_losses)


def test_sharding_stage3_with_tp(ref_losses):
    _check(dist_utils.run(_train, 4, (1, 2, 1, 2, 3, 4, False, 1)), ref_losses)


def test_sharding_stage2_dp_and_accumulation(ref_losses):
    # ZeRO-2 (owned fp32 grad shards, whole params), 2 accumulation steps
    _check(dist_utils.run(_train, 4, (2, 1, 1, 2, 2, 1, False, 1)), ref_losses)


@pytest.mark.parametrize("layout", [(2, 1, 1, 1, 0, 4, False, 1), (1, 1, 1, 2, 1, 4, False, 1),
                                    (1, 1, 1, 2, 2, 4, False, 1)])
def test_reduce_dtype_bf16(ref_losses, layout):
    """Distributed.comm.reduce_dtype=bfloat16: 16-bit gradient reductions
    (reference fp16 all-reduce) stay within bf16 rounding of the fp32 curve."""
    out = dist_utils.run(_train, 2, layout, 3, ("Distributed.comm.reduce_dtype=bfloat16",))
    _check(out, ref_losses, tol=5e-3)


def _stage3_memory_and_resume(rank, world, outdir, stage=3):
    """Shards are 1/n of the model; save gathers full params; a fresh
    engine that loads the checkpoint continues the identical loss curve."""
    from fleetx_amd.utils import config as C
    from fleetx_amd.utils import env
    from fleetx_amd.models import build_module
    from fleetx_amd.core.engine.eager_engine import EagerEngine
    from fleetx_amd.parallel import topology as topo

    def make(extra=()):
        topo.reset_hcg()
        ov = ["Model.hidden_size=64", "Model.num_layers=4", "Model.num_attention_heads=4",
              "Model.vocab_size=%d" % VOCAB, "Model.hidden_dropout_prob=0.0",
              "Model.attention_probs_dropout_prob=0.0", "Model.max_position_embeddings=64",
              "Global.device=cpu", "Global.local_batch_size=4", "Global.micro_batch_size=4",
              "Distributed.dp_degree=1", "Distributed.sharding.sharding_degree=2",
              "Distributed.sharding.sharding_stage=%d" % stage, "Engine.max_steps=10",
              "Engine.save_load.output_dir=%s" % outdir,
              "Data.Train.dataset.name=SyntheticGPTDataset"] + list(extra)
        cfg = C.get_config(CFG, overrides=ov, nranks=world)
        cfg.Optimizer.lr = {"name": "ConstantLR", "learning_rate": 0.01}
        env.init_dist_env(cfg, backend="gloo")
        env.set_seed(cfg.Global.seed)
        return EagerEngine(configs=cfg, module=build_module(cfg), mode="train")

    toks = _global_batch()

    def batch(s):
        t = toks[s % 3, rank * 4:(rank + 1) * 4]
        return [t[:, :-1].contiguous(), torch.arange(SEQ).expand(4, SEQ).contiguous(),
                t[:, 1:].contiguous(), torch.ones(4, SEQ)]

    eng = make()
    rep = eng.buffer.memory_report()
    for s in range(2):
        eng._fit_impl(batch(s))
    eng.save(epoch=0, step=2)
    cont = [eng._reduce_log_loss(eng._fit_impl(batch(s)), 1) for s in (2, 3)]
    ck = os.path.join(outdir, "epoch_0_step_2")
    eng2 = make(["Engine.save_load.ckpt_dir=%s" % ck])
    eng2.load()
    res = [eng2._reduce_log_loss(eng2._fit_impl(batch(s)), 1) for s in (2, 3)]
    return {"rep": rep, "cont": cont, "res": res}


@pytest.mark.parametrize("stage", [2, 3])
def test_sharding_memory_and_resume(tmp_path, stage):
    out = dist_utils.run(_stage3_memory_and_resume, 2, str(tmp_path), stage)
    for r in out:
        rep = r["rep"]
        assert rep["stage"] == stage
        # ZeRO-2 and 3 keep only the owned fp32 gradient shard
        assert rep["shard_grad_bytes"] * 2 == rep["unsharded_grad_bytes"]
        if stage == 3:
            assert rep["resident_param_bytes"] * 2 == rep["unsharded_param_bytes"]
        else:
            assert rep["resident_param_bytes"] == rep["unsharded_param_bytes"]
        for a, b in zip(r["cont"], r["res"]):
            assert abs(a - b) < 1e-6, (r["cont"], r["res"])
    assert (tmp_path / "epoch_0_step_2" / "mp_00_sharding_01_pp_00" / "model.pdparams").exists()


# ------------------------------------------- RCCL collective forms on gloo
@pytest.mark.parametrize("stage,dp,micro", [(1, 1, 4), (2, 1, 4), (3, 1, 4), (1, 2, 1)])
def test_sharding_rccl_collective_forms(ref_losses, monkeypatch, stage, dp, micro):
    """The in-place reduce_scatter_tensor / all_gather_into_tensor calls the
    RCCL path issues (gloo otherwise takes all_reduce stand-ins)."""
    monkeypatch.setenv("FLEETX_GLOO_AS_RCCL", "1")
    world = 2 * dp
    _check(dist_utils.run(_train, world, (dp, 1, 1, 2, stage, micro, False, 1)), ref_losses)


@pytest.mark.parametrize("layout", [(2, 1, 1, 1, 0, 4, False, 1), (1, 2, 1, 2, 2, 4, False, 1)])
def test_fingerprint_mode_trains_identically(ref_losses, layout):
    """Distributed.debug=fingerprint checks every collective of a real step."""
    world = layout[0] * layout[1] * layout[2] * layout[3]
    _check(dist_utils.run(_train, world, layout, 3, ("Distributed.debug=fingerprint",)),
           ref_losses)


@pytest.mark.parametrize("layout", [(1, 2, 1, 1, 0, GBS, False, 1), (1, 2, 1, 1, 0, GBS, True, 1),
                                    (2, 1, 1, 1, 0, 2, False, 1)])
def test_fused_lm_head_ce(ref_losses, layout, monkeypatch):
    """LM head + CE chunked over tokens (ops/lm_head_ce.py) on a vocab-parallel
    head (TP2, TP2 + SP) and under DP with accumulation: the plain head's
    loss curve."""
    monkeypatch.setenv("FLEETX_LM_HEAD_CE_CHUNK", "48")
    _check(dist_utils.run(_train, 2, layout, 3, ("Model.fused_lm_head_ce=True",)), ref_losses)


def test_per_tensor_check_catches_a_permuted_shard():
    """The per-tensor comparison fails on a tensor whose two TP halves were
    concatenated in the wrong order (same values, same norm)."""
    torch.manual_seed(0)
    w0 = {"a": torch.randn(8, 4) * 0.02, "b": torch.zeros(8)}
    ref = {k: v + 0.01 * torch.randn_like(v) for k, v in w0.items()}
    check_master_per_tensor(dict(ref), ref, w0, rel=0.05)
    bad = dict(ref)
    bad["a"] = torch.cat([ref["a"][4:], ref["a"][:4]])
    with pytest.raises(AssertionError):
        check_master_per_tensor(bad, ref, w0, rel=0.05)

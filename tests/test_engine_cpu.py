"""Engine-level CPU tests: recompute equivalence, checkpoint save/load/resume
layout (reference §5.4), fp32 CPU training via tools/train.py (BASELINE
config #1 plumbing), LR schedules, RNG streams."""
import math
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = os.path.join(ROOT, "fleetx_amd", "configs", "nlp", "gpt", "pretrain_gpt_345M_single_card.yaml")


def _engine(tmp_path, extra=()):
    from fleetx_amd.utils import config as C
    from fleetx_amd.utils import env
    from fleetx_amd.models import build_module
    from fleetx_amd.core.engine.eager_engine import EagerEngine
    ov = ["Model.hidden_size=64", "Model.num_layers=2", "Model.num_attention_heads=4",
          "Model.vocab_size=256", "Model.max_position_embeddings=64", "Global.device=cpu",
          "Global.local_batch_size=4", "Global.micro_batch_size=4",
          "Engine.save_load.output_dir=%s" % tmp_path, "Engine.max_steps=100",
          "Data.Train.dataset.name=SyntheticGPTDataset"] + list(extra)
    cfg = C.get_config(CFG, overrides=ov, nranks=1)
    env.set_seed(cfg.Global.seed)
    return EagerEngine(configs=cfg, module=build_module(cfg), mode="train"), cfg


def _batch(seed):
    g = torch.Generator().manual_seed(seed)
    t = torch.randint(0, 256, (4, 33), generator=g)
    return [t[:, :-1].contiguous(), torch.arange(32).expand(4, 32).contiguous(),
            t[:, 1:].contiguous(), torch.ones(4, 32)]


@pytest.mark.parametrize("gran", ["full", "full_attn", "core_attn"])
def test_recompute_matches_no_recompute(tmp_path, gran):
    e1, _ = _engine(tmp_path / "a")
    l1 = [float(e1._fit_impl(_batch(i))) for i in range(3)]
    e2, _ = _engine(tmp_path / "b", ["Model.use_recompute=True",
                                      "Model.recompute_granularity=%s" % gran])
    l2 = [float(e2._fit_impl(_batch(i))) for i in range(3)]
    for a, b in zip(l1, l2):
        assert abs(a - b) < 1e-5, (l1, l2)


def test_checkpoint_layout_and_resume(tmp_path):
    e1, cfg = _engine(tmp_path)
    for i in range(2):
        e1._fit_impl(_batch(i))
    e1.consumed_samples = 8
    e1.save(epoch=0, step=2)
    d = tmp_path / "epoch_0_step_2"
    assert (d / "model.pdparams").exists() and (d / "model_state.pdopt").exists()
    assert (d / "meta_state.pdopt").exists()
    cont = [float(e1._fit_impl(_batch(i))) for i in (2, 3)]
    e2, _ = _engine(tmp_path, ["Engine.save_load.ckpt_dir=%s" % d])
    e2.load()
    assert e2.consumed_samples == 8 and e2._load_recovery["step"] == 2
    res = [float(e2._fit_impl(_batch(i))) for i in (2, 3)]
    for a, b in zip(cont, res):
        assert abs(a - b) < 1e-6, (cont, res)


def test_dropout_rng_replay_after_resume(tmp_path):
    # with dropout on, resumed training must reproduce the masks
    e1, _ = _engine(tmp_path, ["Model.hidden_dropout_prob=0.1",
                               "Model.attention_probs_dropout_prob=0.1"])
    e1._fit_impl(_batch(0))
    e1.save(epoch=0, step=1)
    a = float(e1._fit_impl(_batch(1)))
    e2, _ = _engine(tmp_path, ["Model.hidden_dropout_prob=0.1",
                               "Model.attention_probs_dropout_prob=0.1",
                               "Engine.save_load.ckpt_dir=%s" % (tmp_path / "epoch_0_step_1")])
    e2.load()
    b = float(e2._fit_impl(_batch(1)))
    assert abs(a - b) < 1e-6


def test_lr_schedules():
    from fleetx_amd.optims.lr_scheduler import CosineAnnealingWithWarmupDecay, ViTLRScheduler
    s = CosineAnnealingWithWarmupDecay(max_lr=1.0, min_lr=0.1, warmup_rate=0.1, decay_steps=100)
    assert abs(s() - 0.1) < 1e-9  # Paddle semantics: first lr at last_epoch = 1
    for _ in range(9):
        s.step()
    assert abs(s() - 1.0) < 1e-9
    for _ in range(45):
        s.step()
    assert abs(s() - (0.1 + 0.5 * (math.cos(math.pi * 0.5) + 1) * 0.9)) < 1e-9
    for _ in range(100):
        s.step()
    assert s() == 0.1
    v = ViTLRScheduler(learning_rate=1.0, step_each_epoch=10, epochs=2, warmup_steps=5)
    assert 0 <= v() <= 1.0


def test_rng_streams_and_masks():
    from fleetx_amd.parallel import rng
    rng.model_parallel_random_seed(10, mp_rank=1, pp_rank=0, data_rank=2)
    t = rng.get_rng_state_tracker()
    st = t.get_states()
    assert st["global_seed"][0] == 12 and st["local_seed"][0] == 10 + 123 + 10
    k1 = t.next_key("global_seed")
    t.set_states(st)
    assert t.next_key("global_seed") == k1
    m = rng.keep_mask((1000, 100), 0.1, k1)
    assert abs(m.float().mean().item() - 0.9) < 0.01
    am = rng.attention_keep_mask(2, 64, 64, 0.25, k1)
    assert abs(am.float().mean().item() - 0.75) < 0.02


def test_train_cli_cpu_fp32(tmp_path):
    cmd = [sys.executable, os.path.join(ROOT, "tools", "train.py"), "-c", CFG,
           "-o", "Model.hidden_size=64", "-o", "Model.num_layers=2", "-o",
           "Model.num_attention_heads=4", "-o", "Model.vocab_size=512", "-o", "Engine.max_steps=4",
           "-o", "Engine.eval_freq=2", "-o", "Engine.eval_iters=1", "-o", "Global.device=cpu",
           "-o", "Data.Train.dataset.name=SyntheticGPTDataset", "-o",
           "Data.Eval.dataset.name=SyntheticGPTDataset", "-o", "Data.Train.dataset.max_seq_len=64",
           "-o", "Data.Eval.dataset.max_seq_len=64", "-o", "Data.Train.dataset.vocab_size=512",
           "-o", "Data.Eval.dataset.vocab_size=512", "-o", "Global.local_batch_size=2",
           "-o", "Global.micro_batch_size=2", "-o", "Data.Train.loader.num_workers=0",
           "-o", "Data.Eval.loader.num_workers=0",
           "-o", "Engine.save_load.output_dir=%s" % tmp_path, "-o", "Engine.save_load.save_steps=2",
           "-o", "Engine.metrics_file=%s" % (tmp_path / "metrics.jsonl")]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if "[train]" in l]
    assert len(lines) == 4 and "ips_total" in lines[0] and "tokens/s" in lines[0]
    loss0 = float(lines[0].split("loss: ")[1].split(",")[0])
    assert abs(loss0 - math.log(512)) < 0.3
    assert (tmp_path / "epoch_0_step_2" / "model.pdparams").exists()
    import json
    recs = [json.loads(l) for l in open(tmp_path / "metrics.jsonl")]
    assert [r["step"] for r in recs] == [1, 2, 3, 4]
    assert all(r["tokens_per_s"] > 0 and "grad_norm" in r and "lr" in r for r in recs)


def test_profiler_views(tmp_path):
    """Profiler YAML block -> Chrome trace + Overview/Model/Kernel/Operator/
    Distributed views with the engine's phases (reference §5.1)."""
    class _Loader:
        def __iter__(self):
            return iter([_batch(i) for i in range(6)])

        def __len__(self):
            return 6

    e, _ = _engine(tmp_path, ["Profiler.enable=True", "Profiler.scheduler=[2,4]",
                              "Profiler.profiler_log=%s" % (tmp_path / "prof"),
                              "Engine.max_steps=5", "Engine.logging_freq=1000"])
    e.fit(epoch=1, train_data_loader=_Loader())
    text = (tmp_path / "prof" / "summary_rank0.txt").read_text()
    for view in ("Overview Summary", "Model Summary", "Kernel Summary", "Operator Summary",
                 "Distributed Summary"):
        assert view in text
    for ph in ("Dataloader", "Forward", "Backward", "GradSync", "Optimization"):
        assert ph in text.split("Model Summary")[1].split("Kernel Summary")[0], text
    assert any(p.name.startswith("trace_rank0") for p in (tmp_path / "prof").iterdir())


@pytest.mark.parametrize("micro", [4, 2])
def test_fused_lm_head_ce_matches_plain_head(tmp_path, micro, monkeypatch):
    """ops/lm_head_ce.py: head + CE chunked over tokens (3 chunks of 48 rows
    over 128 tokens, the last one short) with the head's backward inside the
    forward -- same losses and same trained weights as the plain head, with
    and without gradient accumulation (declared upstream gradient 1/2)."""
    monkeypatch.setenv("FLEETX_LM_HEAD_CE_CHUNK", "48")
    runs = []
    for fused in (False, True):
        e, _ = _engine(tmp_path / str(fused), ["Global.micro_batch_size=%d" % micro,
                                               "Model.fused_lm_head_ce=%s" % fused,
                                               "Model.hidden_dropout_prob=0.0",
                                               "Model.attention_probs_dropout_prob=0.0"])
        assert e._fused_head == fused
        losses = [float(e._fit_impl(_batch(i))) for i in range(3)]
        e.optimizer.sync_state()
        runs.append((losses, e.buffer.param_flat.clone()))
    (l0, p0), (l1, p1) = runs
    for a, b in zip(l0, l1):
        assert abs(a - b) < 1e-5 * abs(b), (l0, l1)
    assert torch.allclose(p0, p1, rtol=1e-5, atol=1e-6), float((p0 - p1).abs().max())
    from fleetx_amd.ops import lm_head_ce
    lm_head_ce.check()  # the declared gradient matched every backward


def test_engine_gemm_routing_key(tmp_path, monkeypatch):
    """``Engine.gemm_routing`` sets the GEMM kinds routed to the MFMA kernel
    under FLEETX_GEMM=auto (the ViT-g config routes data gradients too); an
    explicit FLEETX_GEMM_AUTO in the environment wins."""
    from fleetx_amd.ops import gemm as G
    old = set(G.AUTO_KINDS)
    try:
        monkeypatch.delenv("FLEETX_GEMM_AUTO", raising=False)
        _engine(tmp_path / "a", ["Engine.gemm_routing=wgrad,dgrad"])
        assert G.AUTO_KINDS == {"wgrad", "dgrad"}
        G.set_auto_kinds(old)
        monkeypatch.setenv("FLEETX_GEMM_AUTO", "wgrad")
        _engine(tmp_path / "b", ["Engine.gemm_routing=wgrad,dgrad,fwd"])
        assert G.AUTO_KINDS == old
    finally:
        G.set_auto_kinds(old)

"""Whole-step HIP graph training (Engine.cuda_graph): the captured step
(forward, backward, clip, AdamW) replays the eager step's numerics, picks up
the scheduler's learning rate every replay, and draws fresh dropout masks per
replay (device salt) while forward/backward of one step stay consistent."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

CFG = os.path.join(os.path.dirname(__file__), "..", "fleetx_amd", "configs", "nlp", "gpt",
                   "pretrain_gpt_345M_single_card.yaml")


def _engine(graph, drop, lr=None, steps=8, extra=()):
    from fleetx_amd.utils import config as C
    from fleetx_amd.utils import env
    from fleetx_amd.models import build_module
    from fleetx_amd.core.engine.eager_engine import EagerEngine
    from fleetx_amd.parallel import topology as topo
    from fleetx_amd.ops import _lib
    topo.reset_hcg()
    _lib.kernels().set_dropout_salt(0)
    _lib.kernels().set_adamw_lr_ptr(0)
    ov = ["Model.hidden_size=256", "Model.num_layers=3", "Model.num_attention_heads=4",
          "Model.vocab_size=1024", "Model.hidden_dropout_prob=%s" % drop,
          "Model.attention_probs_dropout_prob=%s" % drop, "Model.max_position_embeddings=128",
          "Global.device=gpu", "Global.local_batch_size=4", "Global.micro_batch_size=4",
          "Engine.max_steps=%d" % steps, "Engine.mix_precision.dtype=bfloat16",
          "Engine.cuda_graph=%s" % graph, "Data.Train.dataset.name=SyntheticGPTDataset"]
    ov += list(extra)
    cfg = C.get_config(CFG, overrides=ov, nranks=1)
    if lr is not None:
        cfg.Optimizer.lr = {"name": "ConstantLR", "learning_rate": lr}
    else:
        cfg.Optimizer.lr = {"name": "CosineAnnealingWithWarmupDecay", "decay_steps": 20,
                            "warmup_rate": 0.2, "max_lr": 3e-3, "min_lr": 1e-4}
    env.set_seed(cfg.Global.seed)
    return EagerEngine(configs=cfg, module=build_module(cfg), mode="train")


def _batches(n, seed=0, same=False):
    g = torch.Generator().manual_seed(seed)
    out = []
    t0 = torch.randint(0, 1024, (4, 129), generator=g)
    for _ in range(n):
        t = t0 if same else torch.randint(0, 1024, (4, 129), generator=g)
        t = t.cuda()
        out.append([t[:, :-1].contiguous(), torch.arange(128, device="cuda").expand(4, 128).contiguous(),
                    t[:, 1:].contiguous(), torch.ones(4, 128, device="cuda")])
    return out


def _run(eng, batches):
    losses = []
    for b in batches:
        losses.append(float(eng._fit_impl(b)))
    torch.cuda.synchronize()
    return losses


def test_graph_step_matches_eager_without_dropout():
    bs = _batches(8)
    eager = _run(_engine(False, 0.0), bs)
    eng = _engine(True, 0.0)
    graph = _run(eng, bs)
    assert eng._graph is not None  # captured and replayed
    for a, b in zip(eager, graph):
        assert abs(a - b) <= 2e-3 * abs(a), (eager, graph)
    assert eng.optimizer.step_count == 8
    assert int(eng.optimizer.dev_step.item()) == 8


def test_graph_dropout_masks_change_per_replay():
    # lr 0: weights never move, so loss differences come from dropout masks only
    eng = _engine(True, 0.1, lr=0.0)
    losses = _run(eng, _batches(6, same=True))
    assert eng._graph is not None
    assert all(l == l for l in losses)
    assert len(set(round(x, 6) for x in losses[3:])) == 3, losses
    from fleetx_amd.ops import _lib
    _lib.kernels().set_dropout_salt(0)
    _lib.kernels().set_adamw_lr_ptr(0)


def test_graph_salt_checkpointed(tmp_path):
    """The device dropout salt is saved and restored, so a resumed graph-mode
    run continues the mask sequence instead of replaying it."""
    eng = _engine(True, 0.1)
    _run(eng, _batches(4))
    eng._output_dir = str(tmp_path)
    eng.save(epoch=0, step=4)
    salt = int(eng._graph_salt.item())
    assert salt == 4
    eng2 = _engine(True, 0.1)
    import glob
    eng2.load(ckpt_dir=glob.glob(str(tmp_path / "epoch_0_step_4*"))[0])
    _run(eng2, _batches(1))
    assert int(eng2._graph_salt.item()) == salt + 1
    from fleetx_amd.ops import _lib
    _lib.kernels().set_dropout_salt(0)
    _lib.kernels().set_adamw_lr_ptr(0)


def test_graph_short_batch_runs_eagerly():
    """A batch of another shape than the captured one runs eagerly (and the
    graph keeps serving the regular batches)."""
    eng = _engine(True, 0.0)
    bs = _batches(4)
    _run(eng, bs[:3])
    assert eng._graph is not None
    short = [t[:2].contiguous() for t in bs[3]]
    l_short = float(eng._fit_impl(short))
    l_next = float(eng._fit_impl(bs[0]))
    assert l_short == l_short and l_next == l_next
    assert eng.optimizer.step_count == 5 and int(eng.optimizer.dev_step.item()) == 5
    from fleetx_amd.ops import _lib
    _lib.kernels().set_dropout_salt(0)
    _lib.kernels().set_adamw_lr_ptr(0)


def test_graph_with_deferred_overlapped_update_matches_serial(monkeypatch):
    """Graph mode runs step N's AdamW at the start of step N+1's captured body,
    beside its forward (optimizer.defer_update): parameters after the last
    step (flushed by sync_state) are bitwise those of the graph with the
    serial update, and a flush in between is not applied twice."""
    monkeypatch.setenv("FLEETX_DETERMINISTIC", "1")
    bs = _batches(7)
    ser = _engine(True, 0.0, extra=["Distributed.comm.overlap_optimizer=False"])
    assert not ser.optimizer.defer_update
    _run(ser, bs)
    ser.optimizer.sync_state()
    torch.cuda.synchronize()
    eng = _engine(True, 0.0)
    assert eng.optimizer.defer_update and eng._cuda_graph
    losses = _run(eng, bs[:5])
    assert eng._graph is not None
    eng.optimizer.sync_state()          # applies step 5's update (flush)
    mid = {n: p.detach().clone() for n, p in eng._module.model.named_parameters()}
    _run(eng, bs[5:])                   # the flushed update is not applied twice
    eng.optimizer.sync_state()
    torch.cuda.synchronize()
    for (n, a), (_, b) in zip(ser._module.model.named_parameters(),
                              eng._module.model.named_parameters()):
        assert torch.equal(a, b), n
    assert any(not torch.equal(mid[n], p) for n, p in eng._module.model.named_parameters())
    assert all(l == l for l in losses)


def test_graph_flush_before_capture_keeps_update_in_graph(monkeypatch):
    """A flush (sync_state: eval / save) between the last eager warmup call and
    the capture clears the host's pending update; the captured body must still
    hold the update launch, or every replay would silently skip its AdamW.
    Bitwise against the serial-update graph."""
    monkeypatch.setenv("FLEETX_DETERMINISTIC", "1")
    bs = _batches(6)
    ser = _engine(True, 0.0, extra=["Distributed.comm.overlap_optimizer=False"])
    _run(ser, bs)
    ser.optimizer.sync_state()
    torch.cuda.synchronize()
    eng = _engine(True, 0.0)
    assert eng.optimizer.defer_update and eng._cuda_graph
    _run(eng, bs[:2])                   # the two eager warmup calls
    eng.optimizer.sync_state()          # flush right before the capture call
    assert eng.optimizer._pending is None
    _run(eng, bs[2:])                   # capture + replays
    assert eng._graph is not None
    eng.optimizer.sync_state()
    torch.cuda.synchronize()
    assert int(eng.optimizer.dev_step.item()) == 6
    for (n, a), (_, b) in zip(ser._module.model.named_parameters(),
                              eng._module.model.named_parameters()):
        assert torch.equal(a, b), n

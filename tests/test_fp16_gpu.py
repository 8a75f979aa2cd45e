"""Pure-fp16 (O2) training on the GPU: the reference's ``use_pure_fp16: True,
dtype: float16`` mode (``pretrain_gpt_base.yaml:18-22``,
``eager_engine.py:157-167,421,436-438``) through the f16 MFMA flash kernels,
fused LN / CE and the device-side dynamic loss scaler.

* fp16 and bf16 runs from identical weights follow the same loss curve;
* an injected overflow (loss scale 2^40 -> inf fp16 gradients) skips the
  update entirely (parameters and Adam's step counter unchanged) and the
  scale halves only after ``decr_every_n_nan_or_inf`` (2) consecutive
  overflows (Paddle GradScaler semantics)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

CFG = os.path.join(os.path.dirname(__file__), "..", "fleetx_amd", "configs", "nlp", "gpt",
                   "pretrain_gpt_345M_single_card.yaml")
B, S, V = 4, 256, 2048


def _engine(dtype, extra=()):
    from fleetx_amd.utils import config as C
    from fleetx_amd.utils import env
    from fleetx_amd.models import build_module
    from fleetx_amd.core.engine.eager_engine import EagerEngine
    from fleetx_amd.parallel import topology as topo
    topo.reset_hcg()
    ov = ["Model.hidden_size=512", "Model.num_layers=2", "Model.num_attention_heads=8",
          "Model.vocab_size=%d" % V, "Model.hidden_dropout_prob=0.0",
          "Model.attention_probs_dropout_prob=0.0", "Model.max_position_embeddings=%d" % S,
          "Global.device=gpu", "Global.local_batch_size=%d" % B, "Global.micro_batch_size=%d" % B,
          "Engine.mix_precision.use_pure_fp16=True", "Engine.mix_precision.dtype=%s" % dtype,
          "Engine.mix_precision.scale_loss=1024.0", "Engine.max_steps=100",
          "Data.Train.dataset.name=SyntheticGPTDataset"] + list(extra)
    cfg = C.get_config(CFG, overrides=ov, nranks=1)
    cfg.Optimizer.lr = {"name": "ConstantLR", "learning_rate": 1e-3}
    env.init_dist_env(cfg)
    env.set_seed(cfg.Global.seed)
    return EagerEngine(configs=cfg, module=build_module(cfg), mode="train")


def _batch(step):
    g = torch.Generator().manual_seed(100 + step)
    t = torch.randint(0, V, (B, S + 1), generator=g).cuda()
    return [t[:, :-1].contiguous(), torch.arange(S, device="cuda").expand(B, S).contiguous(),
            t[:, 1:].contiguous(), torch.ones(B, S, device="cuda")]


def test_fp16_matches_bf16_curve():
    curves = {}
    for dt in ("bfloat16", "float16"):
        eng = _engine(dt)
        assert eng._dtype == getattr(torch, dt)
        assert (eng.scaler is not None) == (dt == "float16")
        # the same batch every step: the loss must fall
        curves[dt] = [eng._reduce_log_loss(eng._fit_impl(_batch(0)), 1) for s in range(4)]
    a, b = curves["float16"], curves["bfloat16"]
    for x, y in zip(a, b):
        assert abs(x - y) < 1e-2 * abs(y), curves
    assert a[-1] < a[0], curves


def test_fp16_overflow_skips_update_and_scaler_backs_off():
    eng = _engine("float16")
    eng._fit_impl(_batch(0))                     # one clean step
    torch.cuda.synchronize()
    opt, sc = eng.optimizer, eng.scaler
    step0 = int(opt.dev_step.item())
    params0 = eng.buffer.param_flat.clone()
    sc.scale.fill_(2.0 ** 40)                    # fp16 gradients overflow
    eng.optimizer.loss_scale = sc.scale
    eng._fit_impl(_batch(1))
    torch.cuda.synchronize()
    assert int(opt.found_inf.item()) == 1
    assert torch.equal(eng.buffer.param_flat, params0), "overflowed step changed the weights"
    assert int(opt.dev_step.item()) == step0, "overflowed step advanced Adam's bias correction"
    assert float(sc.scale) == 2.0 ** 40 and int(sc.bad) == 1   # 1st overflow: keep the scale
    eng._fit_impl(_batch(2))
    torch.cuda.synchronize()
    assert float(sc.scale) == 2.0 ** 39 and int(sc.bad) == 0   # 2nd consecutive: halve
    sc.scale.fill_(1024.0)
    eng.optimizer.loss_scale = sc.scale
    eng._fit_impl(_batch(3))
    torch.cuda.synchronize()
    assert int(opt.found_inf.item()) == 0
    assert int(opt.dev_step.item()) == step0 + 1
    assert not torch.equal(eng.buffer.param_flat, params0)


def _fp16_pair(overlap):
    os.environ["FLEETX_DETERMINISTIC"] = "1"
    out = [_fp16_run(False, overlap), _fp16_run(True, overlap)]
    for o in out:
        o["params"] = o["params"].cpu()
        o["gdtype"] = str(o["gdtype"])
    return out


def _fp16_run(graph, overlap, steps=9, inject=(3, 4)):
    """fp16 O2 steps with the scaler growing every 2 good steps; at step
    inject[0] the scale is set to 2^40 (fp16 gradients overflow: skip, and
    with decr_every 1 the scale halves), at inject[1] back to 1024."""
    from fleetx_amd.ops import _lib
    _lib.kernels().set_dropout_salt(0)
    _lib.kernels().set_adamw_lr_ptr(0)
    eng = _engine("float16", extra=(
        "Engine.cuda_graph=%s" % graph, "Engine.mix_precision.incr_every_n_steps=2",
        "Engine.mix_precision.decr_every_n_nan_or_inf=1",
        "Distributed.comm.overlap_optimizer=%s" % overlap))
    assert eng._cuda_graph == graph
    sc, opt = eng.scaler, eng.optimizer
    losses, scales, infs = [], [], []
    for s in range(steps):
        if s == inject[0]:
            sc.scale.fill_(2.0 ** 40)
        elif s == inject[1]:
            sc.scale.fill_(1024.0)
        losses.append(float(eng._fit_impl(_batch(s))))
        torch.cuda.synchronize()
        scales.append(float(sc.scale))
        infs.append(int(opt.found_inf.item()))
    opt.sync_state()
    torch.cuda.synchronize()
    out = {"losses": losses, "scales": scales, "infs": infs,
           "params": eng.buffer.param_flat.detach().clone(), "step": int(opt.dev_step.item()),
           "graph": eng._graph is not None, "gdtype": eng.buffer.grad_dtype}
    _lib.kernels().set_dropout_salt(0)
    _lib.kernels().set_adamw_lr_ptr(0)
    return out


@pytest.mark.parametrize("overlap", [False, True])
def test_fp16_graph_replay_bitwise_eager_across_overflow_and_growth(overlap):
    """The fp16 step captured in the whole-step HIP graph (loss scaler
    updated in place on the device) replays the eager step bit for bit:
    through scale growth, an overflowed (skipped) step with its back-off,
    and the manual reset -- with the serial and with the deferred overlapped
    update.  fp16 O2 stores the GEMM-written gradients in fp16 (grad_dtype
    auto), whose overflow the epilogue's norm partials report."""
    # a fresh process: deterministic routes / tile orders from the first GEMM
    # on (earlier tests of this module raced shapes non-deterministically)
    import multiprocessing as mp
    with mp.get_context("spawn").Pool(1) as pool:
        e, g = pool.apply(_fp16_pair, (overlap,))
    assert g["graph"] and not e["graph"]
    assert e["gdtype"] == g["gdtype"] == "torch.float16"
    assert e["infs"][3] == 1 and sum(e["infs"]) == 1, e["infs"]
    assert e["scales"][3] == 2.0 ** 39                      # overflow: halved
    assert any(b == 2 * a for a, b in zip(e["scales"][4:], e["scales"][5:])), e["scales"]
    assert e["step"] == 9 - 1                                  # the skipped step
    assert e["losses"] == g["losses"], (e["losses"], g["losses"])
    assert e["scales"] == g["scales"] and e["infs"] == g["infs"]
    assert torch.equal(e["params"], g["params"])

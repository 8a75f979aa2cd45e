"""Global gradient norm from the weight-gradient GEMM epilogue
(``grad_buffer.enable_fused_norm``) against the plain second pass over the
fp32 gradient (``fused_grad_norm=False``): same weights, same batches, with
and without micro-batch accumulation.  The clip coefficient of the reference's
``ClipGradByGlobalNorm`` (``optims/optimizer.py``) depends on this value, so
the two must agree to fp32 rounding, and the trained weights must match."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

CFG = os.path.join(os.path.dirname(__file__), "..", "fleetx_amd", "configs", "nlp", "gpt",
                   "pretrain_gpt_345M_single_card.yaml")
B, S, V = 8, 256, 2048


@pytest.fixture(autouse=True)
def hip_gemm():
    from fleetx_amd.ops import gemm as G
    old = G._MODE
    G.set_mode("hip")  # every weight gradient on the hand-written kernel
    yield
    G.set_mode(old)


def _engine(fused, micro):
    from fleetx_amd.utils import config as C
    from fleetx_amd.utils import env
    from fleetx_amd.models import build_module
    from fleetx_amd.core.engine.eager_engine import EagerEngine
    from fleetx_amd.parallel import topology as topo
    topo.reset_hcg()
    ov = ["Model.hidden_size=512", "Model.num_layers=2", "Model.num_attention_heads=8",
          "Model.vocab_size=%d" % V, "Model.hidden_dropout_prob=0.0",
          "Model.attention_probs_dropout_prob=0.0", "Model.max_position_embeddings=%d" % S,
          "Global.device=gpu", "Global.local_batch_size=%d" % B,
          "Global.micro_batch_size=%d" % micro, "Engine.mix_precision.dtype=bfloat16",
          "Engine.max_steps=100", "Data.Train.dataset.name=SyntheticGPTDataset",
          "Distributed.comm.fused_grad_norm=%s" % fused]
    cfg = C.get_config(CFG, overrides=ov, nranks=1)
    env.init_dist_env(cfg)
    env.set_seed(cfg.Global.seed)
    return EagerEngine(configs=cfg, module=build_module(cfg), mode="train")


def _batch(step):
    g = torch.Generator().manual_seed(300 + step)
    t = torch.randint(0, V, (B, S + 1), generator=g).cuda()
    return [t[:, :-1].contiguous(), torch.arange(S, device="cuda").expand(B, S).contiguous(),
            t[:, 1:].contiguous(), torch.ones(B, S, device="cuda")]


@pytest.mark.parametrize("micro", [B, B // 2])
def test_fused_norm_matches_second_pass(micro):
    runs = {}
    for fused in (True, False):
        eng = _engine(fused, micro)
        assert (eng.buffer._fused_norm is not None) == fused
        norms = []
        for s in range(3):
            eng._fit_impl(_batch(s))
            norms.append(float(eng.optimizer.last_grad_norm))
        if fused:
            covered = [p for n, p in eng.buffer.params if getattr(p, "_fx_sq", None) is not None]
            assert covered and all(p._fx_sq_ok for p in covered), "epilogue partials unused"
        eng.optimizer.sync_state()
        runs[fused] = (norms, eng.buffer.param_flat.float().clone())
    (a, pa), (b, pb) = runs[True], runs[False]
    for x, y in zip(a, b):
        assert abs(x - y) <= 2e-5 * y, (a, b)
    assert torch.allclose(pa, pb, rtol=0, atol=1e-3), float((pa - pb).abs().max())

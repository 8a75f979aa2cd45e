"""16-bit gradient storage on the GPU (``Distributed.comm.grad_dtype``): the
weight-gradient GEMM writes bf16 gradients from its fp32 accumulators, the
fused AdamW reads them (28 instead of 30 B per parameter), and training
matches the fp32-gradient run within bf16 rounding of the gradients."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

CFG = os.path.join(os.path.dirname(__file__), "..", "fleetx_amd", "configs", "nlp", "gpt",
                   "pretrain_gpt_345M_single_card.yaml")


def _engine(grad_dtype, graph=False):
    from fleetx_amd.utils import config as C
    from fleetx_amd.utils import env
    from fleetx_amd.models import build_module
    from fleetx_amd.core.engine.eager_engine import EagerEngine
    from fleetx_amd.parallel import topology as topo
    topo.reset_hcg()
    ov = ["Model.hidden_size=256", "Model.num_layers=3", "Model.num_attention_heads=4",
          "Model.vocab_size=1024", "Model.hidden_dropout_prob=0.0",
          "Model.attention_probs_dropout_prob=0.0", "Model.max_position_embeddings=128",
          "Global.device=gpu", "Global.local_batch_size=4", "Global.micro_batch_size=4",
          "Engine.max_steps=8", "Engine.mix_precision.dtype=bfloat16",
          "Engine.cuda_graph=%s" % graph, "Distributed.comm.grad_dtype=%s" % grad_dtype,
          "Data.Train.dataset.name=SyntheticGPTDataset"]
    cfg = C.get_config(CFG, overrides=ov, nranks=1)
    cfg.Optimizer.lr = {"name": "ConstantLR", "learning_rate": 1e-3}
    env.set_seed(cfg.Global.seed)
    return EagerEngine(configs=cfg, module=build_module(cfg), mode="train")


def _train(eng, steps=4):
    g = torch.Generator().manual_seed(3)
    losses = []
    for _ in range(steps):
        t = torch.randint(0, 1024, (4, 129), generator=g).cuda()
        b = [t[:, :-1].contiguous(), torch.arange(128, device="cuda").expand(4, 128).contiguous(),
             t[:, 1:].contiguous(), torch.ones(4, 128, device="cuda")]
        losses.append(float(eng._fit_impl(b)))
    eng.optimizer.sync_state()
    torch.cuda.synchronize()
    return losses


@pytest.mark.parametrize("graph", [False, True])
def test_grad16_training_matches_fp32_gradients(graph):
    e16 = _engine("bfloat16", graph)
    # the GEMM-written weights hold bf16 gradients, the rest fp32
    dts = {p.main_grad.dtype for _, p in e16._module.model.named_parameters()}
    assert dts == {torch.bfloat16, torch.float32}
    l16 = _train(e16)
    e32 = _engine("float32", graph)
    assert all(p.main_grad.dtype == torch.float32
               for _, p in e32._module.model.named_parameters())
    l32 = _train(e32)
    assert abs(l16[0] - l32[0]) < 1e-3 * abs(l32[0])       # same weights, same forward
    for a, b in zip(l16[1:], l32[1:]):
        assert abs(a - b) < 1e-2 * abs(b), (l16, l32)
    # every master after the updates: weight matrices within 2 % of their
    # norm; zero-initialised biases / norms are pure update, where Adam turns
    # bf16-level gradient differences into sign flips (as between any two
    # bf16 runs with another reduction order, tests/test_multirank_gpu.py),
    # so they only get a sanity bound
    from fleetx_amd.parallel.state_gather import gather_master_state
    m16, m32 = gather_master_state(e16), gather_master_state(e32)
    for k in m32:
        err = float((m16[k] - m32[k]).norm())
        rel = 0.02 if m32[k].dim() == 2 else 0.5
        assert err <= rel * float(m32[k].norm()) + 1e-4, (k, err, float(m32[k].norm()))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n", [1, 7, 4096 * 8 + 3, 3_000_001])
def test_sumsq_16_kernel(dtype, n):
    """The gradient norm over 16-bit gradient storage reads the 16-bit values
    in place (``optimizer._sumsq``), against an fp64 reference; an fp16 inf
    (an overflowed gradient) makes the sum non-finite."""
    from fleetx_amd.optims.optimizer import _sumsq
    torch.manual_seed(n)
    x = torch.randn(n + 1, device="cuda").to(dtype)[1:]  # misaligned start included
    ref = float(x.double().pow(2).sum())
    got = float(_sumsq(x))
    assert abs(got - ref) <= 1e-4 * ref + 1e-6, (got, ref)
    if dtype == torch.float16 and n > 1:
        x[n // 2] = float("inf")
        assert not torch.isfinite(_sumsq(x))

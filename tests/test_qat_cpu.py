"""QAT wrapper (reference P11): layers swapped, int8 grid respected, STE grads,
moving-average activation scale, and a GPT module built with Quantization on."""
import os

import torch

from fleetx_amd.utils.qat import quantize_model, QuantizedLinear

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_quantize_linear_grid_and_ste():
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(8, 4), torch.nn.ReLU(), torch.nn.Linear(4, 2))
    quantize_model(m, {"weight_bits": 8, "activation_bits": 8})
    assert isinstance(m[0], QuantizedLinear) and isinstance(m[2], QuantizedLinear)
    x = torch.randn(5, 8, requires_grad=True)
    y = m(x)
    y.sum().backward()
    assert x.grad is not None and m[0].inner.weight.grad is not None
    s = m[0].wq.scale.item()
    assert abs(s - m[0].inner.weight.abs().max().item()) < 1e-6
    q = m[0].wq(m[0].inner.weight.detach())
    steps = q / (s / 127.0)
    assert torch.allclose(steps, steps.round(), atol=1e-3)
    a0 = m[0].aq.scale.item()
    m(3 * x.detach())  # EMA moves towards the larger abs-max, not jumps to it
    a1 = m[0].aq.scale.item()
    big = (3 * x).abs().max().item()
    assert a0 < a1 < big


def test_gpt_module_with_quantization():
    from fleetx_amd.utils import config as C
    from fleetx_amd.models import build_module
    cfg = C.get_config(os.path.join(ROOT, "fleetx_amd/configs/nlp/gpt/pretrain_gpt_345M_mp8_qat.yaml"),
                       overrides=["Model.hidden_size=32", "Model.num_layers=1",
                                  "Model.num_attention_heads=2", "Model.vocab_size=64",
                                  "Model.max_position_embeddings=32", "Global.device=cpu",
                                  "Distributed.mp_degree=1"], nranks=1)
    module = build_module(cfg)
    n_q = sum(isinstance(x, QuantizedLinear) for x in module.model.modules())
    assert n_q >= 4
    toks = torch.randint(0, 64, (2, 16))
    loss = module.training_step((toks, torch.arange(16).expand(2, 16), toks, torch.ones(2, 16)))
    loss.backward()
    assert torch.isfinite(loss)

"""Decode-time fused kernels (K19): the skinny MFMA GEMV with its sub-layer
epilogues (csrc/kernels/decode_gemv.hip) against fp32 torch, and the fused
decode layer against the unfused op chain."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(1, 4096, 4096), (3, 1000, 1024), (16, 12288, 2048),
                                   (7, 2048, 16384), (16, 50304, 1024), (2, 96, 1024)])
@pytest.mark.parametrize("epi", [0, 1, 2])
def test_decode_gemv_epilogues(dtype, M, N, K, epi):
    from fleetx_amd.ops import gemm as G
    g = torch.Generator(device=DEV).manual_seed(M * 7 + N + epi)
    x = torch.randn(M, K, device=DEV, generator=g).to(dtype)
    w = (torch.randn(N, K, device=DEV, generator=g) * K ** -0.5).to(dtype)
    b = torch.randn(N, device=DEV, generator=g).to(dtype)
    res = torch.randn(M, N, device=DEV, generator=g).to(dtype) if epi == G.GV_RES else None
    y = G.decode_linear(x, w, b, epi, res=res)
    assert y is not None
    ref = x.float() @ w.float().t() + b.float()
    if epi == G.GV_GELU:
        ref = torch.nn.functional.gelu(ref, approximate="tanh")
    if epi == G.GV_RES:
        ref = ref + res.float()
    tol = 8e-3 if dtype == torch.bfloat16 else 2e-3
    assert _rel(y, ref) < tol


@pytest.mark.parametrize("M,N,K", [(1, 8192, 2048), (1, 6144, 2048), (1, 12288, 4096),
                                   (3, 1000, 1024), (4, 3072, 2048), (4, 4096, 4096), (8, 3072, 2048),
                                   (16, 6144, 2048), (16, 4096, 4096)])
@pytest.mark.parametrize("epi", [1, 3])
def test_decode_gemv_fused_layernorm(M, N, K, epi):
    """LayerNorm fused as the GEMV prologue (LN1 -> QKV, LN2 -> FFN1) vs fp32
    LayerNorm (rounded to bf16, as the unfused path feeds the GEMV) + GEMM; the
    residual rows carry a large common offset so the shifted one-pass moments
    are exercised."""
    from fleetx_amd.ops import gemm as G
    g = torch.Generator(device=DEV).manual_seed(M + N + K + epi)
    x = (3.0 + torch.randn(M, K, device=DEV, generator=g)).bfloat16()
    w = (torch.randn(N, K, device=DEV, generator=g) * K ** -0.5).bfloat16()
    b = torch.randn(N, device=DEV, generator=g).bfloat16()
    lw = (1 + 0.1 * torch.randn(K, device=DEV, generator=g)).bfloat16()
    lb = (0.1 * torch.randn(K, device=DEV, generator=g)).bfloat16()
    xn = torch.nn.functional.layer_norm(x.float(), (K,), lw.float(), lb.float(), 1e-5)
    ref = xn.bfloat16().float() @ w.float().t() + b.float()
    if M > 4 or M * (K + 8) * 2 > 96 * 1024:  # not covered by the fused prologue: caller falls back
        if epi == G.GV_GELU:
            assert G.decode_linear(x, w, b, epi, ln=(lw, lb, 1e-5)) is None
        return
    if epi == G.GV_GELU:
        y = G.decode_linear(x, w, b, epi, ln=(lw, lb, 1e-5))
        assert y is not None
        ref = torch.nn.functional.gelu(ref, approximate="tanh")
        assert _rel(y, ref) < 8e-3, _rel(y, ref)
    else:
        H, D = N // 192, 64
        if N % 192:
            pytest.skip("QKV needs N = 3 * heads * 64")
        L = 8
        kc = torch.zeros(M, L, H, D, device=DEV, dtype=torch.bfloat16)
        vc = torch.zeros_like(kc)
        pos = torch.arange(M, device=DEV) % L
        q = G.decode_linear(x, w, b, G.GV_QKV, qkv_cache=(kc, vc, pos), ln=(lw, lb, 1e-5))
        assert q is not None
        r = ref.view(M, H, 3, D)
        ar = torch.arange(M, device=DEV)
        assert _rel(q.view(M, H, D), r[:, :, 0]) < 8e-3
        assert _rel(kc[ar, pos], r[:, :, 1]) < 8e-3
        assert _rel(vc[ar, pos], r[:, :, 2]) < 8e-3


def test_decode_gemv_qkv_scatter():
    from fleetx_amd.ops import gemm as G
    B, H, D, L, h = 5, 8, 64, 40, 1024
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randn(B, h, device=DEV, generator=g).bfloat16()
    w = (torch.randn(3 * H * D, h, device=DEV, generator=g) * h ** -0.5).bfloat16()
    b = torch.randn(3 * H * D, device=DEV, generator=g).bfloat16()
    kc = torch.zeros(B, L, H, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    pos = torch.tensor([0, 3, 39, 17, 8], device=DEV)
    q = G.decode_linear(x, w, b, G.GV_QKV, qkv_cache=(kc, vc, pos))
    ref = (x.float() @ w.float().t() + b.float()).view(B, H, 3, D)
    assert _rel(q.view(B, H, D), ref[:, :, 0]) < 8e-3
    ar = torch.arange(B, device=DEV)
    assert _rel(kc[ar, pos], ref[:, :, 1]) < 8e-3
    assert _rel(vc[ar, pos], ref[:, :, 2]) < 8e-3
    mask = torch.ones(B, L, dtype=torch.bool, device=DEV)
    mask[ar, pos] = False
    assert kc[mask].abs().max().item() == 0 and vc[mask].abs().max().item() == 0


def test_fused_decode_step_matches_unfused():
    from fleetx_amd.models.language_model.gpt.model import GPTConfig, GPTForPretraining
    from fleetx_amd.models.language_model.gpt.generation import GPTForGeneration, KVCache
    torch.manual_seed(0)
    cfg = GPTConfig(vocab_size=1024, hidden_size=1024, num_layers=3, num_attention_heads=8,
                    max_position_embeddings=256, hidden_dropout_prob=0.0,
                    attention_probs_dropout_prob=0.0, dtype=torch.bfloat16)
    model = GPTForPretraining(cfg).cuda().eval()
    from fleetx_amd.models.language_model.gpt import generation as gmod
    calls = []
    orig = gmod._layer_decode_fused
    gmod._layer_decode_fused = lambda *a: calls.append(orig(*a)) or calls[-1]
    B = 6
    outs = []
    for fused in (False, True):
        gen = GPTForGeneration(model, {"fused_decode": fused}).eval()
        cache = KVCache(cfg.num_layers, B, 64, 8, 128, torch.bfloat16, DEV)
        g = torch.Generator(device=DEV).manual_seed(5)
        for L in range(cfg.num_layers):
            cache.k[L].normal_(generator=g)
            cache.v[L].normal_(generator=g)
        nxt = torch.randint(0, 1024, (B,), device=DEV, generator=g)
        cur = torch.tensor([3, 10, 0, 63, 20, 41], device=DEV)
        with torch.no_grad():
            lg = gen._decode_step(nxt, cur, cache)
        outs.append((lg, [c.clone() for c in cache.k], [c.clone() for c in cache.v]))
    gmod._layer_decode_fused = orig
    assert len(calls) == cfg.num_layers and all(c is not None for c in calls)  # fused ran
    assert _rel(outs[1][0], outs[0][0]) < 2e-2
    for a, b in zip(outs[0][1] + outs[0][2], outs[1][1] + outs[1][2]):
        assert _rel(b, a) < 2e-2

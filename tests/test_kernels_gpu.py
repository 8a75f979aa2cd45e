"""HIP kernel numerics vs plain PyTorch fp32 references (MI355X only)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from fleetx_amd.ops import _lib
    _lib.kernels()  # fail loudly if the extension is missing


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.fixture(autouse=True)
def _gpu():
    _need_gpu()
    torch.manual_seed(0)


# ---------------------------------------------------------------- LayerNorm
@pytest.mark.parametrize("h", [1024, 4096, 2560, 1408, 768, 1000, 4104])
@pytest.mark.parametrize("fused", [False, True])
def test_layer_norm_fwd_bwd(h, fused):
    from fleetx_amd import ops
    from fleetx_amd.parallel import rng
    rows = 512
    x = torch.randn(rows, h, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(h, device=DEV)).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(h, device=DEV)).bfloat16().requires_grad_()
    p, key = (0.1, 987654321) if fused else (0.0, 0)
    if fused:
        bias = (0.1 * torch.randn(h, device=DEV)).bfloat16().requires_grad_()
        res = torch.randn(rows, h, device=DEV, dtype=torch.bfloat16, requires_grad=True)
        s, y = ops.add_layer_norm(x, bias, res, w, b, 1e-5, p, key)
    else:
        y = ops.layer_norm(x, w, b, 1e-5)
    # fp32 reference (same dropout mask from the shared counter hash)
    xr = x.detach().float().requires_grad_()
    wr, br = w.detach().float().requires_grad_(), b.detach().float().requires_grad_()
    if fused:
        biasr = bias.detach().float().requires_grad_()
        resr = res.detach().float().requires_grad_()
        keep = rng.keep_mask((rows, h), p, key, DEV)
        v = torch.where(keep, (xr + biasr) / (1 - p), torch.zeros_like(xr)) + resr
        sr = v
    else:
        v = xr
    yr = torch.nn.functional.layer_norm(v, (h,), wr, br, 1e-5)
    assert _rel(y, yr) < 1e-2
    if fused:
        assert _rel(s, sr) < 1e-2
    gy = torch.randn_like(yr)
    loss = (y.float() * gy).sum() + ((s.float() * gy).sum() if fused else 0)
    loss.backward()
    lr_ = (yr * gy).sum() + ((sr * gy).sum() if fused else 0)
    lr_.backward()
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(w.grad, wr.grad) < 2e-2
    assert _rel(b.grad, br.grad) < 2e-2
    if fused:
        assert _rel(bias.grad, biasr.grad) < 2e-2
        assert _rel(res.grad, resr.grad) < 2e-2


@pytest.mark.parametrize("rows,h", [(1000, 1408), (3, 1024), (16448, 768), (1000, 4096), (7, 2048), (513, 2560)])
def test_ln_bwd_cols_uneven_rows(rows, h, monkeypatch):
    """The one-pass LayerNorm backward with column sums (ln_bwd_cols_kernel):
    rows that leave the last waves short or empty, masked widths; dgamma,
    dbeta and the fused bias gradient against fp32 torch."""
    from fleetx_amd import ops
    from fleetx_amd.ops import _lib
    monkeypatch.setenv("FLEETX_LN_BWD_FUSED", "2")   # 2 / 4 waves per row for h > 1536
    assert _lib.kernels().ln_bwd_cols_blocks(rows, h, 4096) > 0
    x = torch.randn(rows, h, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(h, device=DEV)).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(h, device=DEV)).bfloat16().requires_grad_()
    bias = (0.1 * torch.randn(h, device=DEV)).bfloat16().requires_grad_()
    res = torch.randn(rows, h, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    s, y = ops.add_layer_norm(x, bias, res, w, b, 1e-5, 0.0, 0)
    xr, wr, br, biasr, resr = (t.detach().float().requires_grad_() for t in (x, w, b, bias, res))
    sr = xr + biasr + resr
    yr = torch.nn.functional.layer_norm(sr, (h,), wr, br, 1e-5)
    gy, gs = torch.randn_like(yr), torch.randn_like(yr)
    ((y.float() * gy).sum() + (s.float() * gs).sum()).backward()
    ((yr * gy).sum() + (sr * gs).sum()).backward()
    for got, ref in ((x.grad, xr.grad), (res.grad, resr.grad), (w.grad, wr.grad),
                     (b.grad, br.grad), (bias.grad, biasr.grad)):
        assert _rel(got, ref) < 2e-2


# ---------------------------------------------------------------- GeLU / dropout
@pytest.mark.parametrize("approx", [True, False])
def test_bias_gelu(approx):
    from fleetx_amd import ops
    x = torch.randn(300, 2048, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    b = (0.1 * torch.randn(2048, device=DEV)).bfloat16().requires_grad_()
    y = ops.bias_gelu(x, b, approximate=approx)
    xr, br = x.detach().float().requires_grad_(), b.detach().float().requires_grad_()
    yr = torch.nn.functional.gelu(xr + br, approximate="tanh" if approx else "none")
    assert _rel(y, yr) < 1e-2
    g = torch.randn_like(yr)
    (y.float() * g).sum().backward()
    (yr * g).sum().backward()
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(b.grad, br.grad) < 2e-2


def test_bias_dropout_add_matches_cpu_mask():
    from fleetx_amd import ops
    x = torch.randn(64, 1024, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    b = torch.randn(1024, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(64, 1024, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    out = ops.bias_dropout_add(x, b, r, 0.1, 42)
    out_cpu = ops.bias_dropout_add(x.detach().cpu().float(), b.detach().cpu().float(),
                                   r.detach().cpu().float(), 0.1, 42)
    assert _rel(out.cpu(), out_cpu) < 1e-2
    keep_frac = ((out.float() - r.float()) != 0).float().mean().item()
    assert 0.88 < keep_frac < 0.92
    g = torch.randn_like(out)
    out.backward(g)
    xr = x.detach().cpu().float().requires_grad_()
    br = b.detach().cpu().float().requires_grad_()
    o2 = ops.bias_dropout_add(xr, br, r.detach().cpu().float(), 0.1, 42)
    o2.backward(g.cpu().float())
    assert _rel(x.grad.cpu(), xr.grad) < 1e-2
    assert _rel(b.grad.cpu(), br.grad) < 1e-2
    assert torch.equal(r.grad, g)


# ---------------------------------------------------------------- CE / embedding
def test_cross_entropy():
    from fleetx_amd import ops
    V = 50304
    logits = (3 * torch.randn(256, V, device=DEV)).bfloat16().requires_grad_()
    labels = torch.randint(0, V, (256,), device=DEV)
    ref_in = logits.detach().float().requires_grad_()
    loss = ops.softmax_cross_entropy(logits.clone(), labels)
    lr_ = torch.nn.functional.cross_entropy(ref_in, labels, reduction="none")
    assert torch.allclose(loss, lr_, atol=2e-3, rtol=1e-3)
    lg = logits.detach().clone().requires_grad_()
    l2 = ops.softmax_cross_entropy(lg, labels, inplace_backward=False)
    g = torch.rand(256, device=DEV)
    (l2 * g).sum().backward()
    (lr_ * g).sum().backward()
    assert _rel(lg.grad, ref_in.grad) < 1e-2


def test_embedding():
    from fleetx_amd import ops
    V, h = 1000, 512
    W = torch.randn(V, h, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    P = torch.randn(128, h, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    ids = torch.randint(0, V, (4, 128), device=DEV)
    pos = torch.arange(128, device=DEV).expand(4, 128)
    out = ops.embedding(ids, W, pos, P)
    ref = W.detach().float()[ids] + P.detach().float()[pos]
    assert _rel(out, ref) < 1e-2
    g = torch.randn_like(out)
    out.backward(g)
    Wr, Pr = W.detach().float().requires_grad_(), P.detach().float().requires_grad_()
    (torch.nn.functional.embedding(ids, Wr) + Pr[pos]).backward(g.float())
    assert _rel(W.grad, Wr.grad) < 1e-2
    assert _rel(P.grad, Pr.grad) < 1e-2
    # vocab shard: ids outside [500, 1000) give zeros
    Ws = W.detach()[500:].contiguous()
    out2 = ops.embedding(ids, Ws, vocab_start=500)
    ref2 = torch.where((ids >= 500)[..., None], W.detach().float()[ids], torch.zeros(()))
    assert _rel(out2, ref2) < 1e-2


# ---------------------------------------------------------------- attention
@pytest.mark.parametrize("D", [64, 96, 128])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_flash_attention(D, causal, p):
    from fleetx_amd import ops
    B, S, H = 2, 384, 4
    qkv = (0.5 * torch.randn(B, S, H, 3, D, device=DEV)).bfloat16().requires_grad_()
    key = 123456789
    out = ops.flash_attention_qkvpacked(qkv, causal=causal, dropout_p=p, key=key)
    ref_in = qkv.detach().float().requires_grad_()
    ref = ops.attention_reference(ref_in[:, :, :, 0], ref_in[:, :, :, 1], ref_in[:, :, :, 2],
                                  causal=causal, dropout_p=p, key=key)
    assert _rel(out, ref) < 2e-2, _rel(out, ref)
    g = torch.randn_like(ref)
    out.backward(g.bfloat16())
    ref.backward(g)
    for i in range(3):
        assert _rel(qkv.grad[:, :, :, i], ref_in.grad[:, :, :, i]) < 3e-2, (i, _rel(
            qkv.grad[:, :, :, i], ref_in.grad[:, :, :, i]))


@pytest.mark.parametrize("D", [128, 40])
def test_flash_attention_row_store_fallback(D, monkeypatch):
    """store_row16 writes whole 16-byte row chunks after the lane-pair swap;
    rows that are not 16-byte aligned take 8-byte halves of the same swapped
    registers (FLEETX_FA_ROW16=0 forces that path): bitwise the same O, dQ,
    dK, dV."""
    from fleetx_amd import ops
    B, S, H = 2, 300, 4
    torch.manual_seed(0)
    qkv0 = (0.5 * torch.randn(B, S, H, 3, D, device=DEV)).bfloat16()
    g = torch.randn(B, S, H, D, device=DEV).bfloat16()

    def run():
        qkv = qkv0.clone().requires_grad_()
        out = ops.flash_attention_qkvpacked(qkv, causal=True, dropout_p=0.1, key=77)
        out.backward(g)
        return out.detach(), qkv.grad
    o16, g16 = run()
    monkeypatch.setenv("FLEETX_FA_ROW16", "0")
    o8, g8 = run()
    monkeypatch.delenv("FLEETX_FA_ROW16")
    torch.cuda.synchronize()
    assert torch.equal(o16, o8)
    assert torch.equal(g16, g8)


@pytest.mark.parametrize("causal", [True, False])
def test_flash_attention_rescale_branch(causal):
    """Deferred online-softmax rescale (FA_RESCALE_THR = 8, log2 units): one key
    row whose scores jump ~13 log2 units mid-row forces the rescale branch at
    a later tile, a second one (~6.5) grows the max WITHOUT a rescale (p up to
    2^6.5 against the stale max).  Full-tensor fp32 reference, fwd + bwd."""
    from fleetx_amd import ops
    B, S, H, D = 1, 512, 2, 128
    torch.manual_seed(7)
    q = (0.5 * torch.randn(B, S, H, D, device=DEV)).abs()
    k = 0.5 * torch.randn(B, S, H, D, device=DEV)
    v = torch.randn(B, S, H, D, device=DEV)
    k[:, 100] = 1.0   # +~6.5 in log2 units: below the threshold
    k[:, 300] = 2.0   # +~13: forces the rescale inside the 5th 64-key tile
    q, k, v = [t.bfloat16().requires_grad_() for t in (q, k, v)]
    out = ops.flash_attention(q, k, v, causal=causal)
    qr, kr, vr = [t.detach().float().requires_grad_() for t in (q, k, v)]
    ref = ops.attention_reference(qr, kr, vr, causal=causal)
    assert _rel(out, ref) < 2e-2, _rel(out, ref)
    g = torch.randn_like(ref)
    out.backward(g.bfloat16())
    ref.backward(g)
    for a, r in ((q, qr), (k, kr), (v, vr)):
        assert _rel(a.grad, r.grad) < 3e-2, _rel(a.grad, r.grad)


@pytest.mark.parametrize("D", [88, 128])
def test_flash_attention_packed_vit_layout(D):
    """[B, S, 3, H, D] packed QKV (ViT / timm order, pack_dim=2): output and the
    packed gradient vs the fp32 reference."""
    from fleetx_amd import ops
    B, S, H = 2, 257, 4
    qkv = (0.5 * torch.randn(B, S, 3, H, D, device=DEV)).bfloat16().requires_grad_()
    out = ops.flash_attention_qkvpacked(qkv, causal=False, pack_dim=2, scale=D ** -0.5)
    ref_in = qkv.detach().float().requires_grad_()
    ref = ops.attention_reference(ref_in[:, :, 0], ref_in[:, :, 1], ref_in[:, :, 2], causal=False)
    assert _rel(out, ref) < 2e-2, _rel(out, ref)
    g = torch.randn_like(ref)
    out.backward(g.bfloat16())
    ref.backward(g)
    assert qkv.grad.shape == qkv.shape
    for i in range(3):
        assert _rel(qkv.grad[:, :, i], ref_in.grad[:, :, i]) < 3e-2


def test_flash_attention_tail_and_kvlens():
    from fleetx_amd import ops
    B, S, H, D = 2, 200, 2, 128
    q = torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    lens = torch.tensor([150, 200], device=DEV, dtype=torch.int32)
    out = ops.flash_attention(q, k, v, causal=False, kv_lens=lens)
    qr, kr, vr = [t.detach().float().requires_grad_() for t in (q, k, v)]
    ref = ops.attention_reference(qr, kr, vr, causal=False, kv_lens=lens)
    assert _rel(out, ref) < 2e-2
    g = torch.randn_like(ref)
    out.backward(g.bfloat16())
    ref.backward(g)
    for a, r in ((q, qr), (k, kr), (v, vr)):
        assert _rel(a.grad, r.grad) < 3e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("nsplit", [1, None, 7])
@pytest.mark.parametrize("BH", [(3, 4), (8, 32)])
def test_decode_attention(dtype, D, nsplit, BH):
    """Split-K decode vs fp32: ragged lengths, splits that end up empty; few
    (batch, head) pairs run the 16-wave workgroup, many the 4-wave one."""
    from fleetx_amd import ops
    (B, H), L = BH, 1300
    q = torch.randn(B, H, D, device=DEV, dtype=dtype)
    kc = torch.randn(B, L, H, D, device=DEV, dtype=dtype)
    vc = torch.randn(B, L, H, D, device=DEV, dtype=dtype)
    lens = torch.tensor([1300, 17, 700, 1, 64, 513, 999, 1299][:B], device=DEV, dtype=torch.int32)
    out = ops.decode_attention(q, kc, vc, lens, nsplit=nsplit)
    assert out.dtype == dtype
    ref = ops.decode_attention(q.cpu().float(), kc.cpu().float(), vc.cpu().float(), lens.cpu())
    assert _rel(out.cpu(), ref) < 1e-2


@pytest.mark.parametrize("D", [64, 96, 128])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_attention_fp16(D, causal):
    """fp16 flash forward + backward (f16 MFMA path) vs fp32."""
    from fleetx_amd import ops
    B, S, H = 2, 320, 4
    qkv = (0.5 * torch.randn(B, S, H, 3, D, device=DEV)).half().requires_grad_()
    out = ops.flash_attention_qkvpacked(qkv, causal=causal)
    assert out.dtype == torch.float16
    ref_in = qkv.detach().float().requires_grad_()
    ref = ops.attention_reference(ref_in[:, :, :, 0], ref_in[:, :, :, 1], ref_in[:, :, :, 2],
                                  causal=causal)
    assert _rel(out, ref) < 5e-3, _rel(out, ref)
    g = torch.randn_like(ref)
    out.backward(g.half())
    ref.backward(g)
    for i in range(3):
        assert _rel(qkv.grad[:, :, :, i], ref_in.grad[:, :, :, i]) < 1e-2


# ---------------------------------------------------------------- optimizer
def test_fused_adamw_matches_torch():
    from fleetx_amd.parallel.grad_buffer import FlatParamGradBuffer
    from fleetx_amd.optims.optimizer import FusedAdamW, ClipGradByGlobalNorm
    torch.manual_seed(1)
    lin = torch.nn.Linear(256, 512).cuda().bfloat16()
    ref = torch.nn.Linear(256, 512).cuda()
    with torch.no_grad():
        ref.weight.copy_(lin.weight.float())
        ref.bias.copy_(lin.bias.float())
    buf = FlatParamGradBuffer(lin.named_parameters())
    opt = FusedAdamW(1e-2, buf, grad_clip=ClipGradByGlobalNorm(0.5), weight_decay=0.1)
    topt = torch.optim.AdamW([{"params": [ref.weight], "weight_decay": 0.1},
                              {"params": [ref.bias], "weight_decay": 0.0}], lr=1e-2,
                             eps=1e-8)
    for _ in range(3):
        x = torch.randn(64, 256, device=DEV)
        lin(x.bfloat16()).float().pow(2).mean().backward()
        buf.finish()
        g = [p.main_grad.float().clone() for _, p in buf.params]
        ref.weight.grad = dict((id(p), gg) for (_, p), gg in zip(buf.params, g))[id(lin.weight)].clone()
        ref.bias.grad = dict((id(p), gg) for (_, p), gg in zip(buf.params, g))[id(lin.bias)].clone()
        torch.nn.utils.clip_grad_norm_(ref.parameters(), 0.5)
        opt.step()
        opt.clear_grad()
        topt.step()
        topt.zero_grad()
    assert _rel(lin.weight, ref.weight) < 1e-2
    assert _rel(lin.bias, ref.bias) < 1e-2


def test_offloaded_adamw_matches_resident():
    """sharding_offload: host-pinned fp32 state streamed through the GPU in
    chunks gives bit-identical updates to the device-resident optimizer."""
    from fleetx_amd.parallel.grad_buffer import FlatParamGradBuffer
    from fleetx_amd.optims import optimizer as O
    torch.manual_seed(3)
    old = O._OFFLOAD_CHUNK
    O._OFFLOAD_CHUNK = 4096  # force many chunks / both staging buffers
    try:
        mods, opts, bufs = [], [], []
        for off in (False, True):
            torch.manual_seed(3)
            m = torch.nn.Sequential(torch.nn.Linear(128, 192), torch.nn.Linear(192, 64)).cuda()
            m = m.bfloat16()
            b = FlatParamGradBuffer(m.named_parameters())
            o = O.FusedAdamW(1e-2, b, grad_clip=O.ClipGradByGlobalNorm(0.5), weight_decay=0.1,
                             offload=off)
            assert o.offload == off
            mods.append(m), opts.append(o), bufs.append(b)
        for step in range(3):
            x = torch.randn(32, 128, device=DEV, dtype=torch.bfloat16)
            for m, o, b in zip(mods, opts, bufs):
                m(x).float().pow(2).mean().backward()
                b.finish()
                o.step()
                o.clear_grad()
        torch.cuda.synchronize()
        for (_, p0), (_, p1) in zip(mods[0].named_parameters(), mods[1].named_parameters()):
            assert torch.equal(p0, p1)
        s0, s1 = opts[0].state_dict(), opts[1].state_dict()
        for a, b in zip(s0["m"], s1["m"]):
            assert torch.equal(a.cpu(), b.cpu())
    finally:
        O._OFFLOAD_CHUNK = old


def test_forward_overlapped_adamw_matches_serial(monkeypatch):
    """Step N's update on a side stream, gated per layer by the next forward,
    reproduces the serial update exactly.  Bitwise needs the deterministic
    embedding backward: the default one adds rows with fp32 atomics, whose
    order (and so the gradient norm, and so every clipped update) varies in
    the last bits from run to run."""
    monkeypatch.setenv("FLEETX_DETERMINISTIC", "1")
    from fleetx_amd.models.language_model.gpt.model import (GPTConfig, GPTForPretraining,
                                                            GPTPretrainingCriterion)
    from fleetx_amd.parallel.grad_buffer import FlatParamGradBuffer
    from fleetx_amd.optims.optimizer import FusedAdamW, ClipGradByGlobalNorm
    runs = []
    for overlap in (False, True):
        torch.manual_seed(0)
        cfg = GPTConfig(vocab_size=1024, hidden_size=256, num_layers=3, num_attention_heads=4,
                        max_position_embeddings=128, hidden_dropout_prob=0.0,
                        attention_probs_dropout_prob=0.0, dtype=torch.bfloat16)
        model = GPTForPretraining(cfg).cuda()
        crit = GPTPretrainingCriterion(cfg)
        buf = FlatParamGradBuffer(model.named_parameters())
        opt = FusedAdamW(1e-3, buf, grad_clip=ClipGradByGlobalNorm(1.0), weight_decay=0.01)
        if overlap:
            assert opt.enable_forward_overlap(model)
            assert len(opt._overlap_groups) == 4  # root + 3 layers
        g = torch.Generator(device=DEV).manual_seed(5)
        losses = []
        for _ in range(4):
            toks = torch.randint(0, 1024, (4, 129), device=DEV, generator=g)
            loss = crit(model(toks[:, :-1]), toks[:, 1:], torch.ones(4, 128, device=DEV))
            loss.backward()
            buf.finish()
            opt.step()
            opt.clear_grad()
            losses.append(loss.detach())
        opt.sync_state()
        runs.append(([l.item() for l in losses], [p.detach().clone() for p in model.parameters()]))
    assert runs[0][0] == runs[1][0], (runs[0][0], runs[1][0])
    for a, b in zip(runs[0][1], runs[1][1]):
        assert torch.equal(a, b)


def test_hip_graph_decode_matches_eager():
    """The HIP-graph-replayed decode step generates exactly the eager tokens."""
    import time
    from fleetx_amd.models.language_model.gpt.model import GPTConfig, GPTForPretraining
    from fleetx_amd.models.language_model.gpt.generation import GPTForGeneration
    torch.manual_seed(0)
    cfg = GPTConfig(vocab_size=1024, hidden_size=256, num_layers=4, num_attention_heads=4,
                    max_position_embeddings=256, hidden_dropout_prob=0.0,
                    attention_probs_dropout_prob=0.0, dtype=torch.bfloat16)
    model = GPTForPretraining(cfg).cuda().eval()
    prompt = torch.randint(0, 1024, (3, 17), device=DEV)
    lens = torch.tensor([17, 9, 12], device=DEV)
    outs, times = [], []
    for graph in (False, True):
        gen = GPTForGeneration(model, {"max_dec_len": 48, "decode_strategy": "greedy_search",
                                       "use_hip_graph": graph})
        gen.generate(prompt, lens)  # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ids, scores = gen.generate(prompt, lens)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        outs.append((ids.cpu(), scores.cpu()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.allclose(outs[0][1], outs[1][1], atol=1e-3)
    print("decode eager %.2f ms/token, hip graph %.2f ms/token"
          % (1e3 * times[0] / 48, 1e3 * times[1] / 48))


def test_fake_quant():
    from fleetx_amd.ops import quant
    x = torch.randn(1000, device=DEV, dtype=torch.bfloat16)
    s = quant.absmax(x)
    assert abs(s.item() - x.float().abs().max().item()) < 1e-6
    y = quant.fake_quant(x, s, 8)
    yr = quant.fake_quant(x.cpu().float(), s.cpu(), 8)
    assert _rel(y.cpu(), yr) < 1e-2


# ---------------------------------------------------------------- end-to-end
def test_gpt_train_step_loss_decreases():
    from fleetx_amd.models.language_model.gpt.model import (GPTConfig, GPTForPretraining,
                                                            GPTPretrainingCriterion)
    from fleetx_amd.parallel.grad_buffer import FlatParamGradBuffer
    from fleetx_amd.optims.optimizer import FusedAdamW, ClipGradByGlobalNorm
    cfg = GPTConfig(vocab_size=2048, hidden_size=256, num_layers=2, num_attention_heads=4,
                    max_position_embeddings=256, dtype=torch.bfloat16)
    model = GPTForPretraining(cfg).cuda()
    crit = GPTPretrainingCriterion(cfg)
    buf = FlatParamGradBuffer(model.named_parameters())
    opt = FusedAdamW(2e-3, buf, grad_clip=ClipGradByGlobalNorm(1.0))
    toks = torch.randint(0, 2048, (4, 257), device=DEV)
    losses = []
    for _ in range(8):
        loss = crit(model(toks[:, :-1]), toks[:, 1:], torch.ones(4, 256, device=DEV))
        loss.backward()
        buf.finish()
        opt.step()
        opt.clear_grad()
        losses.append(loss.item())
    assert abs(losses[0] - math.log(2048)) < 0.5
    assert losses[-1] < losses[0] - 0.5, losses


@pytest.mark.parametrize("D", [40, 88, 112, 100])
def test_flash_attention_padded_head_dim(D):
    """Head dims that are not a tile width: multiples of 8 (ViT-g: 88 on the 96
    tile) run natively with zero-read columns, others (100) via padded copies."""
    from fleetx_amd import ops
    B, S, H = 2, 257, 4  # ViT-style odd token count (cls + 16x16 patches)
    q, k, v = [torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
               for _ in range(3)]
    out = ops.flash_attention(q, k, v, causal=False)
    assert out.shape == (B, S, H, D)
    qr, kr, vr = [t.detach().float().requires_grad_() for t in (q, k, v)]
    ref = ops.attention_reference(qr, kr, vr, causal=False)
    assert _rel(out, ref) < 2e-2
    g = torch.randn_like(ref)
    out.backward(g.bfloat16())
    ref.backward(g)
    for a, r in ((q, qr), (k, kr), (v, vr)):
        assert _rel(a.grad, r.grad) < 3e-2


@pytest.mark.parametrize("S", [257, 190, 96])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_flash_attention_three_wave_tiles(S, causal, p):
    """96-wide tiles over row counts where 3-wave workgroups leave fewer idle
    waves (flash_attn.hip waves_for: ViT-g's 257 tokens): forward, dQ and
    dK/dV with 96-row workgroups, causal and dropout included, vs fp32."""
    from fleetx_amd import ops
    B, H, D = 2, 3, 88
    key = 1234
    qkv = (0.5 * torch.randn(B, S, 3, H, D, device=DEV)).bfloat16().requires_grad_()
    out = ops.flash_attention_qkvpacked(qkv, causal=causal, dropout_p=p, key=key, pack_dim=2)
    ref_in = qkv.detach().float().requires_grad_()
    ref = ops.attention_reference(ref_in[:, :, 0], ref_in[:, :, 1], ref_in[:, :, 2],
                                  causal=causal, dropout_p=p, key=key)
    assert _rel(out, ref) < 2e-2, _rel(out, ref)
    g = torch.randn_like(ref)
    out.backward(g.bfloat16())
    ref.backward(g)
    for i in range(3):
        assert _rel(qkv.grad[:, :, i], ref_in.grad[:, :, i]) < 3e-2, (i, _rel(qkv.grad[:, :, i], ref_in.grad[:, :, i]))


def test_vit_train_step_on_gpu():
    from fleetx_amd.models.vision_model.vit import ViT
    from fleetx_amd.models.vision_model.loss import ViTCELoss
    from fleetx_amd.parallel.grad_buffer import FlatParamGradBuffer
    from fleetx_amd.optims.optimizer import FusedAdamW
    m = ViT(img_size=64, patch_size=8, class_num=10, embed_dim=256, depth=2, num_heads=4,
            qkv_bias=True, epsilon=1e-6).cuda().bfloat16()
    buf = FlatParamGradBuffer(m.named_parameters())
    opt = FusedAdamW(1e-3, buf)
    x = torch.randn(8, 3, 64, 64, device=DEV)
    y = torch.arange(8, device=DEV) % 10
    losses = []
    for _ in range(10):
        loss = ViTCELoss()(m(x), y)
        loss.backward()
        buf.finish()
        opt.step()
        opt.clear_grad()
        losses.append(loss.item())
    assert losses[-1] < losses[0], losses


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_flash_attention_key_bias(D, p):
    """Additive per-key bias (BERT/ERNIE padding mask) evaluated in-kernel."""
    from fleetx_amd import ops
    B, S, H = 3, 300, 2
    qkv = (0.5 * torch.randn(B, S, H, 3, D, device=DEV)).bfloat16().requires_grad_()
    kb = torch.zeros(B, S, device=DEV)
    kb[1, 200:] = -1e4
    kb[2, ::3] = -1e4
    kb[0] = 0.3 * torch.randn(S, device=DEV)
    key = 987654321
    out = ops.flash_attention_qkvpacked(qkv, causal=False, dropout_p=p, key=key, key_bias=kb)
    ref_in = qkv.detach().float().requires_grad_()
    ref = ops.attention_reference(ref_in[:, :, :, 0], ref_in[:, :, :, 1], ref_in[:, :, :, 2],
                                  causal=False, dropout_p=p, key=key, key_bias=kb)
    assert _rel(out, ref) < 2e-2, _rel(out, ref)
    g = torch.randn_like(ref)
    out.backward(g.bfloat16())
    ref.backward(g)
    for i in range(3):
        assert _rel(qkv.grad[:, :, :, i], ref_in.grad[:, :, :, i]) < 3e-2


def test_ernie_train_step_on_gpu():
    from fleetx_amd.models.language_model.ernie import (ErnieModel, ErnieForPretraining,
                                                        ErniePretrainingCriterion, mlm_mask)
    from fleetx_amd.parallel.grad_buffer import FlatParamGradBuffer
    from fleetx_amd.optims.optimizer import FusedAdamW
    m = ErnieForPretraining(ErnieModel(vocab_size=1024, hidden_size=256, num_hidden_layers=2,
                                       num_attention_heads=4, intermediate_size=1024,
                                       dtype=torch.bfloat16)).cuda()
    crit = ErniePretrainingCriterion(with_nsp_loss=False)
    buf = FlatParamGradBuffer(m.named_parameters())
    opt = FusedAdamW(1e-3, buf)
    toks = torch.randint(1, 1024, (4, 128), device=DEV)
    toks[1, 100:] = 0
    g = torch.Generator(device=DEV).manual_seed(0)
    inp, lab = mlm_mask(toks, 1024, 1023, 0.15, special_ids=(0,), generator=g)
    pos = torch.nonzero(lab.reshape(-1) >= 0).reshape(-1)
    losses = []
    for _ in range(10):
        scores, rel = m(inp, masked_positions=pos)
        loss = crit(scores, rel, lab.reshape(-1)[pos])
        loss.backward()
        buf.finish()
        opt.step()
        opt.clear_grad()
        losses.append(loss.item())
    assert losses[-1] < losses[0] - 0.5, losses


@pytest.mark.parametrize("shape,G", [((2, 64, 16, 16), 8), ((1, 128, 64, 64), 8), ((3, 32, 5, 7), 4),
                                     ((1, 64, 256, 256), 8)])
@pytest.mark.parametrize("film", [False, True])
def test_group_norm_silu(shape, G, film):
    from fleetx_amd import ops
    from fleetx_amd.ops.groupnorm import group_norm_silu_reference
    B, C = shape[:2]
    x = (torch.randn(shape, device=DEV) * 2 + 0.5).bfloat16().requires_grad_()
    w = (1 + 0.1 * torch.randn(C, device=DEV)).requires_grad_()
    b = (0.1 * torch.randn(C, device=DEV)).requires_grad_()
    sc = (0.2 * torch.randn(B, C, device=DEV)).requires_grad_() if film else None
    sh = (0.2 * torch.randn(B, C, device=DEV)).requires_grad_() if film else None
    y = ops.group_norm_silu(x, G, w, b, sc, sh)
    leaves = [t for t in (x, w, b, sc, sh) if t is not None]
    refs = [t.detach().float().requires_grad_() for t in leaves]
    rx, rw, rb = refs[:3]
    rsc, rsh = (refs[3], refs[4]) if film else (None, None)
    yr = group_norm_silu_reference(rx, G, rw, rb, rsc, rsh)
    assert _rel(y, yr) < 1e-2
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    for a, r in zip(leaves, refs):
        assert _rel(a.grad, r.grad) < 2e-2, (a.shape, _rel(a.grad, r.grad))


def test_flash_attention_multi_query_broadcast():
    """Imagen multi-query attention: one K/V head broadcast by a stride-0 view."""
    from fleetx_amd import ops
    B, Sq, Sk, H, D = 2, 257, 70, 8, 64
    q = torch.randn(B, Sq, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, Sk, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, Sk, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    out = ops.flash_attention(q, k.unsqueeze(2).expand(B, Sk, H, D),
                              v.unsqueeze(2).expand(B, Sk, H, D), causal=False)
    qr, kr, vr = [t.detach().float().requires_grad_() for t in (q, k, v)]
    ref = ops.attention_reference(qr, kr.unsqueeze(2).expand(B, Sk, H, D),
                                  vr.unsqueeze(2).expand(B, Sk, H, D), causal=False)
    assert _rel(out, ref) < 2e-2
    g = torch.randn_like(ref)
    out.backward(g.bfloat16())
    ref.backward(g)
    for a, r in ((q, qr), (k, kr), (v, vr)):
        assert _rel(a.grad, r.grad) < 3e-2


def test_imagen_unet_train_step_on_gpu():
    from fleetx_amd.models.multimodal_model.imagen import Unet, ImagenModel, ImagenCriterion
    torch.manual_seed(0)
    u = Unet(dim=64, dim_mults=(1, 2), num_resnet_blocks=1, layer_attns=(False, True),
             layer_cross_attns=(False, True), attn_heads=4, attn_dim_head=64, max_text_len=16,
             attn_pool_num_latents=8)
    m = ImagenModel(unets=u, image_sizes=(32,), text_embed_dim=64, timesteps=10).cuda().bfloat16()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    img = torch.rand(4, 3, 32, 32, device=DEV)
    te = torch.randn(4, 12, 64, device=DEV)
    crit = ImagenCriterion()
    for _ in range(3):
        pred, target, ls, gamma = m(img, text_embeds=te)
        loss = crit(pred, target, ls, gamma)
        loss.backward()
        opt.step()
        opt.zero_grad()
        assert torch.isfinite(loss)
    out = m.sample(text_embeds=te[:2], cond_scale=2.0)
    assert out.shape == (2, 3, 32, 32) and torch.isfinite(out).all()


@pytest.mark.parametrize("R,C", [(64, 64), (136, 200), (8192, 1024), (24, 4104)])
def test_transpose2d(R, C):
    from fleetx_amd.ops.elementwise import transpose2d
    x = torch.randn(R, C + 16, device="cuda").to(torch.bfloat16)[:, :C]  # strided rows
    y = transpose2d(x)
    assert y.shape == (C, R) and y.is_contiguous()
    assert torch.equal(y, x.t().contiguous())
    cs = torch.full((C,), 1.0, device="cuda")
    y2 = transpose2d(x, colsum=(cs, True))
    assert torch.equal(y2, y)
    torch.testing.assert_close(cs, 1.0 + x.float().sum(0), rtol=1e-4, atol=1e-3)


def test_tn_wgrad_matches_direct():
    from fleetx_amd.parallel import linear as L
    torch.manual_seed(0)
    M, N, K = 2048, 384, 256
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    ref = dy.float().t() @ x.float()
    for _ in range(1):
        w = torch.nn.Parameter(torch.zeros(N, K, device="cuda", dtype=torch.bfloat16))
        w.main_grad = torch.full((N, K), 7.0, device="cuda")
        w._fx_fresh = True
        b = torch.nn.Parameter(torch.zeros(N, device="cuda", dtype=torch.bfloat16))
        b.main_grad = torch.full((N,), 7.0, device="cuda")
        b._fx_fresh, b._fx_fused_wgrad = True, True
        b2 = torch.nn.Parameter(torch.zeros(N, device="cuda", dtype=torch.bfloat16))
        assert L._tn_operands(dy, x) is not None
        assert L.accumulate_wgrad(w, dy, x, b) is None   # fresh: overwrite
        L.accumulate_wgrad(w, dy, x, b)                  # accumulate
        db = L.accumulate_wgrad(w, dy, x, b2)            # unfused bias: returned
        torch.testing.assert_close(w.main_grad, 3 * ref, rtol=2e-3, atol=3e-2)
        torch.testing.assert_close(b.main_grad, 2 * dy.float().sum(0), rtol=1e-3, atol=1e-2)
        torch.testing.assert_close(db.float(), dy.float().sum(0), rtol=1e-2, atol=1e-1)


# ---------------------------------------------------------------- fused sampling (K18)
@pytest.mark.parametrize("T,k,p", [(1.0, 50, 1.0), (0.7, 0, 0.9), (0.8, 40, 0.8), (1.3, 0, 1.0)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_fused_sample_filter_matches_reference(T, k, p, dtype):
    from fleetx_amd.ops import fused_sample
    from fleetx_amd.models.language_model.gpt.generation import top_k_filter, top_p_filter
    logits = (torch.randn(4, 50304, device="cuda") * 3).to(dtype)
    ids, lse, probs = fused_sample(logits, T, k, p, return_probs=True)
    ref = torch.softmax(logits.float() / T, -1)
    if k:
        ref = top_k_filter(ref, k)
    if p < 1.0:
        ref = top_p_filter(ref, p)
    diff = (probs > 0) != (ref > 0)
    if diff.any():
        # only ties at the nucleus boundary (bf16 logits repeat values) may differ:
        # the kernel keeps every token equal to the threshold, a sort cuts inside the tie
        assert dtype == torch.bfloat16 and p < 1.0
        kmin = torch.where(probs > 0, probs, torch.full_like(probs, 2.0)).min(-1, keepdim=True).values
        assert torch.allclose(probs[diff], kmin.expand_as(probs)[diff], rtol=1e-6)
        ref = torch.where(diff, probs, ref)
    torch.testing.assert_close(probs, ref, rtol=1e-4, atol=1e-7)
    torch.testing.assert_close(lse, torch.logsumexp(logits.float(), -1), rtol=1e-5, atol=1e-4)
    assert bool((ref.gather(1, ids[:, None]) > 0).all())  # drawn tokens survive the filters


def test_fused_sample_greedy_and_distribution():
    from fleetx_amd.ops import fused_sample
    logits = torch.randn(8, 1000, device="cuda")
    ids, _ = fused_sample(logits, 1.0, 1, 1.0)
    assert torch.equal(ids, logits.argmax(-1))
    ids, _ = fused_sample(logits, 1.0, 0, 1e-6)  # nucleus of one token
    assert torch.equal(ids, logits.argmax(-1))
    row = torch.randn(1, 24, device="cuda")
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    ids, _ = fused_sample(row.expand(40000, 24).contiguous(), 1.0, 0, 1.0, generator=g)
    freq = torch.bincount(ids, minlength=24).float() / ids.numel()
    assert (freq - torch.softmax(row[0], -1)).abs().max().item() < 0.01


def test_early_grad_norm_matches_post_backward_norm():
    """Per-bucket sum of squares on a side stream under backward == the
    post-backward norm pass; training curves identical."""
    from fleetx_amd.models.language_model.gpt.model import (GPTConfig, GPTForPretraining,
                                                            GPTPretrainingCriterion)
    from fleetx_amd.parallel.grad_buffer import FlatParamGradBuffer
    from fleetx_amd.optims.optimizer import FusedAdamW, ClipGradByGlobalNorm
    toks = torch.randint(0, 2048, (4, 257), device=DEV)
    runs = []
    for early in (False, True):
        torch.manual_seed(0)
        cfg = GPTConfig(vocab_size=2048, hidden_size=256, num_layers=4, num_attention_heads=4,
                        max_position_embeddings=256, dtype=torch.bfloat16,
                        hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
        model = GPTForPretraining(cfg).cuda()
        crit = GPTPretrainingCriterion(cfg)
        buf = FlatParamGradBuffer(model.named_parameters(), bucket_mb=1)
        assert buf.enable_early_norm() if early else True
        assert len(buf.buckets) > 3
        opt = FusedAdamW(2e-3, buf, grad_clip=ClipGradByGlobalNorm(0.5))
        norms = []
        for _ in range(3):
            loss = crit(model(toks[:, :-1]), toks[:, 1:], torch.ones(4, 256, device=DEV))
            loss.backward()
            buf.finish()
            assert (buf.early_norm is not None) == early
            opt.step()
            opt.clear_grad()
            norms.append(float(opt.last_grad_norm))
        runs.append(norms)
    for a, b in zip(*runs):
        assert abs(a - b) <= 1e-4 * a, runs


def test_profiler_kernel_view_shows_hip_kernels(tmp_path):
    from tests.test_engine_cpu import CFG
    from fleetx_amd.utils import config as C
    from fleetx_amd.utils import env
    from fleetx_amd.models import build_module
    from fleetx_amd.core.engine.eager_engine import EagerEngine
    ov = ["Model.hidden_size=256", "Model.num_layers=2", "Model.num_attention_heads=4",
          "Model.vocab_size=1024", "Model.max_position_embeddings=256",
          "Global.local_batch_size=4", "Global.micro_batch_size=4", "Engine.max_steps=5",
          "Engine.logging_freq=1000", "Engine.mix_precision.dtype=bfloat16",
          "Engine.save_load.output_dir=%s" % tmp_path, "Data.Train.dataset.max_seq_len=256",
          "Data.Train.dataset.name=SyntheticGPTDataset", "Profiler.enable=True",
          "Profiler.scheduler=[2,4]", "Profiler.profiler_log=%s" % (tmp_path / "prof")]
    cfg = C.get_config(CFG, overrides=ov, nranks=1)
    env.set_seed(cfg.Global.seed)
    eng = EagerEngine(configs=cfg, module=build_module(cfg), mode="train")
    g = torch.Generator().manual_seed(0)

    class _Loader:
        def __iter__(self):
            for _ in range(6):
                t = torch.randint(0, 1024, (4, 257), generator=g)
                yield [t[:, :-1].contiguous(), torch.arange(256).expand(4, 256).contiguous(),
                       t[:, 1:].contiguous(), torch.ones(4, 256)]

        def __len__(self):
            return 6

    eng.fit(epoch=1, train_data_loader=_Loader())
    text = (tmp_path / "prof" / "summary_rank0.txt").read_text()
    kern = text.split("Kernel Summary")[1].split("Operator Summary")[0]
    assert "fa_fwd_kernel" in kern and "adamw_flat_kernel" in kern, text
    model = text.split("Model Summary")[1].split("Kernel Summary")[0]
    fwd = [l for l in model.splitlines() if l.startswith("Forward")][0]
    assert float(fwd.split("|")[3]) > 0.0, model  # device time attributed to the phase


def test_tn_dgrad_matches_matmul():
    from fleetx_amd.parallel import linear as L
    dy = torch.randn(16, 512, 384, device="cuda").to(torch.bfloat16)
    w = torch.randn(384, 1024, device="cuda").to(torch.bfloat16)
    ref = dy.float() @ w.float()
    out = L.dgrad(dy, w)
    assert out.shape == (16, 512, 1024)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-1)
    assert torch.equal(out, L.F.linear(dy, w.t().contiguous()))


# ---------------------------------------------------------------- fused softmax (K04)
@pytest.mark.parametrize("Sk", [256, 1024, 4096, 200, 6000])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_softmax_mask_fuse_upper_triangle(Sk, dtype):
    from fleetx_amd.ops.softmax import softmax_mask_fuse_upper_triangle
    B, H = 2, 3
    x = (3 * torch.randn(B, H, Sk, Sk, device=DEV)).to(dtype).requires_grad_()
    y = softmax_mask_fuse_upper_triangle(x, scale=0.5)
    xr = x.detach().float().requires_grad_()
    tri = torch.triu(torch.ones(Sk, Sk, dtype=torch.bool, device=DEV), 1)
    yr = torch.softmax((xr * 0.5).masked_fill(tri, float("-inf")), -1)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert _rel(y, yr) < tol
    assert (y.float().masked_select(tri.expand_as(y)) == 0).all()
    dy = torch.randn_like(yr)
    y.backward(dy.to(dtype))
    yr.backward(dy)
    assert _rel(x.grad, xr.grad) < (1e-4 if dtype == torch.float32 else 3e-2)


@pytest.mark.parametrize("mshape", ["b1", "11", "bh"])
@pytest.mark.parametrize("Sk", [512, 2048, 77])
def test_softmax_mask_fuse(mshape, Sk):
    from fleetx_amd.ops.softmax import softmax_mask_fuse
    B, H, Sq = 2, 4, 64
    x = torch.randn(B, H, Sq, Sk, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    lead = {"b1": (B, 1), "11": (1, 1), "bh": (B, H)}[mshape]
    mask = torch.where(torch.rand(*lead, Sq, Sk, device=DEV) < 0.2, -1e4, 0.0)
    mask[..., 0, :] = float("-inf")  # a fully masked row -> zeros
    y = softmax_mask_fuse(x, mask)
    xr = x.detach().float().requires_grad_()
    yr = torch.nan_to_num(torch.softmax(xr + mask, -1), nan=0.0)
    assert _rel(y, yr) < 2e-2
    assert (y[..., 0, :] == 0).all()
    dy = torch.randn_like(yr)
    y.backward(dy.bfloat16())
    yr.backward(dy)
    # torch's softmax backward of an all -inf row is NaN; the kernel gives 0
    assert (x.grad[..., 0, :] == 0).all()
    assert _rel(x.grad, torch.nan_to_num(xr.grad, nan=0.0)) < 3e-2


def test_unfused_attention_wide_heads():
    """head_dim > 128 runs GEMM + HIP softmax; compare with the fp32 oracle."""
    import warnings
    from fleetx_amd.ops.attention import attention_reference, flash_attention
    B, S, H, D = 2, 256, 2, 160
    q, k, v = (torch.randn(B, S, H, D, device=DEV, dtype=torch.bfloat16, requires_grad=True)
               for _ in range(3))
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        o = flash_attention(q, k, v, causal=True)
    ref = attention_reference(q.detach().float(), k.detach().float(), v.detach().float(), True)
    assert _rel(o, ref) < 2e-2
    o.float().sum().backward()
    assert q.grad is not None and torch.isfinite(q.grad.float()).all()


def test_embedding_bwd_deterministic(monkeypatch):
    """Sorted-segment embedding backward (Global.deterministic) equals the atomic path
    numerically and is bitwise reproducible."""
    from fleetx_amd import ops
    V, h, ntok = 1000, 256, 4096
    ids = torch.randint(0, 50, (ntok,), device=DEV)  # heavy repeats
    w = torch.randn(V, h, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    dy = torch.randn(ntok, h, device=DEV, dtype=torch.bfloat16)

    def grad():
        w.grad = None
        ops.embedding(ids, w).backward(dy)
        return w.grad.float().clone()
    g_atomic = grad()
    monkeypatch.setenv("FLEETX_DETERMINISTIC", "1")
    g1, g2 = grad(), grad()
    assert torch.equal(g1, g2)
    ref = torch.zeros(V, h, device=DEV).index_add_(0, ids, dy.float())
    assert _rel(g1, ref) < 1e-2 and _rel(g_atomic, ref) < 1e-2

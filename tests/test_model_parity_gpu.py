"""Whole-model parity on the GPU: our bf16 model (HIP flash attention, fused
LayerNorm / residual, GEMM epilogues, vocab-parallel CE kernels) against an
INDEPENDENT plain-PyTorch fp32 implementation of the same architecture with
copied weights, dropout off.  Logits, loss and every parameter gradient are
compared with relative-error bounds.

GPT: reference ``gpt/dygraph/single_model.py`` (pre-LN decoder, tied LM head).

Every test runs twice, with the GEMMs forced onto the hand-written MFMA
kernels (``FLEETX_GEMM=hip``) and with the default measured routing
(``auto``), so both GEMM paths are pinned against fp32 torch on purpose.
ERNIE (key-bias padding mask) and ViT (packed-QKV attention, ``pack_dim=2``)
also run in fp16, the dtype of the reference's O2 recipes
(``ViT_base_patch16_224_pt_in1k_2n16c_dp_fp16o2.yaml``).
"""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CFG = os.path.join(os.path.dirname(__file__), "..", "fleetx_amd", "configs", "nlp", "gpt",
                   "pretrain_gpt_345M_single_card.yaml")


@pytest.fixture(autouse=True, params=["hip", "auto"])
def gemm_mode(request):
    from fleetx_amd.ops import gemm as G
    old = G._MODE
    G.set_mode(request.param)
    yield request.param
    G.set_mode(old)


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-6))


def _rel_l2_blocks(a, b, blocks=4):
    """Worst normwise relative error over ``blocks`` row blocks of a
    gradient (the whole tensor for 1-D ones): a gradient term that is off by
    a factor in one part of a fused tensor (the k third of a qkv weight, the
    bias of one head) cannot hide behind the max of the others."""
    a, b = a.detach().float(), b.detach().float()
    if a.dim() < 2 or a.shape[0] < blocks:
        return float((a - b).norm() / b.norm().clamp_min(1e-12))
    worst = 0.0
    for x, y in zip(a.chunk(blocks, 0), b.chunk(blocks, 0)):
        worst = max(worst, float((x - y).norm() / y.norm().clamp_min(1e-12)))
    return worst


def _gpt_reference(P, ids, pos, labels, heads, L, eps=1e-5):
    """Plain fp32 GPT forward + mean CE (no fused ops, no framework code)."""
    b, s = ids.shape
    Hd = P["gpt.embeddings.word_embeddings.weight"].shape[1]
    D = Hd // heads
    x = P["gpt.embeddings.word_embeddings.weight"][ids] + P["gpt.embeddings.position_embeddings"][pos]
    for i in range(L):
        pre = "gpt.layers.%d." % i
        h = F.layer_norm(x, (Hd,), P[pre + "ln1.weight"], P[pre + "ln1.bias"], eps)
        qkv = (h @ P[pre + "attn.qkv_proj.weight"].t() + P[pre + "attn.qkv_proj.bias"])
        qkv = qkv.view(b, s, heads, 3, D)
        q, k, v = (qkv[:, :, :, j].transpose(1, 2) for j in range(3))
        att = (q @ k.transpose(-1, -2)) / D ** 0.5
        mask = torch.ones(s, s, dtype=torch.bool, device=x.device).triu(1)
        att = att.masked_fill(mask, float("-inf")).softmax(-1)
        o = (att @ v).transpose(1, 2).reshape(b, s, Hd)
        x = x + o @ P[pre + "attn.out_proj.weight"].t() + P[pre + "attn.out_proj.bias"]
        h = F.layer_norm(x, (Hd,), P[pre + "ln2.weight"], P[pre + "ln2.bias"], eps)
        a = F.gelu(h @ P[pre + "mlp.fc1.weight"].t() + P[pre + "mlp.fc1.bias"], approximate="tanh")
        x = x + a @ P[pre + "mlp.fc2.weight"].t() + P[pre + "mlp.fc2.bias"]
    x = F.layer_norm(x, (Hd,), P["gpt.final_ln.weight"], P["gpt.final_ln.bias"], eps)
    logits = x @ P["gpt.embeddings.word_embeddings.weight"].t()
    loss = F.cross_entropy(logits.reshape(-1, logits.shape[-1]), labels.reshape(-1))
    return logits, loss


def test_gpt_bf16_hip_vs_fp32_torch():
    from fleetx_amd.utils import config as C
    from fleetx_amd.models import build_module
    from fleetx_amd.parallel import topology as topo
    from fleetx_amd.ops import _lib
    topo.reset_hcg()
    heads, L, V, S, B = 8, 2, 4096, 256, 4
    ov = ["Model.hidden_size=512", "Model.num_layers=%d" % L, "Model.num_attention_heads=%d" % heads,
          "Model.vocab_size=%d" % V, "Model.hidden_dropout_prob=0.0",
          "Model.attention_probs_dropout_prob=0.0", "Model.max_position_embeddings=%d" % S,
          "Global.device=gpu", "Engine.mix_precision.dtype=bfloat16"]
    cfg = C.get_config(CFG, overrides=ov, nranks=1)
    module = build_module(cfg)
    model = module.model.cuda().to(torch.bfloat16)
    assert _lib.kernels() is not None
    torch.manual_seed(0)
    # perturb the zero-initialised biases / unit LN weights so every term is exercised
    with torch.no_grad():
        for n, p in model.named_parameters():
            if p.ndim == 1:
                p.add_(0.05 * torch.randn_like(p))
    ids = torch.randint(0, V, (B, S), device="cuda")
    labels = torch.randint(0, V, (B, S), device="cuda")
    pos = torch.arange(S, device="cuda").unsqueeze(0).expand(B, S)
    P = {n: p.detach().float().clone().requires_grad_(True) for n, p in model.named_parameters()}
    logits = model(ids, pos)
    # the fused CE kernels reuse the logits buffer for the logits gradient
    logits_val = logits.detach().clone()
    from fleetx_amd.models.language_model.gpt.model import GPTPretrainingCriterion
    loss = GPTPretrainingCriterion(model.cfg)(logits, labels, torch.ones(B, S, device="cuda"))
    loss.backward()
    logits = logits_val
    ref_logits, ref_loss = _gpt_reference(P, ids, pos, labels, heads, L)
    ref_loss.backward()
    assert logits.dtype == torch.bfloat16
    assert _rel(logits, ref_logits) < 2e-2, (_rel(logits, ref_logits), float(logits.abs().max()),
                                             float(ref_logits.abs().max()))
    assert abs(float(loss) - float(ref_loss)) < 5e-3 * float(ref_loss), (float(loss), float(ref_loss))
    _check_grads(model, P)


def _mha(q, k, v, scale, key_bias=None):
    att = (q @ k.transpose(-1, -2)) * scale
    if key_bias is not None:
        att = att + key_bias[:, None, None, :]
    return att.softmax(-1) @ v


def _ernie_reference(P, ids, tt, heads, L, pad_id=0, eps=1e-12):
    """Plain fp32 post-LN ERNIE/BERT encoder + pooler."""
    b, s = ids.shape
    Hd = P["embeddings.word_embeddings.weight"].shape[1]
    D = Hd // heads
    pos = torch.arange(s, device=ids.device)
    x = (P["embeddings.word_embeddings.weight"][ids] + P["embeddings.position_embeddings"][pos]
         + P["embeddings.token_type_embeddings"][tt])
    x = F.layer_norm(x, (Hd,), P["embeddings.layer_norm.weight"], P["embeddings.layer_norm.bias"], eps)
    kb = (ids == pad_id).float() * -1e4
    for i in range(L):
        pre = "encoder.%d." % i
        qkv = (x @ P[pre + "qkv.weight"].t() + P[pre + "qkv.bias"]).view(b, s, heads, 3, D)
        q, k, v = (qkv[:, :, :, j].transpose(1, 2) for j in range(3))
        o = _mha(q, k, v, D ** -0.5, kb).transpose(1, 2).reshape(b, s, Hd)
        h = F.layer_norm(x + o @ P[pre + "out_proj.weight"].t() + P[pre + "out_proj.bias"], (Hd,),
                         P[pre + "norm1.weight"], P[pre + "norm1.bias"], eps)
        y = F.gelu(h @ P[pre + "linear1.weight"].t() + P[pre + "linear1.bias"])
        x = F.layer_norm(h + y @ P[pre + "linear2.weight"].t() + P[pre + "linear2.bias"], (Hd,),
                         P[pre + "norm2.weight"], P[pre + "norm2.bias"], eps)
    pooled = torch.tanh(x[:, 0] @ P["pooler.dense.weight"].t() + P["pooler.dense.bias"])
    return x, pooled


def _vit_reference(P, img, heads, L, patch, eps=1e-6):
    """Plain fp32 pre-LN ViT (conv-as-GEMM patch embed, class token, exact GeLU)."""
    B, C, H, W = img.shape
    p = patch
    x = img.reshape(B, C, H // p, p, W // p, p).permute(0, 2, 4, 1, 3, 5)
    x = x.reshape(B, (H // p) * (W // p), C * p * p)
    x = x @ P["patch_embed.proj.weight"].t() + P["patch_embed.proj.bias"]
    x = torch.cat([P["cls_token"].expand(B, -1, -1), x], 1) + P["pos_embed"]
    Hd = x.shape[-1]
    D = Hd // heads
    N = x.shape[1]
    for i in range(L):
        pre = "blocks.%d." % i
        h = F.layer_norm(x, (Hd,), P[pre + "norm1.weight"], P[pre + "norm1.bias"], eps)
        qkv = (h @ P[pre + "attn.qkv.weight"].t() + P[pre + "attn.qkv.bias"]).view(B, N, 3, heads, D)
        q, k, v = (qkv[:, :, j].transpose(1, 2) for j in range(3))
        o = _mha(q, k, v, D ** -0.5).transpose(1, 2).reshape(B, N, Hd)
        x = x + o @ P[pre + "attn.proj.weight"].t() + P[pre + "attn.proj.bias"]
        h = F.layer_norm(x, (Hd,), P[pre + "norm2.weight"], P[pre + "norm2.bias"], eps)
        a = F.gelu(h @ P[pre + "mlp.fc1.weight"].t() + P[pre + "mlp.fc1.bias"])
        x = x + a @ P[pre + "mlp.fc2.weight"].t() + P[pre + "mlp.fc2.bias"]
    x = F.layer_norm(x, (Hd,), P["norm.weight"], P["norm.bias"], eps)[:, 0]
    return x @ P["head.weight"].t() + P["head.bias"]


def _perturb(model):
    with torch.no_grad():
        for n, p in model.named_parameters():
            if p.ndim == 1 or "head" in n or "cls_token" in n:
                p.add_(0.05 * torch.randn_like(p))


def _check_grads(model, P, tol=5e-2, l2tol=2e-2):
    """Every parameter gradient: max-relative error (``tol``) AND the
    normwise relative error of each row block (``l2tol``)."""
    bad = {}
    for n, p in model.named_parameters():
        g = p.grad if p.grad is not None else getattr(p, "main_grad", None)
        assert g is not None, n
        r = _rel(g, P[n].grad)
        r2 = _rel_l2_blocks(g, P[n].grad)
        if r > tol or r2 > l2tol:
            bad[n] = (round(r, 4), round(r2, 4))
    assert not bad, bad


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_ernie_hip_vs_fp32_torch(dtype):
    from fleetx_amd.models.language_model.ernie.model import ErnieModel
    from fleetx_amd.parallel import topology as topo
    topo.reset_hcg()
    torch.manual_seed(1)
    heads, L, V, S, B = 8, 2, 2048, 192, 4
    model = ErnieModel(vocab_size=V, hidden_size=512, num_hidden_layers=L, num_attention_heads=heads,
                       intermediate_size=2048, hidden_dropout_prob=0.0,
                       attention_probs_dropout_prob=0.0).cuda().to(dtype)
    _perturb(model)
    ids = torch.randint(1, V, (B, S), device="cuda")
    ids[1, 150:] = 0                       # padded tail -> key-bias mask
    tt = torch.randint(0, 2, (B, S), device="cuda")
    seq, pooled = model(ids, tt)
    R1 = torch.randn(seq.shape, device="cuda")
    R2 = torch.randn(pooled.shape, device="cuda")
    ((seq.float() * R1).sum() + (pooled.float() * R2).sum()).backward()
    P = {n: p.detach().float().clone().requires_grad_(True) for n, p in model.named_parameters()}
    rs, rp = _ernie_reference(P, ids, tt, heads, L)
    ((rs * R1).sum() + (rp * R2).sum()).backward()
    assert _rel(seq, rs) < 3e-2, _rel(seq, rs)
    assert _rel(pooled, rp) < 3e-2, _rel(pooled, rp)
    _check_grads(model, P)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_vit_hip_vs_fp32_torch(dtype):
    from fleetx_amd.models.vision_model.vit import ViT
    torch.manual_seed(2)
    heads, L, patch = 4, 2, 16
    model = ViT(img_size=128, patch_size=patch, class_num=100, embed_dim=256, depth=L,
                num_heads=heads, qkv_bias=True, epsilon=1e-6).cuda().to(dtype)
    _perturb(model)
    img = torch.randn(8, 3, 128, 128, device="cuda")
    labels = torch.randint(0, 100, (8,), device="cuda")
    logits = model(img.to(dtype))
    F.cross_entropy(logits.float(), labels).backward()
    P = {n: p.detach().float().clone().requires_grad_(True) for n, p in model.named_parameters()}
    ref = _vit_reference(P, img.to(dtype).float(), heads, L, patch)
    F.cross_entropy(ref, labels).backward()
    assert _rel(logits, ref) < 3e-2, _rel(logits, ref)
    _check_grads(model, P)

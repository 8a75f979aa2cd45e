"""Vision Transformer (ViT) with the reference presets B/16 ... 6B/14.

Parity: reference ``models/vision_model/vit/vit.py:49-431`` and
``layers/{attention,mlp,embedding,droppath,initializer}.py`` (C34, K20):
patch embed (conv with kernel = stride = patch) -> cls token + learned
position embedding -> depth x pre-LN blocks (attention + exact-GeLU MLP, with
DropPath) -> LN -> ``x[:, 0]`` -> optional tanh representation layer ->
classifier.  Init: xavier for linears, zeros for the head, -10 head bias with
a representation layer, truncated-normal position embedding.
``load_pretrained`` casts to fp32 and bicubic-interpolates the position
embedding for fine-tuning at another resolution.

MI355X mapping: the patch embed is an unfold + GEMM (no conv), attention uses
the fused non-causal flash kernel through the packed [B, N, 3, H, D] QKV entry
(ViT-g's head dim 88 runs on the 96-wide tile with zero-read columns), LN and
bias+GeLU(erf) are HIP kernels.
"""
import math
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ... import ops
from ...parallel.linear import fused_mlp, linear


def _xavier(lin):
    nn.init.xavier_uniform_(lin.weight)
    if lin.bias is not None:
        nn.init.zeros_(lin.bias)
    return lin


def _apply(mod, x, bias=True):
    """A linear layer: the fused-gradient GEMM for a plain ``nn.Linear``, the
    module itself otherwise (e.g. a QAT-wrapped layer, utils/qat.py)."""
    if type(mod) is nn.Linear:
        return linear(x, mod.weight, mod.bias if bias else None)
    return mod(x)


def _fused_grads(lin):
    """Let the linear's weight / bias gradients go straight into the flat fp32
    ``main_grad`` buffer (parallel/linear.py, ops/norm.py)."""
    lin.weight._fx_fused_wgrad_ok = True
    # its gradient comes from the wgrad GEMM: the epilogue's sums of squares
    # feed the global gradient norm (grad_buffer.enable_fused_norm)
    lin.weight._fx_gemm_wgrad = True
    if lin.bias is not None:
        lin.bias._fx_fused_wgrad_ok = True
    return lin


class DropPath(nn.Module):
    """Stochastic depth per sample (reference ``layers/droppath.py:19-47``)."""

    def __init__(self, p=0.0):
        super().__init__()
        self.p = p

    def forward(self, x):
        if self.p == 0.0 or not self.training:
            return x
        keep = 1.0 - self.p
        mask = torch.empty((x.shape[0],) + (1,) * (x.ndim - 1), device=x.device,
                           dtype=x.dtype).bernoulli_(keep)
        return x * mask / keep


class PatchEmbed(nn.Module):
    """Conv(kernel = stride = patch) as unfold + one GEMM."""

    def __init__(self, img_size=224, patch_size=16, in_chans=3, embed_dim=768):
        super().__init__()
        self.img_size, self.patch_size = img_size, patch_size
        self.num_patches = (img_size // patch_size) ** 2
        self.proj = nn.Linear(in_chans * patch_size * patch_size, embed_dim)
        nn.init.xavier_uniform_(self.proj.weight)
        nn.init.zeros_(self.proj.bias)

    def forward(self, x):
        B, C, H, W = x.shape
        p = self.patch_size
        assert H % p == 0 and W % p == 0, "image size must be a multiple of the patch size"
        x = x.reshape(B, C, H // p, p, W // p, p).permute(0, 2, 4, 1, 3, 5)
        x = x.reshape(B, (H // p) * (W // p), C * p * p)
        return self.proj(x)


class Attention(nn.Module):
    def __init__(self, dim, num_heads=8, qkv_bias=False, qk_scale=None, attn_drop=0.0,
                 proj_drop=0.0):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.scale = qk_scale or self.head_dim ** -0.5
        self.qkv = _fused_grads(_xavier(nn.Linear(dim, dim * 3, bias=qkv_bias)))
        self.proj = _fused_grads(_xavier(nn.Linear(dim, dim)))
        self.attn_drop = attn_drop
        self.proj_drop = nn.Dropout(proj_drop)

    def _core(self, x):
        B, N, C = x.shape
        qkv = _apply(self.qkv, x).view(B, N, 3, self.num_heads, self.head_dim)
        p = self.attn_drop if self.training else 0.0
        key = int(torch.randint(0, 2 ** 62, (1,)).item()) if p > 0 else 0
        # packed entry: dq / dk / dv written into one [B, N, 3, H, D] gradient
        o = ops.flash_attention_qkvpacked(qkv, causal=False, dropout_p=p, key=key,
                                          scale=self.scale, pack_dim=2)
        return o.reshape(B, N, C)

    def forward_nobias(self, x):
        """(proj(o) without its bias, bias): the bias joins the fused residual
        + LayerNorm kernel of the block."""
        return linear(self._core(x), self.proj.weight), self.proj.bias

    def forward(self, x):
        return self.proj_drop(_apply(self.proj, self._core(x)))


class Mlp(nn.Module):
    def __init__(self, dim, hidden, drop=0.0):
        super().__init__()
        self.fc1 = _fused_grads(_xavier(nn.Linear(dim, hidden)))
        self.fc2 = _fused_grads(_xavier(nn.Linear(hidden, dim)))
        self.drop = nn.Dropout(drop)

    def forward(self, x):
        if type(self.fc1) is not nn.Linear:
            return self.drop(self.fc2(self.drop(F.gelu(self.fc1(x)))))
        h = ops.bias_gelu(linear(x, self.fc1.weight), self.fc1.bias, approximate=False)
        return self.drop(_apply(self.fc2, self.drop(h)))


class Block(nn.Module):
    def __init__(self, dim, num_heads, mlp_ratio=4.0, qkv_bias=False, qk_scale=None, drop=0.0,
                 attn_drop=0.0, drop_path=0.0, epsilon=1e-5):
        super().__init__()
        self.norm1 = ops.FusedLayerNorm(dim, epsilon)
        self.attn = Attention(dim, num_heads, qkv_bias, qk_scale, attn_drop, drop)
        self.drop_path = DropPath(drop_path)
        self.norm2 = ops.FusedLayerNorm(dim, epsilon)
        self.mlp = Mlp(dim, int(dim * mlp_ratio), drop)

    def _fusable(self):
        plain = all(type(m) is nn.Linear for m in (self.attn.qkv, self.attn.proj, self.mlp.fc1,
                                                    self.mlp.fc2))
        return plain and (self.drop_path.p == 0.0 or not self.training) and \
            (self.attn.proj_drop.p == 0.0 and self.mlp.drop.p == 0.0 or not self.training)

    def forward(self, x):
        if self._fusable():
            # residual + proj bias + LN2 in one kernel, FFN1+GeLU(erf)+FFN2 as one
            # autograd node, residual + FFN2 bias in one kernel; every weight and
            # bias gradient lands in fp32 main_grad (same blocks as the GPT layer)
            # x comes back as the residual alias: its two branch gradients meet
            # inside the LN1 backward kernel (no separate add pass)
            x, h1 = ops.layer_norm_keep_input(x, self.norm1.weight, self.norm1.bias,
                                              self.norm1.eps)
            a, ab = self.attn.forward_nobias(h1)
            x2, h2 = ops.add_layer_norm(a, ab, x, self.norm2.weight, self.norm2.bias,
                                        self.norm2.eps)
            m = fused_mlp(h2, self.mlp.fc1.weight, self.mlp.fc1.bias, self.mlp.fc2.weight,
                          act="gelu_erf")
            return ops.bias_dropout_add(m, self.mlp.fc2.bias, x2)
        x = x + self.drop_path(self.attn(self.norm1(x)))
        return x + self.drop_path(self.mlp(self.norm2(x)))


class ViT(nn.Module):
    def __init__(self, img_size=224, patch_size=16, in_chans=3, class_num=1000, embed_dim=768,
                 depth=12, num_heads=12, mlp_ratio=4, qkv_bias=False, qk_scale=None, drop_rate=0.0,
                 attn_drop_rate=0.0, drop_path_rate=0.0, epsilon=1e-5, representation_size=None,
                 use_recompute=False, pretrained=None, **kwargs):
        super().__init__()
        self.class_num = class_num
        self.representation_size = representation_size
        self.num_features = self.embed_dim = embed_dim
        self.use_recompute = use_recompute
        self.patch_embed = PatchEmbed(img_size, patch_size, in_chans, embed_dim)
        n = self.patch_embed.num_patches
        self.pos_embed = nn.Parameter(torch.zeros(1, n + 1, embed_dim))
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.pos_drop = nn.Dropout(drop_rate)
        dpr = np.linspace(0, drop_path_rate, depth)
        self.blocks = nn.ModuleList([
            Block(embed_dim, num_heads, mlp_ratio, qkv_bias, qk_scale, drop_rate, attn_drop_rate,
                  float(dpr[i]), epsilon) for i in range(depth)])
        self.norm = ops.FusedLayerNorm(embed_dim, epsilon)
        if representation_size is not None:
            self.head0 = _xavier(nn.Linear(embed_dim, representation_size))
            self.head = nn.Linear(representation_size, class_num) if class_num > 0 else nn.Identity()
            if class_num > 0:
                nn.init.xavier_uniform_(self.head.weight)
                nn.init.constant_(self.head.bias, -10.0)
        else:
            self.head = nn.Linear(embed_dim, class_num) if class_num > 0 else nn.Identity()
            if class_num > 0:
                nn.init.zeros_(self.head.weight)
                nn.init.zeros_(self.head.bias)
        nn.init.trunc_normal_(self.pos_embed, std=0.02)
        if pretrained is not None:
            self.load_pretrained(**pretrained)

    def forward_features(self, x):
        B = x.shape[0]
        x = self.patch_embed(x.to(self.pos_embed.dtype))
        x = torch.cat([self.cls_token.expand(B, -1, -1), x], 1) + self.pos_embed
        x = self.pos_drop(x)
        for blk in self.blocks:
            if self.use_recompute and self.training:
                from ...parallel.recompute import recompute
                x = recompute(blk, x)
            else:
                x = blk(x)
        return self.norm(x)[:, 0]

    def forward(self, x):
        x = self.forward_features(x)
        if self.representation_size is not None:
            x = torch.tanh(self.head0(x))
        return self.head(x)

    def load_pretrained(self, prefix_path, finetune=False):
        path = prefix_path + ".pdparams" if not prefix_path.endswith(".pdparams") else prefix_path
        if not os.path.exists(path):
            raise ValueError("Model pretrain path {} does not exist.".format(path))
        sd = torch.load(path, map_location="cpu", weights_only=True)
        sd = {k: v.float() for k, v in sd.items()}
        if finetune:
            for k in [k for k in sd if k.startswith("head")]:
                sd.pop(k)
            pe = sd.get("pos_embed")
            if pe is not None and pe.shape != self.pos_embed.shape:
                cls, grid = pe[:, :1], pe[:, 1:]
                old = int(math.sqrt(grid.shape[1]))
                new = int(math.sqrt(self.pos_embed.shape[1] - 1))
                grid = grid.reshape(1, old, old, -1).permute(0, 3, 1, 2)
                grid = F.interpolate(grid, size=(new, new), mode="bicubic", align_corners=False)
                grid = grid.permute(0, 2, 3, 1).reshape(1, new * new, -1)
                sd["pos_embed"] = torch.cat([cls, grid], 1)
        self.load_state_dict(sd, strict=False)


_QKV = dict(qkv_bias=True, epsilon=1e-6)
PRESETS = {
    "ViT_base_patch16_224": dict(
        img_size=224, patch_size=16, embed_dim=768, depth=12, num_heads=12, mlp_ratio=4, **_QKV),
    "ViT_base_patch16_384": dict(
        img_size=384, patch_size=16, embed_dim=768, depth=12, num_heads=12, mlp_ratio=4, **_QKV),
    "ViT_base_patch32_224": dict(
        img_size=224, patch_size=32, embed_dim=768, depth=12, num_heads=12, mlp_ratio=4, **_QKV),
    "ViT_base_patch32_384": dict(
        img_size=384, patch_size=32, embed_dim=768, depth=12, num_heads=12, mlp_ratio=4, **_QKV),
    "ViT_large_patch16_224": dict(
        img_size=224, patch_size=16, embed_dim=1024, depth=24, num_heads=16, mlp_ratio=4, **_QKV),
    "ViT_large_patch16_384": dict(
        img_size=384, patch_size=16, embed_dim=1024, depth=24, num_heads=16, mlp_ratio=4, **_QKV),
    "ViT_large_patch32_224": dict(
        img_size=224, patch_size=32, embed_dim=1024, depth=24, num_heads=16, mlp_ratio=4, **_QKV),
    "ViT_large_patch32_384": dict(
        img_size=384, patch_size=32, embed_dim=1024, depth=24, num_heads=16, mlp_ratio=4, **_QKV),
    "ViT_huge_patch14_224": dict(
        img_size=224, patch_size=14, embed_dim=1280, depth=32, num_heads=16, mlp_ratio=4, representation_size=None),
    "ViT_huge_patch14_384": dict(
        img_size=384, patch_size=14, embed_dim=1280, depth=32, num_heads=16, mlp_ratio=4, representation_size=None),
    "ViT_g_patch14_224": dict(
        img_size=224, patch_size=14, embed_dim=1408, depth=40, num_heads=16, mlp_ratio=4.364,
        representation_size=1408, **_QKV),
    "ViT_G_patch14_224": dict(
        img_size=224, patch_size=14, embed_dim=1664, depth=48, num_heads=16, mlp_ratio=4.9231,
        representation_size=1664, **_QKV),
    "ViT_6B_patch14_224": dict(
        img_size=224, patch_size=14, embed_dim=2320, depth=80, num_heads=16, mlp_ratio=4.955,
        representation_size=2320, **_QKV),
}


def build_vit(name, **kwargs):
    if name not in PRESETS:
        raise ValueError("unknown ViT preset {}".format(name))
    cfg = dict(PRESETS[name])
    cfg.update(kwargs)
    return ViT(**cfg)

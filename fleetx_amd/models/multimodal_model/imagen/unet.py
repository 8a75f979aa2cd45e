"""Imagen efficient U-Net.

Parity: reference ``models/multimodal_model/imagen/unet.py:1-1485`` (C35, K21):
ResnetBlocks (GroupNorm -> FiLM(time) -> SiLU -> conv, optional cross-attention
to the conditioning tokens, global-context gating), CrossEmbedLayer stems,
multi-query self-attention with a learned null key/value (and optional
context keys), cross-attention, linear attention, PerceiverResampler text
pooling, learned-sinusoidal time conditioning with time tokens, pixel-shuffle
upsampling, scaled skip connections, memory-efficient (pre-downsample) layout,
classifier-free guidance (``forward_with_cond_scale``) and
``persist_to_file`` / ``hydrate_from_file``.

MI355X mapping:
* every ``Block`` is ``conv3x3(group_norm_silu(x, FiLM))`` — one fused
  two-pass HIP kernel for GroupNorm + scale/shift + SiLU (fwd and bwd) in
  front of a MIOpen convolution;
* all softmax attention (self, multi-query with broadcast K/V, cross, perceiver)
  runs on the non-causal flash kernel; padding masks become its additive key
  bias; the K/V broadcast of multi-query attention is a stride-0 view, so no
  copy is made and autograd sums the per-head K/V gradients;
* token LayerNorms are the HIP LayerNorm kernel.
"""
import copy
import math
from pathlib import Path

import torch
import torch.nn as nn
import torch.nn.functional as F

from .... import ops
from ....parallel.recompute import recompute
from .diffusion import cast_tuple, default, exists, resize_image_to

NEG = -1e9  # additive key bias for masked keys (exp underflows to exactly 0)


def _eps(x):
    return 1e-5 if x.dtype == torch.float32 else 1e-3


class LayerNorm(nn.Module):
    """Last-dim LayerNorm with a gain only (reference ``unet.py:32-47``)."""

    def __init__(self, dim, stable=False):
        super().__init__()
        self.stable = stable
        self.g = nn.Parameter(torch.ones(dim))
        self.register_buffer("zero_bias", torch.zeros(dim), persistent=False)

    def forward(self, x):
        if self.stable:
            x = x / x.amax(dim=-1, keepdim=True).detach()
        return ops.layer_norm(x, self.g, self.zero_bias.to(x.dtype), _eps(x))


class ChanLayerNorm(nn.Module):
    """LayerNorm over the channel dim of NCHW (reference ``unet.py:50-63``)."""

    def __init__(self, dim, stable=False):
        super().__init__()
        self.stable = stable
        self.g = nn.Parameter(torch.ones(1, dim, 1, 1))

    def forward(self, x):
        if self.stable:
            x = x / x.amax(dim=1, keepdim=True).detach()
        xf = x.float()
        var, mean = torch.var_mean(xf, dim=1, unbiased=False, keepdim=True)
        return ((xf - mean) * torch.rsqrt(var + _eps(x)) * self.g.float()).to(x.dtype)


def l2norm(t):
    return F.normalize(t, dim=-1)


def _flash(q, k, v, scale, key_bias=None):
    """q [B,Nq,H,D], k/v [B,Nk,H,D] (views allowed) -> [B,Nq,H*D]."""
    B, Nq, H, D = q.shape
    if key_bias is not None:
        key_bias = key_bias.float()
    o = ops.flash_attention(q, k, v, causal=False, scale=scale, key_bias=key_bias)
    return o.reshape(B, Nq, H * D)


def _mask_bias(mask, pad_front=0, pad_back=0):
    """bool keep-mask [B, N] -> additive bias [B, pad_front + N + pad_back]."""
    bias = torch.where(mask.bool(), 0.0, NEG).float()
    return F.pad(bias, (pad_front, pad_back), value=0.0)


class GlobalContext(nn.Module):
    """Attention-pooled squeeze-excitation (reference ``unet.py:66-86``)."""

    def __init__(self, *, dim_in, dim_out):
        super().__init__()
        self.to_k = nn.Conv2d(dim_in, 1, 1)
        hidden = max(3, dim_out // 2)
        self.net = nn.Sequential(nn.Conv2d(dim_in, hidden, 1), nn.SiLU(),
                                 nn.Conv2d(hidden, dim_out, 1), nn.Sigmoid())

    def forward(self, x):
        ctx = self.to_k(x).flatten(2)  # [b,1,n]
        xs = x.flatten(2)  # [b,c,n]
        out = torch.einsum("bin,bcn->bci", F.softmax(ctx.float(), -1).to(x.dtype), xs)
        return self.net(out[..., None])


class FeedForward(nn.Sequential):
    def __init__(self, dim, mult=2):
        hidden = int(dim * mult)
        super().__init__(LayerNorm(dim), nn.Linear(dim, hidden, bias=False), nn.GELU(),
                         LayerNorm(hidden), nn.Linear(hidden, dim, bias=False))


class ChanFeedForward(nn.Sequential):
    def __init__(self, dim, mult=2):
        hidden = int(dim * mult)
        super().__init__(ChanLayerNorm(dim), nn.Conv2d(dim, hidden, 1, bias=False), nn.GELU(),
                         ChanLayerNorm(hidden), nn.Conv2d(hidden, dim, 1, bias=False))


class PerceiverAttention(nn.Module):
    def __init__(self, *, dim, dim_head=64, heads=8, cosine_sim_attn=False):
        super().__init__()
        self.scale = dim_head ** -0.5 if not cosine_sim_attn else 16.0
        self.cosine_sim_attn = cosine_sim_attn
        self.heads, self.dim_head = heads, dim_head
        inner = dim_head * heads
        self.norm = nn.LayerNorm(dim)
        self.norm_latents = nn.LayerNorm(dim)
        self.to_q = nn.Linear(dim, inner, bias=False)
        self.to_kv = nn.Linear(dim, inner * 2, bias=False)
        self.to_out = nn.Sequential(nn.Linear(inner, dim, bias=False), nn.LayerNorm(dim))

    def forward(self, x, latents, mask=None):
        x = self.norm(x)
        latents = self.norm_latents(latents)
        b, h, d = x.shape[0], self.heads, self.dim_head
        q = self.to_q(latents).view(b, -1, h, d)
        kv = self.to_kv(torch.cat((x, latents), dim=-2))
        k, v = kv.view(b, kv.shape[1], 2, h, d).unbind(2)
        if self.cosine_sim_attn:
            q, k = l2norm(q), l2norm(k)
        kb = _mask_bias(mask, 0, latents.shape[-2]) if exists(mask) else None
        return self.to_out(_flash(q, k, v, self.scale, kb))


class PerceiverResampler(nn.Module):
    def __init__(self, *, dim, depth, dim_head=64, heads=8, num_latents=64,
                 num_latents_mean_pooled=4, max_seq_len=512, ff_mult=4, cosine_sim_attn=False):
        super().__init__()
        self.pos_emb = nn.Embedding(max_seq_len, dim)
        self.latents = nn.Parameter(torch.randn(num_latents, dim))
        self.to_latents_from_mean_pooled_seq = None
        self.num_latents_mean_pooled = num_latents_mean_pooled
        if num_latents_mean_pooled > 0:
            self.to_latents_from_mean_pooled_seq = nn.Sequential(
                LayerNorm(dim), nn.Linear(dim, dim * num_latents_mean_pooled))
        self.layers = nn.ModuleList([
            nn.ModuleList([PerceiverAttention(dim=dim, dim_head=dim_head, heads=heads,
                                              cosine_sim_attn=cosine_sim_attn),
                           FeedForward(dim, ff_mult)]) for _ in range(depth)])

    def forward(self, x, mask=None):
        n = x.shape[1]
        x_with_pos = x + self.pos_emb(torch.arange(n, device=x.device))
        latents = self.latents.unsqueeze(0).expand(x.shape[0], -1, -1)
        if exists(self.to_latents_from_mean_pooled_seq):
            pooled = self.to_latents_from_mean_pooled_seq(x.mean(dim=1))
            pooled = pooled.view(x.shape[0], self.num_latents_mean_pooled, -1)
            latents = torch.cat((pooled, latents), dim=-2)
        for attn, ff in self.layers:
            latents = attn(x_with_pos, latents, mask=mask) + latents
            latents = ff(latents) + latents
        return latents


class CrossAttention(nn.Module):
    def __init__(self, dim, *, context_dim=None, dim_head=64, heads=8, norm_context=False,
                 cosine_sim_attn=False):
        super().__init__()
        self.scale = dim_head ** -0.5 if not cosine_sim_attn else 16.0
        self.cosine_sim_attn = cosine_sim_attn
        self.heads, self.dim_head = heads, dim_head
        inner = dim_head * heads
        context_dim = default(context_dim, dim)
        self.norm = LayerNorm(dim)
        self.norm_context = LayerNorm(context_dim) if norm_context else nn.Identity()
        self.null_kv = nn.Parameter(torch.randn(2, dim_head))
        self.to_q = nn.Linear(dim, inner, bias=False)
        self.to_kv = nn.Linear(context_dim, inner * 2, bias=False)
        self.to_out = nn.Sequential(nn.Linear(inner, dim, bias=False), LayerNorm(dim))

    def _qkv(self, x, context):
        b = x.shape[0]
        h, d = self.heads, self.dim_head
        x = self.norm(x)
        context = self.norm_context(context)
        q = self.to_q(x).view(b, -1, h, d)
        k, v = self.to_kv(context).view(b, context.shape[1], 2, h, d).unbind(2)
        nk, nv = (t.view(1, 1, 1, d).expand(b, 1, h, d).to(k.dtype) for t in self.null_kv.unbind(0))
        return q, torch.cat((nk, k), 1), torch.cat((nv, v), 1)

    def forward(self, x, context, mask=None):
        q, k, v = self._qkv(x, context)
        if self.cosine_sim_attn:
            q, k = l2norm(q), l2norm(k)
        kb = _mask_bias(mask, 1, 0) if exists(mask) else None
        return self.to_out(_flash(q, k, v, self.scale, kb))


class LinearCrossAttention(CrossAttention):
    """Softmax-kernel linear attention over the context (reference ``unet.py:288-327``)."""

    def forward(self, x, context, mask=None):
        q, k, v = self._qkv(x, context)
        b, _, h, d = q.shape
        q, k, v = (t.permute(0, 2, 1, 3).reshape(b * h, -1, d).float() for t in (q, k, v))
        if exists(mask):
            m = F.pad(mask.bool(), (1, 0), value=True)
            m = m.repeat_interleave(h, 0)[..., None]
            k = k.masked_fill(~m, NEG)
            v = v.masked_fill(~m, 0.0)
        q = F.softmax(q * self.scale, dim=-1)
        k = F.softmax(k, dim=-2)
        ctx = torch.einsum("bnd,bne->bde", k, v)
        out = torch.einsum("bnd,bde->bne", q, ctx)
        out = out.view(b, h, -1, d).permute(0, 2, 1, 3).reshape(b, -1, h * d).to(x.dtype)
        return self.to_out(out)


class Block(nn.Module):
    """GroupNorm -> FiLM -> SiLU -> conv3x3, the first three fused on the GPU."""

    def __init__(self, dim, dim_out, groups=8, norm=True):
        super().__init__()
        self.norm = norm
        self.groups = groups
        if norm:
            self.gn_weight = nn.Parameter(torch.ones(dim))
            self.gn_bias = nn.Parameter(torch.zeros(dim))
        self.project = nn.Conv2d(dim, dim_out, 3, padding=1)

    def forward(self, x, scale_shift=None):
        scale, shift = scale_shift if exists(scale_shift) else (None, None)
        if self.norm:
            x = ops.group_norm_silu(x, self.groups, self.gn_weight, self.gn_bias, scale, shift)
        else:
            if exists(scale):
                x = x * (scale[..., None, None] + 1) + shift[..., None, None]
            x = F.silu(x)
        return self.project(x)


class ToTokens(nn.Module):
    """Runs a token module on NCHW maps: b c h w -> b (h w) c -> back."""

    def __init__(self, fn):
        super().__init__()
        self.fn = fn

    def forward(self, x, **kw):
        b, c, hh, ww = x.shape
        t = x.flatten(2).transpose(1, 2)
        t = self.fn(t, **kw)
        return t.transpose(1, 2).reshape(b, c, hh, ww)


class ResnetBlock(nn.Module):
    def __init__(self, dim, dim_out, *, cond_dim=None, time_cond_dim=None, groups=8,
                 linear_attn=False, use_gca=False, squeeze_excite=False, **attn_kwargs):
        super().__init__()
        self.time_mlp = None
        if exists(time_cond_dim):
            self.time_mlp = nn.Sequential(nn.SiLU(), nn.Linear(time_cond_dim, dim_out * 2))
        self.cross_attn = None
        if exists(cond_dim):
            klass = CrossAttention if not linear_attn else LinearCrossAttention
            self.cross_attn = ToTokens(klass(dim=dim_out, context_dim=cond_dim, **attn_kwargs))
        self.block1 = Block(dim, dim_out, groups=groups)
        self.block2 = Block(dim_out, dim_out, groups=groups)
        self.gca = GlobalContext(dim_in=dim_out, dim_out=dim_out) if use_gca else None
        self.res_conv = nn.Conv2d(dim, dim_out, 1) if dim != dim_out else nn.Identity()

    def forward(self, x, time_emb=None, cond=None):
        scale_shift = None
        if exists(self.time_mlp) and exists(time_emb):
            scale_shift = self.time_mlp(time_emb).float().chunk(2, dim=1)
        h = self.block1(x)
        if exists(self.cross_attn):
            assert exists(cond)
            h = self.cross_attn(h, context=cond) + h
        h = self.block2(h, scale_shift=scale_shift)
        if exists(self.gca):
            h = h * self.gca(h)
        return h + self.res_conv(x)


class Attention(nn.Module):
    """Multi-query self-attention with null key/value and optional context keys."""

    def __init__(self, dim, *, dim_head=64, heads=8, context_dim=None, cosine_sim_attn=False):
        super().__init__()
        self.scale = dim_head ** -0.5 if not cosine_sim_attn else 16.0
        self.cosine_sim_attn = cosine_sim_attn
        self.heads, self.dim_head = heads, dim_head
        inner = dim_head * heads
        self.norm = LayerNorm(dim)
        self.null_kv = nn.Parameter(torch.randn(2, dim_head))
        self.to_q = nn.Linear(dim, inner, bias=False)
        self.to_kv = nn.Linear(dim, dim_head * 2, bias=False)
        self.to_context = nn.Sequential(nn.LayerNorm(context_dim), nn.Linear(context_dim, dim_head * 2)) \
            if exists(context_dim) else None
        self.to_out = nn.Sequential(nn.Linear(inner, dim, bias=False), LayerNorm(dim))

    def forward(self, x, context=None, mask=None):
        b, n = x.shape[:2]
        h, d = self.heads, self.dim_head
        x = self.norm(x)
        q = self.to_q(x).view(b, n, h, d)
        k, v = self.to_kv(x).chunk(2, dim=-1)
        nk, nv = (t.view(1, 1, d).expand(b, 1, d).to(k.dtype) for t in self.null_kv.unbind(0))
        k, v = torch.cat((nk, k), 1), torch.cat((nv, v), 1)
        if exists(context):
            ck, cv = self.to_context(context).chunk(2, dim=-1)
            k, v = torch.cat((ck.to(k.dtype), k), 1), torch.cat((cv.to(v.dtype), v), 1)
        if self.cosine_sim_attn:
            q, k = l2norm(q), l2norm(k)
        kb = None
        if exists(mask):
            kb = _mask_bias(mask, k.shape[1] - mask.shape[1], 0)
        # multi-query: one K/V head broadcast over the query heads (stride-0 view)
        k4 = k.unsqueeze(2).expand(b, k.shape[1], h, d)
        v4 = v.unsqueeze(2).expand(b, v.shape[1], h, d)
        return self.to_out(_flash(q, k4, v4, self.scale, kb))


class Residual(nn.Module):
    def __init__(self, fn):
        super().__init__()
        self.fn = fn

    def forward(self, x, **kw):
        return self.fn(x, **kw) + x


class TransformerBlock(nn.Module):
    def __init__(self, dim, *, depth=1, heads=8, dim_head=32, ff_mult=2, context_dim=None,
                 cosine_sim_attn=False):
        super().__init__()
        self.layers = nn.ModuleList([
            nn.ModuleList([ToTokens(Attention(dim=dim, heads=heads, dim_head=dim_head,
                                              context_dim=context_dim,
                                              cosine_sim_attn=cosine_sim_attn)),
                           ChanFeedForward(dim=dim, mult=ff_mult)]) for _ in range(depth)])

    def forward(self, x, context=None):
        for attn, ff in self.layers:
            x = attn(x, context=context) + x
            x = ff(x) + x
        return x


class LearnedSinusoidalPosEmb(nn.Module):
    def __init__(self, dim):
        super().__init__()
        assert dim % 2 == 0
        self.weights = nn.Parameter(torch.randn(dim // 2))

    def forward(self, x):
        x = x[:, None].float()
        freqs = x * self.weights[None, :].float() * 2 * math.pi
        out = torch.cat((x, freqs.sin(), freqs.cos()), dim=-1)
        return out.to(self.weights.dtype)


class LinearAttention(nn.Module):
    def __init__(self, dim, dim_head=32, heads=8, dropout=0.05, context_dim=None, **kwargs):
        super().__init__()
        self.scale = dim_head ** -0.5
        self.heads = heads
        inner = dim_head * heads
        self.norm = ChanLayerNorm(dim)
        self.nonlin = nn.SiLU()

        def proj():
            return nn.Sequential(nn.Dropout(dropout), nn.Conv2d(dim, inner, 1, bias=False),
                                 nn.Conv2d(inner, inner, 3, bias=False, padding=1, groups=inner))
        self.to_q, self.to_k, self.to_v = proj(), proj(), proj()
        self.to_context = nn.Sequential(nn.LayerNorm(context_dim),
                                        nn.Linear(context_dim, inner * 2, bias=False)) \
            if exists(context_dim) else None
        self.to_out = nn.Sequential(nn.Conv2d(inner, dim, 1, bias=False), ChanLayerNorm(dim))

    def forward(self, fmap, context=None):
        h = self.heads
        b, _, xx, yy = fmap.shape
        fmap = self.norm(fmap)
        q, k, v = (fn(fmap) for fn in (self.to_q, self.to_k, self.to_v))
        c = q.shape[1] // h
        q, k, v = (t.reshape(b * h, c, xx * yy).transpose(1, 2).float() for t in (q, k, v))
        if exists(context):
            ck, cv = self.to_context(context).chunk(2, dim=-1)
            ck, cv = (t.reshape(b, -1, h, c).permute(0, 2, 1, 3).reshape(b * h, -1, c).float()
                      for t in (ck, cv))
            k, v = torch.cat((k, ck), 1), torch.cat((v, cv), 1)
        q = F.softmax(q, dim=-1) * self.scale
        k = F.softmax(k, dim=-2)
        ctx = torch.einsum("bnd,bne->bde", k, v)
        out = torch.einsum("bnd,bde->bne", q, ctx)
        out = out.transpose(1, 2).reshape(b, h * c, xx, yy).to(fmap.dtype)
        return self.to_out(self.nonlin(out))


class LinearAttentionTransformerBlock(nn.Module):
    def __init__(self, dim, *, depth=1, heads=8, dim_head=32, ff_mult=2, context_dim=None,
                 **kwargs):
        super().__init__()
        self.layers = nn.ModuleList([
            nn.ModuleList([LinearAttention(dim=dim, heads=heads, dim_head=dim_head,
                                           context_dim=context_dim),
                           ChanFeedForward(dim=dim, mult=ff_mult)]) for _ in range(depth)])

    def forward(self, x, context=None):
        for attn, ff in self.layers:
            x = attn(x, context=context) + x
            x = ff(x) + x
        return x


class Identity(nn.Module):
    def forward(self, x, *args, **kwargs):
        return x


class CrossEmbedLayer(nn.Module):
    def __init__(self, dim_in, kernel_sizes, dim_out=None, stride=2):
        super().__init__()
        assert all(k % 2 == stride % 2 for k in kernel_sizes)
        dim_out = default(dim_out, dim_in)
        kernel_sizes = sorted(kernel_sizes)
        n = len(kernel_sizes)
        scales = [int(dim_out / (2 ** i)) for i in range(1, n)]
        scales = [*scales, dim_out - sum(scales)]
        self.convs = nn.ModuleList([nn.Conv2d(dim_in, s, k, stride=stride, padding=(k - stride) // 2)
                                    for k, s in zip(kernel_sizes, scales)])

    def forward(self, x):
        return torch.cat([c(x) for c in self.convs], dim=1)


class Parallel(nn.Module):
    def __init__(self, *fns):
        super().__init__()
        self.fns = nn.ModuleList(fns)

    def forward(self, x):
        return sum(fn(x) for fn in self.fns)


def Downsample(dim, dim_out=None):
    return nn.Conv2d(dim, default(dim_out, dim), 4, 2, 1)


def Upsample(dim, dim_out=None):
    return nn.Sequential(nn.Upsample(scale_factor=2, mode="nearest"),
                         nn.Conv2d(dim, default(dim_out, dim), 3, padding=1))


class PixelShuffleUpsample(nn.Module):
    def __init__(self, dim, dim_out=None):
        super().__init__()
        dim_out = default(dim_out, dim)
        conv = nn.Conv2d(dim, dim_out * 4, 1)
        self.net = nn.Sequential(conv, nn.SiLU(), nn.PixelShuffle(2))
        o, i, hh, ww = conv.weight.shape
        w = torch.empty(o // 4, i, hh, ww)
        nn.init.kaiming_uniform_(w)
        with torch.no_grad():
            conv.weight.copy_(w.repeat_interleave(4, 0))
            conv.bias.zero_()

    def forward(self, x):
        return self.net(x)


class UpsampleCombiner(nn.Module):
    def __init__(self, dim, *, enabled=False, dim_ins=tuple(), dim_outs=tuple()):
        super().__init__()
        dim_outs = cast_tuple(dim_outs, len(dim_ins))
        self.enabled = enabled
        if not enabled:
            self.dim_out = dim
            return
        self.fmap_convs = nn.ModuleList([Block(a, b) for a, b in zip(dim_ins, dim_outs)])
        self.dim_out = dim + (sum(dim_outs) if len(dim_outs) > 0 else 0)

    def forward(self, x, fmaps=None):
        fmaps = default(fmaps, tuple())
        if not self.enabled or len(fmaps) == 0 or len(self.fmap_convs) == 0:
            return x
        fmaps = [resize_image_to(f, x.shape[-1]) for f in fmaps]
        return torch.cat((x, *[c(f) for f, c in zip(fmaps, self.fmap_convs)]), dim=1)


def prob_mask_like(shape, prob, device):
    if prob == 1:
        return torch.ones(shape, dtype=torch.bool, device=device)
    if prob == 0:
        return torch.zeros(shape, dtype=torch.bool, device=device)
    return torch.rand(shape, device=device) < prob


class Unet(nn.Module):
    def __init__(self, *, dim, image_embed_dim=1024, text_embed_dim=1024, num_resnet_blocks=1,
                 cond_dim=None, num_image_tokens=4, num_time_tokens=2, learned_sinu_pos_emb_dim=16,
                 out_dim=None, dim_mults=(1, 2, 4, 8), cond_images_channels=0, channels=3,
                 channels_out=None, attn_dim_head=64, attn_heads=8, ff_mult=2., lowres_cond=False,
                 layer_attns=True, layer_attns_depth=1, layer_attns_add_text_cond=True,
                 attend_at_middle=True, layer_cross_attns=True, use_linear_attn=False,
                 use_linear_cross_attn=False, cond_on_text=True, max_text_len=256, init_dim=None,
                 resnet_groups=8, init_conv_kernel_size=7, init_cross_embed=True,
                 init_cross_embed_kernel_sizes=(3, 7, 15), cross_embed_downsample=False,
                 cross_embed_downsample_kernel_sizes=(2, 4), attn_pool_text=True,
                 attn_pool_num_latents=32, dropout=0., memory_efficient=False,
                 init_conv_to_final_conv_residual=False, use_global_context_attn=True,
                 scale_skip_connection=True, final_resnet_block=True, final_conv_kernel_size=3,
                 cosine_sim_attn=False, self_cond=False, combine_upsample_fmaps=False,
                 pixel_shuffle_upsample=True, use_recompute=False):
        super().__init__()
        assert attn_heads > 1, "you need more than 1 attention head"
        self._config = {k: v for k, v in locals().items() if k not in ("self", "__class__")}
        self.use_recompute = use_recompute
        self.channels = channels
        self.channels_out = default(channels_out, channels)
        init_channels = channels * (1 + int(lowres_cond) + int(self_cond)) + cond_images_channels
        init_dim = default(init_dim, dim)
        self.self_cond = self_cond
        self.has_cond_image = cond_images_channels > 0
        self.cond_images_channels = cond_images_channels
        self.init_conv = CrossEmbedLayer(init_channels, dim_out=init_dim,
                                         kernel_sizes=init_cross_embed_kernel_sizes, stride=1) \
            if init_cross_embed else nn.Conv2d(init_channels, init_dim, init_conv_kernel_size,
                                               padding=init_conv_kernel_size // 2)
        dims = [init_dim, *[dim * m for m in dim_mults]]
        in_out = list(zip(dims[:-1], dims[1:]))
        cond_dim = default(cond_dim, dim)
        time_cond_dim = dim * 4 * (2 if lowres_cond else 1)
        self.num_time_tokens = num_time_tokens
        self.cond_dim = cond_dim
        self.to_time_hiddens = nn.Sequential(LearnedSinusoidalPosEmb(learned_sinu_pos_emb_dim),
                                             nn.Linear(learned_sinu_pos_emb_dim + 1, time_cond_dim),
                                             nn.SiLU())
        self.to_time_cond = nn.Sequential(nn.Linear(time_cond_dim, time_cond_dim))
        self.to_time_tokens = nn.Linear(time_cond_dim, cond_dim * num_time_tokens)
        self.lowres_cond = lowres_cond
        if lowres_cond:
            self.to_lowres_time_hiddens = nn.Sequential(
                LearnedSinusoidalPosEmb(learned_sinu_pos_emb_dim),
                nn.Linear(learned_sinu_pos_emb_dim + 1, time_cond_dim), nn.SiLU())
            self.to_lowres_time_cond = nn.Sequential(nn.Linear(time_cond_dim, time_cond_dim))
            self.to_lowres_time_tokens = nn.Linear(time_cond_dim, cond_dim * num_time_tokens)
        self.norm_cond = nn.LayerNorm(cond_dim)
        self.text_to_cond = nn.Linear(text_embed_dim, cond_dim) if cond_on_text else None
        self.cond_on_text = cond_on_text
        self.attn_pool = PerceiverResampler(dim=cond_dim, depth=2, dim_head=attn_dim_head,
                                            heads=attn_heads, num_latents=attn_pool_num_latents,
                                            cosine_sim_attn=cosine_sim_attn) \
            if attn_pool_text else None
        self.max_text_len = max_text_len
        self.null_text_embed = nn.Parameter(torch.randn(1, max_text_len, cond_dim))
        self.null_text_hidden = nn.Parameter(torch.randn(1, time_cond_dim))
        self.to_text_non_attn_cond = nn.Sequential(
            nn.LayerNorm(cond_dim), nn.Linear(cond_dim, time_cond_dim), nn.SiLU(),
            nn.Linear(time_cond_dim, time_cond_dim)) if cond_on_text else None
        attn_kwargs = dict(heads=attn_heads, dim_head=attn_dim_head, cosine_sim_attn=cosine_sim_attn)
        L = len(in_out)
        num_resnet_blocks = cast_tuple(num_resnet_blocks, L)
        resnet_groups = cast_tuple(resnet_groups, L)
        layer_attns = cast_tuple(layer_attns, L)
        layer_attns_depth = cast_tuple(layer_attns_depth, L)
        layer_cross_attns = cast_tuple(layer_cross_attns, L)
        assert all(len(t) == L for t in (resnet_groups, layer_attns, layer_cross_attns))

        def resnet(*a, **k):
            return ResnetBlock(*a, **{**attn_kwargs, **k})

        def downsample(a, b):
            if cross_embed_downsample:
                return CrossEmbedLayer(a, cross_embed_downsample_kernel_sizes, dim_out=b)
            return Downsample(a, b)

        self.init_resnet_block = resnet(init_dim, init_dim, time_cond_dim=time_cond_dim,
                                        groups=resnet_groups[0],
                                        use_gca=use_global_context_attn) if memory_efficient else None
        self.skip_connect_scale = 1.0 if not scale_skip_connection else 2 ** -0.5
        self.downs = nn.ModuleList([])
        self.ups = nn.ModuleList([])
        skip_dims = []
        params = [num_resnet_blocks, resnet_groups, layer_attns, layer_attns_depth,
                  layer_cross_attns]

        def tblock(layer_attn):
            if layer_attn:
                return TransformerBlock
            return LinearAttentionTransformerBlock if use_linear_attn else None

        for ind, ((d_in, d_out), nblocks, groups, lattn, ldepth, lcross) in enumerate(
                zip(in_out, *params)):
            is_last = ind >= L - 1
            lin_cross = not lcross and use_linear_cross_attn
            lcond = cond_dim if lcross or lin_cross else None
            cur = d_in
            pre = None
            if memory_efficient:
                pre = downsample(d_in, d_out)
                cur = d_out
            skip_dims.append(cur)
            post = None
            if not memory_efficient:
                post = downsample(cur, d_out) if not is_last else Parallel(
                    nn.Conv2d(d_in, d_out, 3, padding=1), nn.Conv2d(d_in, d_out, 1))
            tb = tblock(lattn)
            self.downs.append(nn.ModuleList([
                pre if pre is not None else Identity(),
                resnet(cur, cur, cond_dim=lcond, linear_attn=lin_cross, time_cond_dim=time_cond_dim,
                       groups=groups),
                nn.ModuleList([ResnetBlock(cur, cur, time_cond_dim=time_cond_dim, groups=groups,
                                           use_gca=use_global_context_attn) for _ in range(nblocks)]),
                tb(dim=cur, depth=ldepth, ff_mult=ff_mult, context_dim=cond_dim, **attn_kwargs)
                if tb is not None else Identity(),
                post if post is not None else Identity()]))
        mid = dims[-1]
        self.mid_block1 = ResnetBlock(mid, mid, cond_dim=cond_dim, time_cond_dim=time_cond_dim,
                                      groups=resnet_groups[-1], **attn_kwargs)
        self.mid_attn = ToTokens(Residual(Attention(mid, **attn_kwargs))) if attend_at_middle else None
        self.mid_block2 = ResnetBlock(mid, mid, cond_dim=cond_dim, time_cond_dim=time_cond_dim,
                                      groups=resnet_groups[-1], **attn_kwargs)
        up_klass = Upsample if not pixel_shuffle_upsample else PixelShuffleUpsample
        up_fmap_dims = []
        for ind, ((d_in, d_out), nblocks, groups, lattn, ldepth, lcross) in enumerate(
                zip(reversed(in_out), *[list(reversed(p)) for p in params])):
            is_last = ind == L - 1
            lin_cross = not lcross and use_linear_cross_attn
            lcond = cond_dim if lcross or lin_cross else None
            skip = skip_dims.pop()
            tb = tblock(lattn)
            up_fmap_dims.append(d_out)
            self.ups.append(nn.ModuleList([
                resnet(d_out + skip, d_out, cond_dim=lcond, linear_attn=lin_cross,
                       time_cond_dim=time_cond_dim, groups=groups),
                nn.ModuleList([ResnetBlock(d_out + skip, d_out, time_cond_dim=time_cond_dim,
                                           groups=groups, use_gca=use_global_context_attn)
                               for _ in range(nblocks)]),
                tb(dim=d_out, depth=ldepth, ff_mult=ff_mult, context_dim=cond_dim, **attn_kwargs)
                if tb is not None else Identity(),
                up_klass(d_out, d_in) if (not is_last or memory_efficient) else Identity()]))
        self.upsample_combiner = UpsampleCombiner(dim=dim, enabled=combine_upsample_fmaps,
                                                  dim_ins=up_fmap_dims, dim_outs=dim)
        self.init_conv_to_final_conv_residual = init_conv_to_final_conv_residual
        final_dim = self.upsample_combiner.dim_out + (dim if init_conv_to_final_conv_residual else 0)
        self.final_res_block = ResnetBlock(final_dim, dim, time_cond_dim=time_cond_dim,
                                           groups=resnet_groups[0], use_gca=True) \
            if final_resnet_block else None
        fin = (dim if final_resnet_block else final_dim) + (channels if lowres_cond else 0)
        self.final_conv = nn.Conv2d(fin, self.channels_out, final_conv_kernel_size,
                                    padding=final_conv_kernel_size // 2)
        nn.init.zeros_(self.final_conv.weight)
        nn.init.zeros_(self.final_conv.bias)

    # ---------------------------------------------------------------- config io
    def cast_model_parameters(self, *, lowres_cond, text_embed_dim, channels, channels_out,
                              cond_on_text):
        c = self._config
        if (lowres_cond == c["lowres_cond"] and channels == c["channels"]
                and cond_on_text == c["cond_on_text"] and text_embed_dim == c["text_embed_dim"]
                and channels_out == self.channels_out):
            return self
        cfg = dict(c)
        cfg.update(lowres_cond=lowres_cond, text_embed_dim=text_embed_dim, channels=channels,
                   channels_out=channels_out, cond_on_text=cond_on_text)
        return Unet(**cfg)

    def to_config_and_state_dict(self):
        return dict(self._config), self.state_dict()

    @classmethod
    def from_config_and_state_dict(cls, config, state_dict):
        u = Unet(**config)
        u.load_state_dict(state_dict)
        return u

    def persist_to_file(self, path):
        path = Path(path)
        path.parent.mkdir(parents=True, exist_ok=True)
        cfg, sd = self.to_config_and_state_dict()
        torch.save({"config": cfg, "state_dict": sd}, str(path))

    @classmethod
    def hydrate_from_file(cls, path):
        pkg = torch.load(str(path), map_location="cpu", weights_only=True)
        assert "config" in pkg and "state_dict" in pkg
        return Unet.from_config_and_state_dict(pkg["config"], pkg["state_dict"])

    # ---------------------------------------------------------------- forward
    def forward_with_cond_scale(self, *args, cond_scale=1., **kwargs):
        logits = self.forward(*args, **kwargs)
        if cond_scale == 1:
            return logits
        null_logits = self.forward(*args, **{**kwargs, "cond_drop_prob": 1.})
        return null_logits + (logits - null_logits) * cond_scale

    def _run(self, block, *args):
        if self.use_recompute and self.training and torch.is_grad_enabled():
            return recompute(block, *args)
        return block(*args)

    def forward(self, x, time, *, lowres_cond_img=None, lowres_noise_times=None, text_embeds=None,
                text_mask=None, cond_images=None, cond_drop_prob=0.):
        dt = self.final_conv.weight.dtype
        x = x.to(dt)
        b, dev = x.shape[0], x.device
        assert not (self.lowres_cond and not exists(lowres_cond_img)), \
            "low resolution conditioning image must be present"
        assert not (self.lowres_cond and not exists(lowres_noise_times)), \
            "low resolution conditioning noise time must be present"
        if exists(lowres_cond_img):
            lowres_cond_img = lowres_cond_img.to(dt)
            x = torch.cat((x, lowres_cond_img), dim=1)
        assert not (self.has_cond_image ^ exists(cond_images))
        if exists(cond_images):
            assert cond_images.shape[1] == self.cond_images_channels
            x = torch.cat((resize_image_to(cond_images.to(dt), x.shape[-1]), x), dim=1)
        x = self.init_conv(x)
        init_res = x.clone() if self.init_conv_to_final_conv_residual else None

        time_hiddens = self.to_time_hiddens(time)
        time_tokens = self.to_time_tokens(time_hiddens).view(b, self.num_time_tokens, -1)
        t = self.to_time_cond(time_hiddens)
        if self.lowres_cond:
            lh = self.to_lowres_time_hiddens(lowres_noise_times)
            t = t + self.to_lowres_time_cond(lh)
            time_tokens = torch.cat(
                (time_tokens, self.to_lowres_time_tokens(lh).view(b, self.num_time_tokens, -1)), -2)

        text_tokens = None
        if exists(text_embeds) and self.cond_on_text:
            keep = prob_mask_like((b,), 1 - cond_drop_prob, dev)
            keep_embed = keep[:, None, None]
            text_tokens = self.text_to_cond(text_embeds.to(dt))[:, :self.max_text_len]
            if exists(text_mask):
                text_mask = text_mask[:, :self.max_text_len].bool()
            rem = self.max_text_len - text_tokens.shape[1]
            if rem > 0:
                text_tokens = F.pad(text_tokens, (0, 0, 0, rem))
            if exists(text_mask):
                if rem > 0:
                    text_mask = F.pad(text_mask, (0, rem), value=False)
                keep_embed = text_mask[:, :, None] & keep_embed
            text_tokens = torch.where(keep_embed, text_tokens, self.null_text_embed.to(dt))
            if exists(self.attn_pool):
                text_tokens = self.attn_pool(text_tokens)
            text_hiddens = self.to_text_non_attn_cond(text_tokens.mean(dim=-2))
            text_hiddens = torch.where(keep[:, None], text_hiddens, self.null_text_hidden.to(dt))
            t = t + text_hiddens
        c = time_tokens if text_tokens is None else torch.cat((time_tokens, text_tokens), dim=-2)
        c = self.norm_cond(c)

        if exists(self.init_resnet_block):
            x = self._run(self.init_resnet_block, x, t)
        hiddens = []
        for pre, init_block, blocks, attn_block, post in self.downs:
            x = pre(x)
            x = self._run(init_block, x, t, c)
            for blk in blocks:
                x = self._run(blk, x, t)
                hiddens.append(x)
            x = self._run(attn_block, x, c) if not isinstance(attn_block, Identity) else x
            hiddens.append(x)
            x = post(x)
        x = self._run(self.mid_block1, x, t, c)
        if exists(self.mid_attn):
            x = self.mid_attn(x)
        x = self._run(self.mid_block2, x, t, c)

        def skip(x):
            return torch.cat((x, hiddens.pop() * self.skip_connect_scale), dim=1)

        up_hiddens = []
        for init_block, blocks, attn_block, up in self.ups:
            x = skip(x)
            x = self._run(init_block, x, t, c)
            for blk in blocks:
                x = skip(x)
                x = self._run(blk, x, t)
            x = self._run(attn_block, x, c) if not isinstance(attn_block, Identity) else x
            up_hiddens.append(x)
            x = up(x)
        x = self.upsample_combiner(x, up_hiddens)
        if self.init_conv_to_final_conv_residual:
            x = torch.cat((x, init_res), dim=1)
        if exists(self.final_res_block):
            x = self._run(self.final_res_block, x, t)
        if exists(lowres_cond_img):
            x = torch.cat((x, lowres_cond_img), dim=1)
        return self.final_conv(x)


def _preset(defaults):
    def make(**kwargs):
        cfg = copy.deepcopy(defaults)
        cfg.update(kwargs)
        return Unet(**cfg)
    return make


Unet64_397M = _preset(dict(dim=256, dim_mults=(1, 2, 3, 4), num_resnet_blocks=3,
                           layer_attns=(False, True, True, True),
                           layer_cross_attns=(False, True, True, True), attn_heads=8, ff_mult=2.,
                           memory_efficient=False))
BaseUnet64 = _preset(dict(dim=512, dim_mults=(1, 2, 3, 4), num_resnet_blocks=3,
                          layer_attns=(False, True, True, True),
                          layer_cross_attns=(False, True, True, True), attn_heads=8, ff_mult=2.,
                          memory_efficient=False))
SRUnet256 = _preset(dict(dim=128, dim_mults=(1, 2, 4, 8), num_resnet_blocks=(2, 4, 8, 8),
                         layer_attns=(False, False, False, True),
                         layer_cross_attns=(False, False, False, True), attn_heads=8, ff_mult=2.,
                         memory_efficient=True))
SRUnet1024 = _preset(dict(dim=128, dim_mults=(1, 2, 4, 8), num_resnet_blocks=(2, 4, 8, 8),
                          layer_attns=False, layer_cross_attns=(False, False, False, True),
                          attn_heads=8, ff_mult=2., memory_efficient=True))

"""Fused multi-head attention (flash-style) on the HIP kernels.

Reference K03-K06 (``single_model.py:189-213``, ``hybrid_model.py:268-298``):
scaled QK^T, causal softmax (``softmax_mask_fuse_upper_triangle``),
attention-prob dropout under the ``local_seed`` stream, PV and head merge.

Layouts are passed as strides, so the packed QKV GEMM output
``[b, s, heads, 3, d]`` (per-head interleave, which is what a column-split
QKV weight produces under tensor parallelism) is consumed without a
transpose/split copy, and the backward writes ``dq/dk/dv`` straight into one
packed gradient buffer.  The sequence-parallel ``[s, b, ...]`` layout works
the same way (only strides differ).
"""
import math

import torch

from . import _lib
from ..parallel import rng as _rng


def _strides(t):
    # t: [B, S, H, D] view
    return [t.stride(0), t.stride(1), t.stride(2)]


def attention_reference(q, k, v, causal=True, dropout_p=0.0, key=0, scale=None, kv_lens=None,
                        key_bias=None):
    """PyTorch math for ``[B, S, H, D]`` inputs (CPU path and test oracle).

    ``key_bias``: optional additive ``[B, Sk]`` score bias (e.g. ``-1e4`` on
    padding keys, the BERT/ERNIE convention)."""
    B, Sq, H, D = q.shape
    Sk = k.shape[1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    qf = q.float().permute(0, 2, 1, 3)
    kf = k.float().permute(0, 2, 1, 3)
    vf = v.float().permute(0, 2, 1, 3)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if key_bias is not None:
        s = s + key_bias.float().view(B, 1, 1, Sk)
    mask = torch.zeros(Sq, Sk, dtype=torch.bool, device=q.device)
    if causal:
        mask = torch.triu(torch.ones(Sq, Sk, dtype=torch.bool, device=q.device), diagonal=1)
    mask = mask.view(1, 1, Sq, Sk).expand(B, H, Sq, Sk)
    if kv_lens is not None:
        kl = kv_lens.to(q.device).view(B, 1, 1, 1)
        mask = mask | (torch.arange(Sk, device=q.device).view(1, 1, 1, Sk) >= kl)
    s = s.masked_fill(mask, float("-inf"))
    p = torch.softmax(s, dim=-1)
    p = torch.nan_to_num(p, nan=0.0)
    if dropout_p > 0.0:
        keep = _rng.attention_keep_mask(B * H, Sq, Sk, dropout_p, key, q.device).view(B, H, Sq, Sk)
        p = torch.where(keep, p / (1.0 - dropout_p), torch.zeros_like(p))
    o = torch.matmul(p, vf).permute(0, 2, 1, 3)
    return o.to(q.dtype)


class _FlashAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, packed, causal, p, key, scale, kv_lens, key_bias=None):
        # packed: None or the [B,S,H,3,D] tensor q/k/v are views of
        B, Sq, H, D = q.shape
        Sk = k.shape[1]
        if not _native_dim(D):
            raise NotImplementedError("flash attention supports head_dim multiples of 8 up to 128 "
                                      "(got %d)" % D)
        for t in (q, k, v):
            if t.stride(-1) != 1:
                raise ValueError("head dim must be contiguous")
            if t.dtype != q.dtype:
                raise TypeError("flash attention: q/k/v dtypes differ ({}, {})".format(q.dtype, t.dtype))
        dt = _lib.dt_code(q.dtype)  # bf16 / fp16 kernels; anything else raises
        ctx.dt = dt
        k_ = _lib.kernels()
        out = torch.empty(B, Sq, H, D, device=q.device, dtype=q.dtype)
        lse = torch.empty(B * H * Sq, device=q.device, dtype=torch.float32)
        kl = kv_lens.to(torch.int32).contiguous() if kv_lens is not None else None
        kb = _padded_bias(key_bias, B, Sk, q.device)
        rc = k_.flash_fwd(dt, q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), lse.data_ptr(),
                          _strides(q), _strides(k), _strides(v), _strides(out), _lib.ptr(kl),
                          _lib.ptr(kb), kb.shape[1] if kb is not None else 0,
                          B, H, Sq, Sk, D, int(causal), float(scale), float(p), key,
                          _lib.stream())
        if rc != 0:
            raise RuntimeError("flash_fwd failed (%d)" % rc)
        _lib.maybe_sync()
        ctx.causal, ctx.p, ctx.key, ctx.scale = causal, p, key, scale
        ctx.packed = packed is not None
        ctx.save_for_backward(q, k, v, out, lse, kl, kb)
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse, kl, kb = ctx.saved_tensors
        B, Sq, H, D = q.shape
        Sk = k.shape[1]
        dout = dout.contiguous()
        if ctx.packed:
            pd = getattr(ctx, "pack_dim", 3)  # [B,S,H,3,D] (GPT) or [B,S,3,H,D] (ViT)
            shape = (B, Sq, H, 3, D) if pd == 3 else (B, Sq, 3, H, D)
            dqkv = torch.empty(shape, device=q.device, dtype=q.dtype)
            dq, dk, dv = dqkv.select(pd, 0), dqkv.select(pd, 1), dqkv.select(pd, 2)
        else:
            dq = torch.empty(B, Sq, H, D, device=q.device, dtype=q.dtype)
            dk = torch.empty(B, Sk, H, D, device=q.device, dtype=q.dtype)
            dv = torch.empty_like(dk)
        delta = torch.empty(B * H * Sq, device=q.device, dtype=torch.float32)
        rc = _lib.kernels().flash_bwd(
            ctx.dt, q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), dout.data_ptr(),
            lse.data_ptr(), delta.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(),
            _strides(q), _strides(k), _strides(v), _strides(out), _strides(dq), _strides(dk),
            _lib.ptr(kl), _lib.ptr(kb), kb.shape[1] if kb is not None else 0,
            B, H, Sq, Sk, D, int(ctx.causal), float(ctx.scale), float(ctx.p),
            ctx.key, _lib.stream())
        if rc != 0:
            raise RuntimeError("flash_bwd failed (%d)" % rc)
        _lib.maybe_sync()
        if ctx.packed:
            return None, None, None, dqkv, None, None, None, None, None, None
        return dq, dk, dv, None, None, None, None, None, None, None


class _PackedEntry(torch.autograd.Function):
    """Routes the packed-QKV gradient back to the packed tensor."""

    @staticmethod
    def forward(ctx, qkv, causal, p, key, scale, kv_lens, key_bias, pack_dim=3):
        ctx.pack_dim = pack_dim
        q, k, v = qkv.select(pack_dim, 0), qkv.select(pack_dim, 1), qkv.select(pack_dim, 2)
        return _FlashAttn.forward(ctx, q, k, v, qkv, causal, p, key, scale, kv_lens, key_bias)

    @staticmethod
    def backward(ctx, dout):
        grads = _FlashAttn.backward(ctx, dout)
        return grads[3], None, None, None, None, None, None, None


_WARNED = {}


def _padded_bias(key_bias, B, Sk, device):
    """fp32 ``[B, round_up(Sk, 128)]`` copy: the kernels read whole key groups."""
    if key_bias is None:
        return None
    width = (Sk + 127) // 128 * 128
    kb = torch.zeros(B, width, device=device, dtype=torch.float32)
    kb[:, :Sk] = key_bias.reshape(B, Sk)
    return kb


def _unfused_attention(q, k, v, causal, dropout_p, key, scale, kv_lens, key_bias):
    """Materialised-scores path (reference ``core_attn``, ``single_model.py:189-213``)
    for head dims the flash tiles do not cover: hipBLASLt QK^T / PV GEMMs in
    the model dtype around the fused HIP softmax (``ops/softmax.py``);
    padding keys / key bias enter as one additive ``[B, 1, 1|Sq, Sk]`` mask."""
    from .softmax import fused_softmax
    B, Sq, H, D = q.shape
    Sk = k.shape[1]
    qh, kh, vh = (t.permute(0, 2, 1, 3) for t in (q, k, v))
    s = torch.matmul(qh, kh.transpose(-1, -2))
    mask = None
    if key_bias is not None or kv_lens is not None:
        mask = torch.zeros(B, 1, 1, Sk, dtype=torch.float32, device=q.device)
        if key_bias is not None:
            mask = mask + key_bias.float().view(B, 1, 1, Sk)
        if kv_lens is not None:
            pad = torch.arange(Sk, device=q.device).view(1, 1, 1, Sk) >= \
                kv_lens.to(q.device).view(B, 1, 1, 1)
            mask = mask.masked_fill(pad, float("-inf"))
        mask = mask.expand(B, 1, Sq, Sk)
    p = fused_softmax(s, mask, causal, scale)
    if dropout_p > 0.0:
        keep = _rng.attention_keep_mask(B * H, Sq, Sk, dropout_p, key, q.device).view(B, H, Sq, Sk)
        p = torch.where(keep, p * (1.0 / (1.0 - dropout_p)), torch.zeros_like(p))
    return torch.matmul(p, vh).permute(0, 2, 1, 3)


# head dims with a kernel tile (csrc/kernels/flash_attn.hip: 32-wide output
# column blocks, 16-deep k-steps, 512-B LDS chunk groups)
FLASH_DIMS = (64, 96, 128)


def _padded_dim(d):
    """Smallest kernel tile width >= d: ViT-g's 88 runs the 96 tile (8 % zero
    columns) instead of the 128 one (31 %)."""
    return next(x for x in FLASH_DIMS if x >= d)


def _native_dim(d):
    """Head dims the kernels take as they are: the tile columns past ``d`` are
    read as zeros by the loaders and never stored (16-byte column chunks)."""
    return 0 < d <= 128 and d % 8 == 0


def flash_attention(q, k, v, causal=True, dropout_p=0.0, key=0, scale=None, kv_lens=None,
                    key_bias=None):
    """q: [B, Sq, H, D], k/v: [B, Sk, H, D] (strided views allowed).

    Head dims that are multiples of 8 up to 128 run natively on the next tile
    width (ViT-g's 88 on the 96 tile: the loaders read the missing columns as
    zeros, no padded copies).  Other dims <= 128 are zero-padded to the tile
    width: zero columns add nothing to QK^T and produce zero output
    columns that are sliced off (the softmax scale keeps the true ``D``)."""
    D = q.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if key_bias is not None and causal:
        raise ValueError("key_bias is supported for non-causal attention only")
    if not q.is_cuda:
        return attention_reference(q, k, v, causal, dropout_p, key, scale, kv_lens, key_bias)
    if not _native_dim(D):
        if D > 128:
            # wider heads than one MFMA tile row: exact fp32 math path (S x S materialised)
            if not _WARNED.get(D):
                _WARNED[D] = True
                import warnings
                warnings.warn("head_dim %d > 128: attention runs unfused (GEMM + HIP softmax)" % D)
            return _unfused_attention(q, k, v, causal, dropout_p, key, scale, kv_lens, key_bias)
        P = _padded_dim(D) - D
        pad = lambda t: torch.nn.functional.pad(t, (0, P))  # noqa: E731
        out = _FlashAttn.apply(pad(q), pad(k), pad(v), None, causal, float(dropout_p), key,
                               scale, kv_lens, key_bias)
        return out[..., :D]
    return _FlashAttn.apply(q, k, v, None, causal, float(dropout_p), key, scale, kv_lens, key_bias)


def flash_attention_qkvpacked(qkv, causal=True, dropout_p=0.0, key=0, scale=None, kv_lens=None,
                              key_bias=None, pack_dim=3):
    """qkv: [B, S, H, 3, D] (``pack_dim=3``, GPT's per-head interleave) or
    [B, S, 3, H, D] (``pack_dim=2``, ViT / timm) -> out [B, S, H, D].  The
    q / k / v gradients land straight in one packed buffer of qkv's layout
    (no per-slice zero fill + copy + add in autograd)."""
    D = qkv.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if pack_dim not in (2, 3):
        raise ValueError("pack_dim must be 2 or 3")
    if not qkv.is_cuda or not _native_dim(D):
        return flash_attention(qkv.select(pack_dim, 0), qkv.select(pack_dim, 1),
                               qkv.select(pack_dim, 2), causal, dropout_p, key, scale, kv_lens,
                               key_bias)
    if key_bias is not None and causal:
        raise ValueError("key_bias is supported for non-causal attention only")
    return _PackedEntry.apply(qkv, causal, float(dropout_p), key, scale, kv_lens, key_bias,
                              pack_dim)


def decode_splits(B, H, maxlen, target_wgs=2048, min_chunk=512):
    """Split-K factor for decode attention: enough workgroups to cover the 256
    CUs about eight deep (measured: 512 WGs reach 3.2 TB/s, >=1024 5.3 TB/s), at least
    ``min_chunk`` keys per split (a single split writes the output directly:
    short-context decode runs one kernel, no combine pass)."""
    n = max(1, -(-target_wgs // max(1, B * H)))
    return max(1, min(n, -(-maxlen // min_chunk)))


def decode_attention(q, k_cache, v_cache, lens, scale=None, nsplit=None):
    """Single-token attention over a KV cache (split-K, bf16 / fp16).

    q: [B, H, D]; caches: [B, maxlen, H, D]; lens: int32 [B] valid lengths.
    """
    B, H, D = q.shape
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if not q.is_cuda:
        L = k_cache.shape[1]
        s = torch.einsum("bhd,blhd->bhl", q.float(), k_cache.float()) * scale
        m = torch.arange(L, device=q.device).view(1, 1, L) >= lens.view(B, 1, 1).to(q.device)
        p = torch.softmax(s.masked_fill(m, float("-inf")), -1)
        return torch.einsum("bhl,blhd->bhd", p, v_cache.float()).to(q.dtype)
    dt = _lib.dt_code(q.dtype)
    if k_cache.dtype != q.dtype or v_cache.dtype != q.dtype:
        raise TypeError("decode attention: q / cache dtypes differ")
    if k_cache.stride() != v_cache.stride() or k_cache.stride(-1) != 1 or q.stride(-1) != 1:
        raise ValueError("decode attention: caches must share a layout with contiguous head dim")
    maxlen = k_cache.shape[1]
    ns = nsplit or decode_splits(B, H, maxlen)
    out = torch.empty(B, H, D, device=q.device, dtype=q.dtype)
    ws = torch.empty(B * H * ns * (D + 2), device=q.device, dtype=torch.float32)
    rc = _lib.kernels().decode_attn(dt, q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                                    out.data_ptr(), lens.to(torch.int32).contiguous().data_ptr(),
                                    B, H, D, maxlen, ns, ws.data_ptr(), q.stride(0), q.stride(1),
                                    k_cache.stride(0), k_cache.stride(1), k_cache.stride(2),
                                    out.stride(0), float(scale), _lib.stream())
    if rc != 0:
        raise NotImplementedError("decode attention supports head_dim 64/128 (rc %d)" % rc)
    return out

"""Tied LM head + vocab-parallel softmax cross-entropy, chunked over tokens,
without ever materialising the ``[tokens, vocab]`` logits.

Reference: the LM head ``parallel_matmul`` + ``ParallelCrossEntropy`` pair
(``hybrid_model.py:45-66,781-783,822-827``; SURVEY N-8 / K11).  The unfused
path here (``ops.softmax_cross_entropy`` on the full logits) keeps a bf16
``[b*s, V/t]`` tensor alive from the forward to the backward -- 824 MB for
GPT-3 at 8 x 1024 tokens, growing with micro-batch and sequence length.

MI355X design.  The loss is ``sum_i mask_i ce_i / sum_i mask_i`` and its
upstream gradient is one scalar, so the whole backward of the head can run
inside the forward, chunk by chunk:

    for each chunk of C token rows:
        logits_c = h_c W^T                       (GEMM, [C, V/t] bf16, transient)
        (max, sumexp, target) -> lse_c, ce_c     (ce_stats kernel + mp combine)
        logits_c <- (softmax - onehot) g_c       (ce_bwd kernel, in place)
        dh_c = logits_c W                        (dgrad GEMM)
        main_grad(W) += logits_c^T h_c           (fp32 wgrad GEMM, beta = 1 after
                                                  the first chunk of the step)

with ``g_c = mask_c / sum(mask) x s`` where ``s`` is the upstream gradient the
engine declares before the forward (``declare_grad_scale``: 1 / accumulation
steps x the fp16 loss scale, a device scalar).  Backward only rescales the
stored ``dh`` (``[tokens, h]``, 64 MB for 6.7B) by ``g / s``.  A backward
called with any other gradient cannot re-scale the weight gradient already in
``main_grad``; it raises the device flag that ``check()`` turns into an error
(the engine calls it at every logging sync).

Cost: the wgrad of the head becomes one accumulation per chunk (an extra
read + write of the fp32 ``[V/t, h]`` gradient per chunk), so this trades a
little time for the logits' memory: ``Model.fused_lm_head_ce`` (default off)
turns it on where the memory matters (long sequences, large micro-batches).
"""
import os

import torch

from . import _lib

_STATE = {"scale": None, "bad": None}


def declare_grad_scale(loss_scale=None, accumulate_steps=1):
    """The upstream gradient the next backward will feed the loss: ``1 /
    accumulate_steps`` times ``loss_scale`` (a device scalar or None)."""
    s = _STATE["scale"]
    dev = loss_scale.device if torch.is_tensor(loss_scale) else None
    if s is None or (dev is not None and s.device != dev):
        if dev is None:
            dev = "cuda" if torch.cuda.is_available() else "cpu"
        s = torch.ones((), dtype=torch.float32, device=dev)
        _STATE["scale"] = s
        _STATE["bad"] = torch.zeros((), dtype=torch.int32, device=s.device)
    s.fill_(1.0 / float(accumulate_steps))
    if loss_scale is not None:
        s.mul_(loss_scale)
    return s


def _scale(device):
    s = _STATE["scale"]
    if s is None or s.device != device:
        s = torch.ones((), dtype=torch.float32, device=device)
        _STATE["scale"] = s
        _STATE["bad"] = torch.zeros((), dtype=torch.int32, device=device)
    return s


def check():
    """Raise if a backward ran with a gradient other than the declared one."""
    bad = _STATE["bad"]
    if bad is not None and int(bad.item()) != 0:
        bad.zero_()
        raise RuntimeError("fused LM-head cross-entropy: the backward's upstream gradient "
                           "differs from declare_grad_scale(); the tied weight's gradient "
                           "is wrong for this step")


def chunk_rows(vocab_local, budget_mb=128):
    """Token rows per chunk: transient logits of at most ``budget_mb`` (bf16),
    a multiple of 256 (whole GEMM tiles), at least 256."""
    c = int(budget_mb * 2 ** 20 // (2 * max(1, vocab_local)))
    return max(256, c // 256 * 256)


class _ChunkedHeadCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h2, weight, labels, mask, group, vocab_start, chunk, ignore_index):
        from ..parallel.linear import fwd_gemm, dgrad_gemm, _accumulate_wgrad
        from .loss_embed import _allreduce
        import torch.distributed as dist
        T, H = h2.shape
        V = weight.shape[0]
        dev = h2.device
        k = _lib.kernels() if h2.is_cuda else None
        st = _lib.stream() if k is not None else None
        dc = _lib.dt_code(h2.dtype) if k is not None else None
        lab = labels.reshape(-1).contiguous()
        m = mask.reshape(-1).float()
        denom = m.sum()
        s = _scale(dev)
        g_rows = (m / denom) * s                       # d loss_total / d ce_i, declared scale
        ce = torch.empty(T, device=dev, dtype=torch.float32)
        dh = torch.empty(T, H, device=dev, dtype=h2.dtype)
        tp = group is not None and group.nranks > 1
        for r0 in range(0, T, chunk):
            r1 = min(T, r0 + chunk)
            hc = h2[r0:r1]
            logits = fwd_gemm(hc, weight)             # [c, V] bf16, transient
            rows = r1 - r0
            mx = torch.empty(rows, device=dev, dtype=torch.float32)
            sm = torch.empty_like(mx)
            tg = torch.empty_like(mx)
            lc = lab[r0:r1]
            local = lc - vocab_start
            inr = (local >= 0) & (local < V) & (lc != ignore_index)
            if k is not None:
                k.ce_stats(dc, logits.data_ptr(), lc.data_ptr(), rows, V, int(vocab_start),
                           mx.data_ptr(), sm.data_ptr(), tg.data_ptr(), int(ignore_index), st)
            else:  # CPU: the same statistics in PyTorch
                xf = logits.float()
                mx = xf.max(-1).values
                sm = torch.exp(xf - mx[:, None]).sum(-1)
                tg = torch.where(inr, xf.gather(1, local.clamp(0, V - 1)[:, None])[:, 0],
                                 torch.zeros_like(mx))
            if tp:
                gmx = _allreduce(mx.clone(), dist.ReduceOp.MAX, group)
                pair = torch.stack([sm * torch.exp(mx - gmx), tg])
                _allreduce(pair, dist.ReduceOp.SUM, group)
                sm, tg, mx = pair[0], pair[1], gmx
            lse = torch.log(sm) + mx
            ce[r0:r1] = torch.where(lc == ignore_index, torch.zeros_like(lse), lse - tg)
            gc = g_rows[r0:r1].contiguous()
            if k is not None:
                k.ce_bwd(dc, logits.data_ptr(), logits.data_ptr(), lc.data_ptr(), lse.data_ptr(),
                         gc.data_ptr(), rows, V, int(vocab_start), int(ignore_index), st)
            else:
                p = torch.exp(logits.float() - lse[:, None])
                p[inr, local[inr]] -= 1.0
                logits = (p * gc[:, None]).to(logits.dtype)
            dh[r0:r1] = dgrad_gemm(logits, weight)
            # the tied weight's LM-head part: notified once, after the last chunk
            _accumulate_wgrad(weight, logits, hc, notify=r1 == T)
            del logits
        loss = (ce * m).sum() / denom
        ctx.save_for_backward(dh, s.clone())
        return loss

    @staticmethod
    def backward(ctx, g):
        dh, s = ctx.saved_tensors
        bad = _STATE["bad"]
        if bad is not None and bad.device == g.device:
            bad.add_(((g.float() - s).abs() > 1e-6 * s.abs()).int())
        return dh * (g.float() / s).to(dh.dtype), None, None, None, None, None, None, None


def supported(h2, weight):
    """The fused path needs the tied weight's fp32 ``main_grad`` (the flat
    gradient buffer); on the CPU the CE statistics / gradient run in PyTorch."""
    return (h2.dim() == 2 and getattr(weight, "_fx_fused_wgrad", False)
            and hasattr(weight, "main_grad")
            and (not h2.is_cuda or h2.dtype in (torch.bfloat16, torch.float16)))


def lm_head_cross_entropy(h2, weight, labels, mask, group=None, vocab_start=0, chunk=None,
                          ignore_index=-100):
    """``sum(ce(h2 W^T, labels) * mask) / sum(mask)`` over a vocab shard
    (``group``: the mp group of a vocab-parallel head), logits never whole.
    ``h2`` is ``[tokens, h]`` after the mp copy / sequence gather."""
    if chunk is None:
        chunk = int(os.environ.get("FLEETX_LM_HEAD_CE_CHUNK", "0")) or chunk_rows(weight.shape[0])
    return _ChunkedHeadCE.apply(h2, weight, labels, mask, group, vocab_start, int(chunk),
                                int(ignore_index))

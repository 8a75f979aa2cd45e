"""Softmax cross-entropy (vocab-parallel) and (vocab-parallel) embedding.

Reference K10 / K11 (``single_model.py:448-472,626,647-653``;
``hybrid_model.py:590-594,799,822-832``; ``ParallelCrossEntropy`` with its
three mp all-reduces).  Here the statistics kernel emits per-row
``(max, sum-exp, target-logit)`` for the local vocab shard, and the
tensor-parallel combine is two RCCL all-reduces of [tokens] fp32 vectors
(max, then the packed [sum, target] pair).  Backward overwrites the logits in
place with ``(softmax - onehot) * g``.
"""
import os

import torch
import torch.distributed as dist

from . import _lib


def _allreduce(t, op, group):
    # latency-bound [tokens] fp32 vectors: the one-shot IPC kernel when the mp
    # group is one node, RCCL otherwise (parallel/comm.py)
    if group is not None and group.nranks > 1:
        if t.is_cuda:
            from ..parallel.comm import get_communicator
            return get_communicator(group).all_reduce(t, op)
        dist.all_reduce(t, op=op, group=group.group)
    return t


class _SoftmaxCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, group, vocab_start, ignore_index, inplace_backward):
        V = logits.shape[-1]
        x = logits.reshape(-1, V)
        lab = labels.reshape(-1).contiguous()
        rows = x.shape[0]
        if x.is_cuda:
            x = x.contiguous()
            k = _lib.kernels()
            mx = torch.empty(rows, device=x.device, dtype=torch.float32)
            sm = torch.empty_like(mx)
            tg = torch.empty_like(mx)
            k.ce_stats(_lib.dt_code(x.dtype), x.data_ptr(), lab.data_ptr(), rows, V,
                       int(vocab_start), mx.data_ptr(), sm.data_ptr(), tg.data_ptr(),
                       int(ignore_index), _lib.stream())
        else:
            xf = x.float()
            mx = xf.max(-1).values
            sm = torch.exp(xf - mx[:, None]).sum(-1)
            local = lab - vocab_start
            inr = (local >= 0) & (local < V) & (lab != ignore_index)
            tg = torch.where(inr, xf.gather(1, local.clamp(0, V - 1)[:, None])[:, 0],
                             torch.zeros_like(mx))
        if group is not None and group.nranks > 1:
            gmx = _allreduce(mx.clone(), dist.ReduceOp.MAX, group)
            pair = torch.stack([sm * torch.exp(mx - gmx), tg])
            _allreduce(pair, dist.ReduceOp.SUM, group)
            sm, tg, mx = pair[0], pair[1], gmx
        lse = torch.log(sm) + mx
        loss = lse - tg
        loss = torch.where(lab == ignore_index, torch.zeros_like(loss), loss)
        ctx.vocab_start, ctx.ignore_index, ctx.inplace = vocab_start, ignore_index, inplace_backward
        ctx.shape = logits.shape
        ctx.save_for_backward(x, lab, lse)
        return loss.view(labels.shape)

    @staticmethod
    def backward(ctx, dloss):
        x, lab, lse = ctx.saved_tensors
        rows, V = x.shape
        g = dloss.reshape(-1).float().contiguous()
        if x.is_cuda:
            dx = x if ctx.inplace else torch.empty_like(x)
            _lib.kernels().ce_bwd(_lib.dt_code(x.dtype), x.data_ptr(), dx.data_ptr(),
                                  lab.data_ptr(), lse.data_ptr(), g.data_ptr(), rows, V,
                                  int(ctx.vocab_start), int(ctx.ignore_index), _lib.stream())
        else:
            p = torch.exp(x.float() - lse[:, None])
            local = lab - ctx.vocab_start
            inr = (local >= 0) & (local < V) & (lab != ctx.ignore_index)
            onehot = torch.zeros_like(p)
            onehot[inr, local[inr]] = 1.0
            dx = ((p - onehot) * g[:, None]).to(x.dtype)
        return dx.view(ctx.shape), None, None, None, None, None


def softmax_cross_entropy(logits, labels, group=None, vocab_start=0, ignore_index=-100,
                          inplace_backward=True):
    """Per-token CE in fp32. ``group``: mp CommGroup for a vocab-sharded logits."""
    return _SoftmaxCE.apply(logits, labels, group, vocab_start, ignore_index, inplace_backward)


def deterministic():
    """``Global.deterministic`` / ``FLEETX_DETERMINISTIC=1``: reproducible
    reductions (no fp32 atomics in the embedding backward)."""
    return os.environ.get("FLEETX_DETERMINISTIC", "0") == "1"


def _embedding_bwd(k, dc, ids, d, dw32, ntok, h, vstart, vsize, st):
    if deterministic():
        sid, perm = torch.sort(ids.reshape(-1), stable=True)
        k.embedding_bwd_sorted(dc, sid.data_ptr(), perm.data_ptr(), d.data_ptr(), dw32.data_ptr(),
                               ntok, h, vstart, vsize, st)
        return
    k.embedding_bwd(dc, ids.data_ptr(), d.data_ptr(), dw32.data_ptr(), ntok, h, vstart, vsize, st)


def _grad_target(p, shape, device):
    """fp32 buffer the scatter-add kernel accumulates into: the parameter's
    flat-buffer ``main_grad`` when it takes fused gradients (no bf16 round
    trip, no extra 4 B/elt copy), else a fresh zeroed tensor."""
    if p is not None and getattr(p, "_fx_fused_wgrad", False) and hasattr(p, "main_grad"):
        if getattr(p, "_fx_fresh", False):
            p.main_grad.zero_()
            p._fx_fresh = False
        return p.main_grad, True
    return torch.zeros(*shape, device=device, dtype=torch.float32), False


def _grad_finish(p, g32, fused, dtype):
    if fused:
        from ..parallel.linear import grad_part_done
        grad_part_done(p)
        return None
    return g32.to(dtype)


class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight, pos_ids, pos_weight, vocab_start):
        ntok = ids.numel()
        h = weight.shape[1]
        vsize = weight.shape[0]
        ids_c = ids.reshape(-1).contiguous()
        pos_c = pos_ids.reshape(-1).contiguous() if pos_ids is not None else None
        if weight.is_cuda:
            out = torch.empty(ntok, h, device=weight.device, dtype=weight.dtype)
            _lib.kernels().embedding_fwd(_lib.dt_code(weight.dtype), ids_c.data_ptr(),
                                         _lib.ptr(pos_c), weight.data_ptr(), _lib.ptr(pos_weight),
                                         out.data_ptr(), ntok, h, int(vocab_start), vsize,
                                         _lib.stream())
        else:
            local = ids_c - vocab_start
            inr = (local >= 0) & (local < vsize)
            out = weight[local.clamp(0, vsize - 1)] * inr[:, None].to(weight.dtype)
            if pos_weight is not None:
                out = out + pos_weight[pos_c]
        ctx.vocab_start, ctx.vsize, ctx.h = vocab_start, vsize, h
        ctx.has_pos = pos_weight is not None
        ctx.pos_rows = pos_weight.shape[0] if pos_weight is not None else 0
        ctx.save_for_backward(ids_c, pos_c)
        ctx.wdtype = weight.dtype
        ctx.params = (weight, pos_weight)
        return out.view(*ids.shape, h)

    @staticmethod
    def backward(ctx, dout):
        ids_c, pos_c = ctx.saved_tensors
        h = ctx.h
        d = dout.reshape(-1, h).contiguous()
        ntok = d.shape[0]
        dpos = None
        if d.is_cuda:
            k = _lib.kernels()
            dc = _lib.dt_code(d.dtype)
            st = _lib.stream()
            wp, pp = ctx.params
            dw32, fused = _grad_target(wp, (ctx.vsize, h), d.device)
            _embedding_bwd(k, dc, ids_c, d, dw32, ntok, h, int(ctx.vocab_start), ctx.vsize, st)
            dw = _grad_finish(wp, dw32, fused, ctx.wdtype)
            if ctx.has_pos:
                dp32, fused = _grad_target(pp, (ctx.pos_rows, h), d.device)
                _embedding_bwd(k, dc, pos_c, d, dp32, ntok, h, 0, ctx.pos_rows, st)
                dpos = _grad_finish(pp, dp32, fused, ctx.wdtype)
        else:
            wp, pp = ctx.params
            local = ids_c - ctx.vocab_start
            inr = (local >= 0) & (local < ctx.vsize)
            dw32, fused = _grad_target(wp, (ctx.vsize, h), d.device)
            dw32.index_add_(0, local[inr], d[inr].float())
            dw = _grad_finish(wp, dw32, fused, ctx.wdtype)
            if ctx.has_pos:
                dp32, fused = _grad_target(pp, (ctx.pos_rows, h), d.device)
                dp32.index_add_(0, pos_c, d.float())
                dpos = _grad_finish(pp, dp32, fused, ctx.wdtype)
        return None, dw, None, dpos, None


def embedding(ids, weight, pos_ids=None, pos_weight=None, vocab_start=0):
    """Fused word (+ position) embedding; rows outside the shard give zeros."""
    return _Embedding.apply(ids, weight, pos_ids, pos_weight, vocab_start)

"""Sequence-parallel linears with the all-gather / reduce-scatter cut into
chunks that overlap the GEMMs (reference ``ColumnSequenceParallelLinear`` /
``RowSequenceParallelLinear``, ``sequence_parallel_utils.py:99-126,226-228,319``;
SURVEY N06/N07).

Activations under sequence parallelism are sequence-first ``[s/t, b, h]``
shards.  Each rank's shard is cut into ``c`` contiguous sub-chunks along the
sequence; sub-chunk ``k`` of every rank travels in ONE RCCL collective, and the
GEMM of sub-chunk ``k`` runs while the collective of sub-chunk ``k+1`` is in
flight on RCCL's stream (all collectives are posted up front, the compute
stream waits per chunk):

* column (fwd): all-gather(k) -> ``t`` GEMMs writing straight into the full
  output rows of sub-chunk ``k`` of every rank (contiguous row blocks, no
  reorder pass);
* column (bwd): per chunk, ``t`` dgrad GEMMs into a staging block, its
  reduce-scatter posted at once, the weight gradient accumulates chunk by
  chunk in fp32 (``main_grad``) under the reduce-scatters;
* row (fwd): per chunk, ``t`` GEMMs into a staging block, reduce-scatter
  posted at once -> the next chunk's GEMMs hide it.  The last chunk's
  scatter is exposed: the output feeds the residual add and LayerNorm of
  every row, and the next linear's gather needs those; hiding it would mean
  running the next layer's norm and gather chunk by chunk as well;
* row (bwd): chunked all-gather of the output gradient, dgrad / wgrad per
  chunk as it lands.

On xGMI the ring collectives are per-link bandwidth bound, so ``c = 2`` (two
half-size collectives) already hides most of the transfer behind GEMMs of a
GPT-3 layer; more chunks only add launch latency.

Chunk-major layout (``chunk_major=True``, the MLP's FC1 -> GeLU -> FC2):
the full-sequence activation between a column-SP and a row-SP linear is
only ever touched row-wise (bias + GeLU), so its rows may be kept in
(chunk, rank, row) order instead of sequence order.  Sub-chunk ``k`` of
every rank is then ONE contiguous ``[t * s/(t c) * b, .]`` block, and each
chunk is a single GEMM instead of ``t`` (FC1 forward / data gradient, FC2
forward / data gradient, and both weight gradients).  Attention needs the
sequence order, so QKV and the output projection keep it.
"""
import torch
import torch.distributed as dist

from .linear import accumulate_wgrad, grad_part_done, G

SP_CHUNKS = {"chunks": 2}


def _mm_into(a2, w, out2, bias=None):
    """``out2 = a2 @ w^T (+ bias)`` into a contiguous 2-D block."""
    if G.use("fwd", a2, w) and G.linear_fwd(a2, w, bias, out=out2) is not None:
        return
    if bias is not None:
        torch.addmm(bias, a2, w.t(), out=out2)
    else:
        torch.mm(a2, w.t(), out=out2)


def _dgrad_into(dy2, w, out2):
    """``out2 = dy2 @ w`` (the MFMA kernel when the shipped plan / route
    picks it for this shape, as the non-SP data gradients)."""
    if G.use("dgrad", dy2, w) and G.linear_dgrad(dy2, w, out=out2) is not None:
        return
    torch.mm(dy2, w, out=out2)


def _post_ag(x, g, c):
    """Post ``c`` all-gathers of the sub-chunks of ``x`` [S, ...]; returns
    [(work, gathered [t, S/c, ...])]."""
    t = g.nranks
    sc = x.shape[0] // c
    out = []
    for k in range(c):
        part = x[k * sc:(k + 1) * sc].contiguous()
        buf = torch.empty((t * sc,) + tuple(part.shape[1:]), dtype=x.dtype, device=x.device)
        w = dist.all_gather_into_tensor(buf, part, group=g.group, async_op=True)
        out.append((w, buf.view((t,) + tuple(part.shape)), part))
    return out


def _wgrad_chunks(weight, pairs, want_bias):
    """Weight (and bias) gradient from (dy2, x2) row blocks.  Fused fp32
    main_grad accumulation when the weight lives in a flat grad buffer (the
    buffer is notified once, after the last block); else a plain tensor."""
    fused = hasattr(weight, "main_grad") and getattr(weight, "_fx_fused_wgrad", False)
    if fused:
        for i, (dy2, x2) in enumerate(pairs):
            accumulate_wgrad(weight, dy2, x2, notify=(i == len(pairs) - 1))
        dw = None
    else:
        dw = None
        for dy2, x2 in pairs:
            part = torch.mm(dy2.t(), x2)
            dw = part if dw is None else dw.add_(part)
        dw = dw.to(weight.dtype)
    db = None
    if want_bias:
        db = sum(dy2.float().sum(0) for dy2, _ in pairs)
    return dw, db


class _ColumnSP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, g, c, cm):
        t = g.nranks
        S, B, h = x.shape
        n = weight.shape[0]
        sc = S // c
        gathered = _post_ag(x, g, c)
        y = torch.empty(t * S, B, n, dtype=x.dtype, device=x.device)
        yv = y.view(c, t * sc * B, n) if cm else y.view(t, c, sc * B, n)
        bufs = []
        for k, (w, buf, _) in enumerate(gathered):
            w.wait()
            if cm:  # chunk k of every rank: one GEMM into one contiguous block
                _mm_into(buf.view(t * sc * B, h), weight, yv[k], bias)
            else:
                for r in range(t):
                    _mm_into(buf[r].view(sc * B, h), weight, yv[r, k], bias)
            bufs.append(buf)
        ctx.g, ctx.c, ctx.cm, ctx.has_bias = g, c, cm, bias is not None
        ctx.shape = (S, B, h, n)
        ctx.save_for_backward(weight, *bufs)
        return y

    @staticmethod
    def backward(ctx, dy):
        weight, *bufs = ctx.saved_tensors
        g, c, cm = ctx.g, ctx.c, ctx.cm
        t = g.nranks
        S, B, h, n = ctx.shape
        sc = S // c
        dyv = dy.contiguous().view(c, t * sc * B, n) if cm else dy.contiguous().view(t, c, sc * B, n)
        dx = torch.empty(S, B, h, dtype=dy.dtype, device=dy.device)
        works = []
        for k in range(c):
            stage = torch.empty(t, sc * B, h, dtype=dy.dtype, device=dy.device)
            if cm:
                _dgrad_into(dyv[k], weight, stage.view(t * sc * B, h))
            else:
                for r in range(t):
                    _dgrad_into(dyv[r, k], weight, stage[r])
            works.append((dist.reduce_scatter_tensor(dx[k * sc:(k + 1) * sc].view(sc * B, h),
                                                     stage.view(t * sc * B, h), group=g.group,
                                                     async_op=True), stage))
        if cm:
            pairs = [(dyv[k], bufs[k].view(t * sc * B, h)) for k in range(c)]
        else:
            pairs = [(dyv[r, k], bufs[k][r].view(sc * B, h)) for k in range(c) for r in range(t)]
        dw, db = _wgrad_chunks(weight, pairs, ctx.has_bias)
        for w, _ in works:
            w.wait()
        if db is not None:
            db = db.to(weight.dtype)
        return dx, dw, db, None, None, None


class _RowSP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, g, c, cm):
        t = g.nranks
        S_full, B, hin = x.shape
        S = S_full // t
        n = weight.shape[0]
        sc = S // c
        xv = x.contiguous().view(c, t * sc * B, hin) if cm else x.contiguous().view(t, c, sc * B, hin)
        y = torch.empty(S, B, n, dtype=x.dtype, device=x.device)
        works = []
        for k in range(c):
            stage = torch.empty(t, sc * B, n, dtype=x.dtype, device=x.device)
            if cm:
                _mm_into(xv[k], weight, stage.view(t * sc * B, n))
            else:
                for r in range(t):
                    _mm_into(xv[r, k], weight, stage[r])
            works.append((dist.reduce_scatter_tensor(y[k * sc:(k + 1) * sc].view(sc * B, n),
                                                     stage.view(t * sc * B, n), group=g.group,
                                                     async_op=True), stage))
        for w, _ in works:
            w.wait()
        ctx.g, ctx.c, ctx.cm = g, c, cm
        ctx.save_for_backward(x, weight)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        g, c, cm = ctx.g, ctx.c, ctx.cm
        t = g.nranks
        S_full, B, hin = x.shape
        S = S_full // t
        n = weight.shape[0]
        sc = S // c
        xv = x.contiguous().view(c, t * sc * B, hin) if cm else x.contiguous().view(t, c, sc * B, hin)
        gathered = _post_ag(dy.contiguous(), g, c)
        dx = torch.empty(S_full, B, hin, dtype=dy.dtype, device=dy.device)
        dxv = dx.view(c, t * sc * B, hin) if cm else dx.view(t, c, sc * B, hin)
        pairs = []
        for k, (w, buf, _) in enumerate(gathered):
            w.wait()
            if cm:
                dyb = buf.view(t * sc * B, n)
                _dgrad_into(dyb, weight, dxv[k])
                pairs.append((dyb, xv[k]))
            else:
                for r in range(t):
                    dyb = buf[r].view(sc * B, n)
                    _dgrad_into(dyb, weight, dxv[r, k])
                    pairs.append((dyb, xv[r, k]))
        dw, _ = _wgrad_chunks(weight, pairs, False)
        return dx, dw, None, None, None


def _chunks_for(S):
    c = max(1, int(SP_CHUNKS["chunks"]))
    while c > 1 and S % c:
        c -= 1
    return c


def column_sp_linear(x, weight, bias, group, chunk_major=False):
    """``all_gather_seq(x) @ W^T (+ b)`` with the gather overlapped; rows in
    (chunk, rank, row) order with ``chunk_major`` (feed a chunk-major
    :func:`row_sp_linear` only)."""
    return _ColumnSP.apply(x, weight, bias, group, _chunks_for(x.shape[0]), bool(chunk_major))


def row_sp_linear(x, weight, group, chunk_major=False):
    """``reduce_scatter_seq(x @ W^T)`` with the scatter overlapped; ``x`` in
    the chunk-major row order of a chunk-major :func:`column_sp_linear`."""
    return _RowSP.apply(x, weight, group, _chunks_for(x.shape[0] // group.nranks),
                        bool(chunk_major))


__all__ = ["column_sp_linear", "row_sp_linear", "SP_CHUNKS", "grad_part_done"]

"""Linear layers on the hand-written gfx950 GEMM (``ops.gemm``), with the
weight-gradient GEMM accumulating straight into the fp32 ``main_grad`` buffer.

GEMM routing: every forward / data-gradient / weight-gradient GEMM first tries
the MFMA kernel in its native operand layout (no transposed copies), with the
bias, GeLU and GeLU-derivative fused into its epilogue (``fused_mlp``); shapes
it does not cover (or ``FLEETX_GEMM=blas``) take the hipBLASLt paths below.

Without this, every weight gradient goes hipBLASLt (bf16 dW) -> autograd
``.grad`` -> a post-accumulate hook that adds it into the fp32 flat buffer:
an extra read-modify-write of the whole fp32 gradient (~22 ms per step for
GPT-3 6.7B on one MI355X, measured with rocprofv3) plus the bf16 temporaries.
Here the wgrad GEMM writes fp32 directly (``mm``/``addmm`` with
``out_dtype=float32``, beta = 0 for the first micro-batch of a step and 1
afterwards), so the flat gradient buffer is never zero-filled either.

Operand layout: the reduction of the wgrad GEMM runs over tokens, the slow
axis of both row-major activations, and hipBLASLt's kernels for that "NT"
case reach only ~1.0 PFLOP/s on gfx950.  On GPU both operands are first
transposed to token-contiguous copies by the LDS-tiled HIP transpose
(``ops.elementwise.transpose2d``) so the GEMM runs as "TN" (~1.35 PFLOP/s
with fp32 accumulate; ``tools/bench_gemm.py``).
"""

import torch
import torch.nn.functional as F

from ..ops import gemm as G

_MM_DTYPE_OUT = None


def _mm_out_supported():
    global _MM_DTYPE_OUT
    if _MM_DTYPE_OUT is None:
        _MM_DTYPE_OUT = hasattr(torch.ops.aten.mm, "dtype_out") and \
            hasattr(torch.ops.aten.addmm, "dtype_out")
    return _MM_DTYPE_OUT



def dgrad(dy, w):
    """``dy @ w`` (data gradient of ``F.linear(x, w)``).  On GPU the weight is
    first transposed (LDS-tiled HIP transpose, ~2 B/elt each way) so the GEMM
    runs as ``F.linear(dy, w^T)`` -- the "TN" layout hipBLASLt's tuned kernels
    cover (~1.5 vs ~1.3 PFLOP/s for the "NN" call on the GPT-3 6.7B shapes;
    ``tools/bench_gemm.py``).

    The transpose costs ~4 B per weight element at ~4.5 TB/s while the GEMM
    saves ~13 % of 2*M FLOPs per element at ~1.4 PFLOP/s: it pays off from
    M ~ 4.5k rows, so smaller micro-batches (pipeline schedules) keep NN.
    (Caching ``w^T`` -- rewritten by the forward-overlapped optimizer beside
    the next forward -- measured 4.7 ms/step SLOWER on 6.7B than transposing
    here: that region is already bandwidth-saturated; profiles/r4_step/.)"""
    if dy.is_cuda and dy.dtype in (torch.bfloat16, torch.float16) \
            and w.dtype == dy.dtype and w.dim() == 2 and w.shape[0] % 8 == 0 \
            and w.shape[1] % 8 == 0 and dy.numel() // dy.shape[-1] >= 6144:
        from ..ops.elementwise import transpose2d
        return F.linear(dy, transpose2d(w))
    return torch.matmul(dy, w)


G.VENDOR["dgrad"] = dgrad
G.VENDOR["fwd"] = F.linear


def _fused(p):
    return p is not None and getattr(p, "_fx_fused_wgrad", False) and hasattr(p, "main_grad")


def _tn_operands(dy2, x2, colsum=None):
    """(dy2^T, x2) as (token-contiguous dyT, xT^T view) when the TN path applies;
    ``colsum`` = (fp32 target, accumulate) takes dy2's column sums on the way."""
    if not (dy2.is_cuda and dy2.dtype in (torch.bfloat16, torch.float16)
            and x2.dtype == dy2.dtype):
        return None
    from ..ops.elementwise import transpose2d
    M = dy2.shape[0]
    if M % 8 or dy2.shape[1] % 8 or x2.shape[1] % 8 or M < 256:
        return None
    return transpose2d(dy2, colsum=colsum), transpose2d(x2).t()


# Weight-gradient GEMMs on the shared side stream (Distributed.comm.wgrad_stream,
# opt-in): the data-gradient chain of backward never waits for them, so on
# models whose GEMMs under-fill the 256 CUs (hidden <= 2048: 8192 x 1024 x 1024
# is 128 tiles of 256 x 256) the wgrad of layer l runs beside the dgrad of
# layer l-1 (+1.5 % on 345M / 1.3B).  Joined by the gradient buffer before any
# collective / the optimizer.  Only wgrads on the hand-written kernel go there
# (see accumulate_wgrad): two concurrent vendor stream-K GEMMs can deadlock.
WGRAD_STREAM = {"enabled": False, "stream": None}


def _wgrad_side_stream(dev):
    if not WGRAD_STREAM["enabled"]:
        return None
    s = WGRAD_STREAM["stream"]
    if s is None or s.device != dev:
        from ..utils.streams import side_stream
        s = side_stream(dev)
        WGRAD_STREAM["stream"] = s
    return s


def join_wgrad_stream():
    """Order the current stream after every weight gradient issued so far."""
    s = WGRAD_STREAM["stream"]
    if s is not None and WGRAD_STREAM["enabled"]:
        torch.cuda.current_stream(s.device).wait_stream(s)


def accumulate_wgrad(weight, dy2, x2, bias=None, notify=True):
    """``weight.main_grad (+)= dy2^T @ x2`` in fp32; notifies the grad buffer
    (``notify=False``: a partial contribution, more follow in this backward).

    With ``bias`` (a Parameter) the bias gradient ``sum_rows(dy2)`` is produced
    too: straight into ``bias.main_grad`` when the bias takes fused grads
    (returns None), else returned as a tensor for autograd."""
    # Side stream only (a) for weights with ONE gradient part: a tied weight
    # (word embedding: LM-head wgrad + lookup backward) has its other part
    # accumulated into the same main_grad on the main stream; and (b) when
    # the GEMM runs on the hand-written kernel: two vendor stream-K GEMMs in
    # flight on two streams can deadlock (workgroups of one spin on tiles the
    # other's resident workgroups keep from being scheduled; seen on ViT-g)
    side = None
    if dy2.is_cuda and (bias is None or _fused(bias)) and \
            getattr(weight, "_fx_grad_parts", 1) == 1 and G.use("wgrad", dy2, x2) and \
            G.covers_wgrad(dy2, x2):
        side = _wgrad_side_stream(dy2.device)
    if side is None:
        return _accumulate_wgrad(weight, dy2, x2, bias, notify)
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        r = _accumulate_wgrad(weight, dy2, x2, bias, notify=False, bias_notify=False,
                              kernel_only=True)
    if r is _DECLINED:
        # the kernel declined after all (rc != 0): the vendor fallback runs on
        # the main stream, never concurrently with another stream-K GEMM
        return _accumulate_wgrad(weight, dy2, x2, bias, notify)
    dy2.record_stream(side)
    x2.record_stream(side)
    # readiness callbacks may launch collectives: those join the side stream
    if bias is not None:
        grad_part_done(bias)
    if notify:
        grad_part_done(weight)
    return None


_DECLINED = object()


def _accumulate_wgrad(weight, dy2, x2, bias=None, notify=True, bias_notify=True,
                      kernel_only=False):
    """``kernel_only``: return ``_DECLINED`` (nothing written) instead of
    running the hipBLASLt fallback when the MFMA kernel declines."""
    mg = weight.main_grad
    fresh = getattr(weight, "_fx_fresh", False)
    # gradient-norm partials from the epilogue (grad_buffer.enable_fused_norm):
    # valid only while EVERY write of this step's gradient produced them
    sq = getattr(weight, "_fx_sq", None)
    done = False
    if G.use("wgrad", dy2, x2):
        if sq is not None and (fresh or weight._fx_sq_ok):
            done = G.linear_wgrad(dy2, x2, mg, not fresh, sq=sq)
            weight._fx_sq_ok = done
        if not done:
            if sq is not None:
                weight._fx_sq_ok = False
            done = G.linear_wgrad(dy2, x2, mg, not fresh)
    elif sq is not None:
        weight._fx_sq_ok = False
    if not done and kernel_only:
        return _DECLINED
    if done:
        db = None
        if bias is not None:
            if _fused(bias):
                colsum_into(dy2, bias.main_grad, not getattr(bias, "_fx_fresh", False))
                bias._fx_fresh = False
                if bias_notify:
                    grad_part_done(bias)
            else:
                db = torch.empty(bias.shape, device=dy2.device, dtype=torch.float32)
                colsum_into(dy2, db, False)
                db = db.to(bias.dtype)
        weight._fx_fresh = False
        if notify:
            grad_part_done(weight)
        return db
    db, colsum = None, None
    if bias is not None:
        if _fused(bias):
            colsum = (bias.main_grad, not getattr(bias, "_fx_fresh", False))
        else:
            db = torch.empty(bias.shape, device=dy2.device, dtype=torch.float32)
            colsum = (db, False)
    tn = _tn_operands(dy2, x2, colsum)
    if tn is None and colsum is not None:
        s = dy2.float().sum(0)
        if colsum[1]:
            colsum[0].add_(s)
        else:
            colsum[0].copy_(s)
    if bias is not None:
        if db is None:
            bias._fx_fresh = False
            if bias_notify:
                grad_part_done(bias)
        else:
            db = db.to(bias.dtype)
    a, b = tn if tn is not None else (dy2.t(), x2)
    if mg.dtype != torch.float32:
        # 16-bit gradient storage (grad_dtype): the vendor GEMM's own fp32
        # accumulation, rounded once into main_grad
        if fresh:
            torch.mm(a, b, out=mg)
        else:
            mg.add_(torch.mm(a, b))
    elif dy2.dtype == torch.float32:
        if fresh:
            torch.mm(a, b, out=mg)
        else:
            mg.addmm_(a, b)
    elif _mm_out_supported() and dy2.is_cuda:
        if fresh:
            torch.ops.aten.mm.dtype_out(a, b, torch.float32, out=mg)
        else:
            torch.ops.aten.addmm.dtype_out(mg, a, b, torch.float32, out=mg)
    else:  # CPU 16-bit models / older torch: fp32 product
        g = torch.mm(a.float(), b.float())
        if fresh:
            mg.copy_(g)
        else:
            mg.add_(g)
    weight._fx_fresh = False
    if notify:
        grad_part_done(weight)
    return db


def grad_part_done(p):
    """One fused contribution to ``p.main_grad`` is in.  A weight used twice in
    a step (the tied word embedding: lookup + LM head, ``_fx_grad_parts = 2``)
    is reported ready to the gradient buffer only after its last part."""
    parts = getattr(p, "_fx_grad_parts", 1)
    if parts > 1:
        p._fx_parts_seen = getattr(p, "_fx_parts_seen", 0) + 1
        if p._fx_parts_seen < parts:
            return
        p._fx_parts_seen = 0
    cb = getattr(p, "_fx_grad_ready", None)
    if cb is not None:
        cb()


def fwd_gemm(x, weight, bias=None):
    """``F.linear`` on the MFMA kernel when it covers the shape."""
    if G.use("fwd", x, weight):
        x2 = x.reshape(-1, x.shape[-1])
        y = G.linear_fwd(x2, weight, bias)
        if y is not None:
            return y.view(*x.shape[:-1], weight.shape[0])
    return F.linear(x, weight, bias)


def dgrad_gemm(dy, w, act_input=None, act="gelu", colsum=None):
    """``dy @ w`` (times ``gelu'(act_input)`` when given) on the MFMA kernel.
    ``colsum = (dst_f32, accumulate)``: column sums of the result as well (the
    fallback takes them from the dGeLU pass; the caller reduces otherwise and
    gets ``done = False`` back through ``colsum_done``).

    With ``act_input`` the GeLU' is fused into the GEMM epilogue only where
    the routing table says so (``dgrad_act``); otherwise the GEMM runs plain
    (MFMA kernel or hipBLASLt, ``dgrad``) and the separate dGeLU pass also
    takes the bias column sums."""
    dy2 = dy.reshape(-1, dy.shape[-1])
    if act_input is not None and G.use("dgrad_act", dy, w):
        ai = act_input.reshape(-1, act_input.shape[-1])
        dx = G.linear_dgrad(dy2, w, act_input=ai, act=act)
        if dx is not None:
            if colsum is not None:
                colsum_into(dx, colsum[0], colsum[1])
            return dx.view(*dy.shape[:-1], w.shape[1])
    dx = None
    if G.use("dgrad", dy, w):
        dx = G.linear_dgrad(dy2, w)
        if dx is not None:
            dx = dx.view(*dy.shape[:-1], w.shape[1])
    if dx is None:
        dx = dgrad(dy, w)
    if act_input is not None:
        from ..ops.elementwise import gelu_grad
        dx = gelu_grad(dx, act_input, erf=(act != "gelu"), colsum=colsum)
    elif colsum is not None:
        colsum_into(dx.reshape(-1, dx.shape[-1]), colsum[0], colsum[1])
    return dx


def colsum_into(dy2, dst, accumulate):
    """``dst (+)= dy2.sum(0)`` in fp32 (HIP column-tile reduction on GPU)."""
    from ..ops.norm import col_sum_f32
    col_sum_f32(dy2, dst, accumulate)


class _FusedWgradLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.bias = bias
        return fwd_gemm(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = dgrad_gemm(dy, w)
        dy2 = dy.reshape(-1, dy.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        db = accumulate_wgrad(w, dy2, x2, ctx.bias)
        return dx, None, db


def linear(x, weight, bias=None):
    """``F.linear`` whose weight gradient lands in ``weight.main_grad`` when the
    weight lives in a :class:`FlatParamGradBuffer` (training); plain otherwise."""
    if torch.is_grad_enabled() and weight.requires_grad and hasattr(weight, "main_grad") \
            and getattr(weight, "_fx_fused_wgrad", False):
        return _FusedWgradLinear.apply(x, weight, bias)
    return F.linear(x, weight, bias)


# ----------------------------------------------------------------------------
# Tensor-parallel linears with communication / compute overlap (xGMI)
# ----------------------------------------------------------------------------
def _wgrad(w, dy2, x2):
    """fp32 fused accumulation when the weight lives in a flat grad buffer,
    else a plain dW to hand back to autograd."""
    if hasattr(w, "main_grad") and getattr(w, "_fx_fused_wgrad", False):
        accumulate_wgrad(w, dy2, x2)
        return None
    if G.use("wgrad", dy2, x2):
        dw = G.wgrad_16(dy2, x2)
        if dw is not None:
            return dw
    return torch.mm(dy2.t(), x2).to(w.dtype)


class _ColumnTPLinear(torch.autograd.Function):
    """y = x W^T (+b) with x replicated over the mp group.

    backward: dX = dY W is all-reduced over mp ASYNCHRONOUSLY while the wgrad
    GEMM runs (reference: ``_c_identity`` backward all-reduce, N02); the wait
    comes after dW, so the xGMI transfer hides behind the GEMM.
    """

    @staticmethod
    def forward(ctx, x, weight, bias, group):
        ctx.save_for_backward(x, weight)
        ctx.group = group
        ctx.has_bias = bias is not None
        return fwd_gemm(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        import torch.distributed as dist
        x, w = ctx.saved_tensors
        dx = dgrad_gemm(dy, w)
        work = dist.all_reduce(dx, group=ctx.group.group, async_op=True)
        dy2 = dy.reshape(-1, dy.shape[-1])
        dw = _wgrad(w, dy2, x.reshape(-1, x.shape[-1]))
        db = dy2.sum(0) if ctx.has_bias else None
        work.wait()
        return dx, dw, db, None


class _RowTPLinear(torch.autograd.Function):
    """y = all_reduce(x W^T) with the GEMM cut into ``chunks`` token slices:
    the all-reduce of slice i (RCCL stream) overlaps the GEMM of slice i+1
    (reference: RowParallelLinear output all-reduce, N03, on the critical
    path).  backward needs no communication (dY is replicated)."""

    @staticmethod
    def forward(ctx, x, weight, group, chunks):
        import torch.distributed as dist
        ctx.save_for_backward(x, weight)
        x2 = x.reshape(-1, x.shape[-1])
        M = x2.shape[0]
        y = torch.empty(M, weight.shape[0], dtype=x.dtype, device=x.device)
        n = max(1, min(chunks, M // 256))
        bounds = [M * i // n for i in range(n + 1)]
        works = []
        wt = weight.t()
        for i in range(n):
            a, b = bounds[i], bounds[i + 1]
            if not (G.use("fwd", x2, weight) and G.linear_fwd(x2[a:b], weight, out=y[a:b])
                    is not None):
                torch.mm(x2[a:b], wt, out=y[a:b])
            works.append(dist.all_reduce(y[a:b], group=group.group, async_op=True))
        for wk in works:
            wk.wait()
        return y.view(*x.shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = dgrad_gemm(dy, w)
        dy2 = dy.reshape(-1, dy.shape[-1])
        dw = _wgrad(w, dy2, x.reshape(-1, x.shape[-1]))
        return dx, dw, None, None


def column_tp_linear(x, weight, bias, group):
    return _ColumnTPLinear.apply(x, weight, bias, group)


def row_tp_linear(x, weight, group, chunks=2):
    return _RowTPLinear.apply(x, weight, group, chunks)


# ----------------------------------------------------------------------------
# Fused MLP (single mp rank): FC1 GEMM + bias + GeLU in one kernel, FC2 GEMM,
# and in backward FC2's data-gradient GEMM applies gelu'(h) in its epilogue.
# ----------------------------------------------------------------------------
class _FusedMLP(torch.autograd.Function):
    """``y = gelu(x W1^T + b1) W2^T`` (FC2 bias left to the caller's epilogue).

    Saves x, the pre-activation h and the activation a (a feeds FC2's weight
    gradient); backward: dW2 (+)= dy^T a, dH = (dy W2) * gelu'(h) (one GEMM),
    db1 = colsum(dH), dW1 (+)= dH^T x, dx = dH W1.  Parity: reference
    ``GPTMLP`` / fused_feedforward (``gpt/dygraph/single_model.py:375``)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, act):
        ctx.act = act
        x2 = x.reshape(-1, x.shape[-1])
        r = G.linear_fwd(x2, w1, b1, act=act) if G.use("fwd_act", x2, w1) else None
        if r is None:
            from ..ops.elementwise import gelu_plain
            h = F.linear(x2, w1, b1)
            a = gelu_plain(h, erf=(act != "gelu"))
        else:
            a, h = r
        y = G.linear_fwd(a, w2) if G.use("fwd", a, w2) else None
        if y is None:
            y = F.linear(a, w2)
        ctx.save_for_backward(x, h, a, w1, b1, w2)
        return y.view(*x.shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x, h, a, w1, b1, w2 = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        dw2 = _wgrad(w2, dy2, a)
        # db1 = colsum(dH) from the same pass as dH where possible; fp32 straight
        # into main_grad when the bias lives in the flat buffer
        db1, cs, into_main = None, None, False
        if b1 is not None:
            if hasattr(b1, "main_grad") and getattr(b1, "_fx_grad_ready", None) is not None:
                cs = (b1.main_grad, not getattr(b1, "_fx_fresh", False))
                into_main = True
            else:
                cs = (torch.empty(b1.shape, device=dy.device, dtype=torch.float32), False)
        dh = dgrad_gemm(dy2, w2, act_input=h, act=ctx.act, colsum=cs)
        if b1 is not None:
            if into_main:
                b1._fx_fresh = False
                grad_part_done(b1)
            else:
                db1 = cs[0].to(b1.dtype)
        dw1 = _wgrad(w1, dh, x2)
        dx = dgrad_gemm(dh, w1)
        return dx.view_as(x), dw1, db1, dw2, None


def fused_mlp(x, w1, b1, w2, act="gelu"):
    return _FusedMLP.apply(x, w1, b1, w2, act)

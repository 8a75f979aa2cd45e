"""Linear with the weight-gradient GEMM accumulating straight into the fp32
``main_grad`` buffer.

Without this, every weight gradient goes hipBLASLt (bf16 dW) -> autograd
``.grad`` -> a post-accumulate hook that adds it into the fp32 flat buffer:
an extra read-modify-write of the whole fp32 gradient (~22 ms per step for
GPT-3 6.7B on one MI355X, measured with rocprofv3) plus the bf16 temporaries.
Here the wgrad GEMM writes fp32 directly (``mm``/``addmm`` with
``out_dtype=float32``, beta = 0 for the first micro-batch of a step and 1
afterwards), so the flat gradient buffer is never zero-filled either.
"""
import torch
import torch.nn.functional as F

_MM_DTYPE_OUT = None


def _mm_out_supported():
    global _MM_DTYPE_OUT
    if _MM_DTYPE_OUT is None:
        _MM_DTYPE_OUT = hasattr(torch.ops.aten.mm, "dtype_out") and \
            hasattr(torch.ops.aten.addmm, "dtype_out")
    return _MM_DTYPE_OUT


def accumulate_wgrad(weight, dy2, x2):
    """``weight.main_grad (+)= dy2^T @ x2`` in fp32; notifies the grad buffer."""
    mg = weight.main_grad
    fresh = getattr(weight, "_fx_fresh", False)
    a, b = dy2.t(), x2
    if dy2.dtype == torch.float32:
        if fresh:
            torch.mm(a, b, out=mg)
        else:
            mg.addmm_(a, b)
    elif _mm_out_supported():
        if fresh:
            torch.ops.aten.mm.dtype_out(a, b, torch.float32, out=mg)
        else:
            torch.ops.aten.addmm.dtype_out(mg, a, b, torch.float32, out=mg)
    else:  # pragma: no cover - older torch
        g = torch.mm(a, b)
        if fresh:
            mg.copy_(g)
        else:
            mg.add_(g)
    weight._fx_fresh = False
    cb = getattr(weight, "_fx_grad_ready", None)
    if cb is not None:
        cb()


class _FusedWgradLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = torch.matmul(dy, w)
        dy2 = dy.reshape(-1, dy.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        accumulate_wgrad(w, dy2, x2)
        db = dy2.sum(0) if ctx.has_bias else None
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
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        import torch.distributed as dist
        x, w = ctx.saved_tensors
        dx = torch.matmul(dy, w)
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
            torch.mm(x2[a:b], wt, out=y[a:b])
            works.append(dist.all_reduce(y[a:b], group=group.group, async_op=True))
        for wk in works:
            wk.wait()
        return y.view(*x.shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = torch.matmul(dy, w)
        dy2 = dy.reshape(-1, dy.shape[-1])
        dw = _wgrad(w, dy2, x.reshape(-1, x.shape[-1]))
        return dx, dw, None, None


def column_tp_linear(x, weight, bias, group):
    return _ColumnTPLinear.apply(x, weight, bias, group)


def row_tp_linear(x, weight, group, chunks=2):
    return _RowTPLinear.apply(x, weight, group, chunks)

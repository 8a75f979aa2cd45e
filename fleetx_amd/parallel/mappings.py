"""Autograd-aware collectives for tensor and sequence parallelism.

Parity:

* ``copy_to_mp``   identity fwd / all-reduce bwd   (Paddle ``_c_identity``)
* ``reduce_from_mp`` all-reduce fwd / identity bwd (RowParallelLinear output)
* ``gather_from_mp`` all-gather last dim / split bwd (``_c_concat``)
* ``scatter_to_seq`` split seq dim / all-gather bwd (``ScatterOp``,
  ``sequence_parallel_utils.py:73-82``)
* ``gather_from_seq`` all-gather seq / split bwd (``GatherOp``, ``:85-94``)
* ``all_gather_seq`` all-gather seq / reduce-scatter bwd (``AllGatherOp``, ``:99-110``)
* ``reduce_scatter_seq`` reduce-scatter seq / all-gather bwd (``ReduceScatterOp``, ``:115-126``)

All collectives run on the mp communicator (RCCL over xGMI) with
``all_gather_into_tensor`` / ``reduce_scatter_tensor`` on contiguous
buffers, i.e. one RCCL call each, no per-rank list of tensors.
"""
import torch
import torch.distributed as dist

from . import topology as topo


def _grp():
    return topo.mp_group()  # None inside topology.serial_scope()


def _ws(g):
    return 1 if g is None else g.nranks


def _all_reduce(x, g):
    if _ws(g) > 1:
        if x.is_cuda:
            # small messages (decode, short sequences) take the one-shot IPC
            # kernel, large ones RCCL (parallel/comm.py)
            from .comm import get_communicator
            return get_communicator(g).all_reduce(x)
        dist.all_reduce(x, group=g.group)
    return x


def _all_gather(x, g, dim):
    n = _ws(g)
    if n == 1:
        return x
    x = x.contiguous()
    if dim == 0:
        out = torch.empty((x.shape[0] * n,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out, x, group=g.group)
        return out
    # gather along a later dim: gather on dim 0 of a moved view
    xm = x.movedim(dim, 0).contiguous()
    out = torch.empty((xm.shape[0] * n,) + tuple(xm.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, xm, group=g.group)
    return out.movedim(0, dim).contiguous()


def _reduce_scatter(x, g, dim=0):
    n = _ws(g)
    if n == 1:
        return x
    xm = x.movedim(dim, 0).contiguous() if dim != 0 else x.contiguous()
    assert xm.shape[0] % n == 0, "dim {} of size {} not divisible by {}".format(dim, xm.shape[0], n)
    out = torch.empty((xm.shape[0] // n,) + tuple(xm.shape[1:]), dtype=x.dtype, device=x.device)
    dist.reduce_scatter_tensor(out, xm, group=g.group)
    return out.movedim(0, dim).contiguous() if dim != 0 else out


def _split(x, g, dim):
    n = _ws(g)
    if n == 1:
        return x
    assert x.shape[dim] % n == 0, "dim {} of size {} not divisible by {}".format(dim, x.shape[dim], n)
    return x.chunk(n, dim=dim)[g.rank].contiguous()


class _CopyToMP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g):
        ctx.g = g
        return x

    @staticmethod
    def backward(ctx, dy):
        return _all_reduce(dy.contiguous(), ctx.g), None


class _ReduceFromMP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g):
        return _all_reduce(x.contiguous(), g)

    @staticmethod
    def backward(ctx, dy):
        return dy, None


class _GatherFromMP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g):
        ctx.g = g
        return _all_gather(x, g, x.dim() - 1)

    @staticmethod
    def backward(ctx, dy):
        return _split(dy, ctx.g, dy.dim() - 1), None


class _ScatterToMP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g):
        ctx.g = g
        return _split(x, g, x.dim() - 1)

    @staticmethod
    def backward(ctx, dy):
        return _all_gather(dy, ctx.g, dy.dim() - 1), None


class _ScatterToSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g):
        ctx.g = g
        return _split(x, g, 0)

    @staticmethod
    def backward(ctx, dy):
        return _all_gather(dy, ctx.g, 0), None


class _GatherFromSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g):
        ctx.g = g
        return _all_gather(x, g, 0)

    @staticmethod
    def backward(ctx, dy):
        return _split(dy, ctx.g, 0), None


class _AllGatherSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g):
        ctx.g = g
        return _all_gather(x, g, 0)

    @staticmethod
    def backward(ctx, dy):
        return _reduce_scatter(dy, ctx.g, 0), None


class _ReduceScatterSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g):
        ctx.g = g
        return _reduce_scatter(x, g, 0)

    @staticmethod
    def backward(ctx, dy):
        return _all_gather(dy, ctx.g, 0), None


def copy_to_mp(x, g=None):
    g = g or _grp()
    return x if _ws(g) == 1 else _CopyToMP.apply(x, g)


def reduce_from_mp(x, g=None):
    g = g or _grp()
    return x if _ws(g) == 1 else _ReduceFromMP.apply(x, g)


def gather_from_mp(x, g=None):
    g = g or _grp()
    return x if _ws(g) == 1 else _GatherFromMP.apply(x, g)


def scatter_to_mp(x, g=None):
    g = g or _grp()
    return x if _ws(g) == 1 else _ScatterToMP.apply(x, g)


def scatter_to_seq(x, g=None):
    g = g or _grp()
    return x if _ws(g) == 1 else _ScatterToSeq.apply(x, g)


def gather_from_seq(x, g=None):
    g = g or _grp()
    return x if _ws(g) == 1 else _GatherFromSeq.apply(x, g)


def all_gather_seq(x, g=None):
    g = g or _grp()
    return x if _ws(g) == 1 else _AllGatherSeq.apply(x, g)


def reduce_scatter_seq(x, g=None):
    g = g or _grp()
    return x if _ws(g) == 1 else _ReduceScatterSeq.apply(x, g)

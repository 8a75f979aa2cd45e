"""Activation recompute (checkpointing) that replays dropout exactly.

Parity: ``fleet.utils.recompute`` at reference ``single_model.py:243-244,
308-310,404-406`` / ``hybrid_model.py:332-333,406-408,537-539`` with the
three granularities ``full`` / ``full_attn`` / ``core_attn``
(``projects/gpt/docs/README.md:176``).

Because every dropout mask comes from a ``(stream, offset)`` key drawn from
:mod:`fleetx_amd.parallel.rng`, recompute only has to snapshot the tracker
state before the segment and restore it for the replay; no device generator
state is captured.
"""
import torch

from .rng import get_rng_state_tracker


class _Recompute(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fn, n_out_hint, *args):
        tracker = get_rng_state_tracker()
        ctx.fn = fn
        ctx.rng_before = tracker.get_states()
        ctx.cpu_rng = torch.get_rng_state()
        tensor_idx, tensors, others = [], [], []
        for i, a in enumerate(args):
            if torch.is_tensor(a):
                tensor_idx.append(i)
                tensors.append(a)
            others.append(a)
        ctx.tensor_idx = tensor_idx
        ctx.others = [None if torch.is_tensor(a) else a for a in others]
        ctx.save_for_backward(*tensors)
        with torch.no_grad():
            out = fn(*args)
        for o in (out if isinstance(out, tuple) else (out,)):
            if isinstance(o, torch.nn.Parameter):
                raise ValueError("recompute segments must not return parameters; "
                                 "return them outside the checkpointed function")
        ctx.rng_after = tracker.get_states()
        ctx.tuple_out = isinstance(out, tuple)
        return out

    @staticmethod
    def backward(ctx, *grads):
        tracker = get_rng_state_tracker()
        saved = ctx.saved_tensors
        args = list(ctx.others)
        for i, t in zip(ctx.tensor_idx, saved):
            d = t.detach()
            d.requires_grad_(t.requires_grad)
            args[i] = d
        after = tracker.get_states()
        cpu_now = torch.get_rng_state()
        tracker.set_states(ctx.rng_before)
        torch.set_rng_state(ctx.cpu_rng)
        try:
            with torch.enable_grad():
                out = ctx.fn(*args)
        finally:
            tracker.set_states(after)
            torch.set_rng_state(cpu_now)
        outs = out if isinstance(out, tuple) else (out,)
        pairs = [(o, g) for o, g in zip(outs, grads) if torch.is_tensor(o) and o.requires_grad
                 and g is not None]
        if pairs:
            torch.autograd.backward([p[0] for p in pairs], [p[1] for p in pairs])
        in_grads = []
        for a in args:
            in_grads.append(a.grad if torch.is_tensor(a) and a.requires_grad else None)
        return (None, None) + tuple(in_grads)


def recompute(fn, *args):
    """Run ``fn(*args)`` without storing activations; replay in backward."""
    if not torch.is_grad_enabled():
        return fn(*args)
    return _Recompute.apply(fn, 0, *args)

"""Fused top-k / top-p sampling (K18; csrc/kernels/sampling.hip).

One launch per decode step replaces softmax -> topk -> sort/cumsum/scatter ->
multinomial -> log_softmax/gather (reference ``single_model.py:907-988``).
The uniforms come from a torch generator so seeded generation is
reproducible; CPU tensors take the PyTorch reference path
(``generation.top_k_filter`` / ``top_p_filter`` + ``torch.multinomial``).
"""
import torch

from . import _lib


def fused_sample(logits, temperature=1.0, top_k=0, top_p=1.0, generator=None,
                 return_probs=False):
    """Sample one token per row of ``logits`` [B, V] (fp32 or bf16).

    Returns ``(ids int64 [B], lse fp32 [B])`` where ``lse`` is the logsumexp of
    the raw logits (the token log-prob is ``logits[ids] - lse``); with
    ``return_probs`` also the filtered, unnormalised probabilities [B, V]."""
    if logits.dim() != 2:
        raise ValueError("fused_sample expects [B, V] logits")
    B, V = logits.shape
    dev = logits.device
    if not logits.is_cuda:
        from ..models.language_model.gpt.generation import top_k_filter, top_p_filter
        lse = torch.logsumexp(logits.float(), -1)
        lg = logits.float() / temperature if temperature not in (None, 1.0) else logits.float()
        probs = torch.softmax(lg, -1)
        if top_k:
            probs = top_k_filter(probs, top_k)
        if top_p is not None and top_p < 1.0:
            probs = top_p_filter(probs, top_p)
        ids = torch.multinomial(probs, 1, generator=generator).squeeze(1)
        return (ids, lse, probs) if return_probs else (ids, lse)
    if logits.dtype == torch.float32:
        dc = 2
    elif logits.dtype == torch.bfloat16:
        dc = 0
    else:
        logits = logits.float()
        dc = 2
    if logits.stride(1) != 1:
        logits = logits.contiguous()
    u = torch.rand(B, device=dev, generator=generator)
    ids = torch.empty(B, device=dev, dtype=torch.int64)
    lse = torch.empty(B, device=dev, dtype=torch.float32)
    probs = torch.empty(B, V, device=dev, dtype=torch.float32) if return_probs else None
    inv_t = 1.0 / float(temperature) if temperature not in (None, 0.0) else 1.0
    rc = _lib.kernels().sample(dc, logits.data_ptr(), logits.stride(0), B, V, inv_t,
                               int(top_k or 0), float(1.0 if top_p is None else top_p),
                               u.data_ptr(), ids.data_ptr(), lse.data_ptr(), _lib.ptr(probs),
                               _lib.stream())
    if rc != 0:
        raise RuntimeError("fused sampling launch failed ({})".format(rc))
    _lib.maybe_sync()
    return (ids, lse, probs) if return_probs else (ids, lse)

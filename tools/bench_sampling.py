"""Decode-step sampling cost: fused HIP top-k/top-p kernel vs the PyTorch op
chain (softmax, topk, sort/cumsum/scatter, multinomial, log_softmax).

    python tools/bench_sampling.py [--batch 8 --vocab 50304]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--vocab", type=int, default=50304)
    a = ap.parse_args()
    from fleetx_amd.ops import fused_sample
    from fleetx_amd.models.language_model.gpt.generation import top_k_filter, top_p_filter
    lg = torch.randn(a.batch, a.vocab, device="cuda") * 3

    def chain():
        logp = torch.log_softmax(lg, -1)
        probs = top_p_filter(top_k_filter(torch.softmax(lg / 0.8, -1), 40), 0.9)
        nxt = torch.multinomial(probs, 1).squeeze(1)
        return logp.gather(1, nxt[:, None])

    def fused():
        nxt, lse = fused_sample(lg, 0.8, 40, 0.9)
        return lg.gather(1, nxt[:, None]).squeeze(1) - lse

    print(json.dumps({"batch": a.batch, "vocab": a.vocab, "torch_chain_us": round(timeit(chain), 1),
                      "fused_us": round(timeit(fused), 1)}))


if __name__ == "__main__":
    main()

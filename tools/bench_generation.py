"""Decode throughput of GPT generation (greedy, HIP-graph replay) with and
without the fused decode layer (K19: weight-streaming GEMVs with sub-layer
epilogues).  Random-init weights, bf16.

    python tools/bench_generation.py [--model gpt3-1.3B] [--batch 1 8 16] [--tokens 64]

One JSON line per (batch, fused): ms/token, tokens/s and the effective weight
stream rate (parameter bytes / ms per token)."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

MODELS = {"gpt-345M": (1024, 24, 16), "gpt3-1.3B": (2048, 24, 16), "gpt3-6.7B": (4096, 32, 32)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt3-1.3B", choices=sorted(MODELS))
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 8, 16])
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--tokens", type=int, default=64)
    ap.add_argument("--fused-only", action="store_true")
    args = ap.parse_args()
    from fleetx_amd.models.language_model.gpt.model import GPTConfig, GPTForPretraining
    from fleetx_amd.models.language_model.gpt.generation import GPTForGeneration
    h, L, a = MODELS[args.model]
    cfg = GPTConfig(vocab_size=50304, hidden_size=h, num_layers=L, num_attention_heads=a,
                    max_position_embeddings=1024, hidden_dropout_prob=0.0,
                    attention_probs_dropout_prob=0.0, dtype=torch.bfloat16)
    model = GPTForPretraining(cfg).cuda().eval()
    nbytes = sum(p.numel() * p.element_size() for p in model.parameters())
    for B in args.batch:
        prompt = torch.randint(0, 50304, (B, args.prompt), device="cuda")
        for fused in ((True,) if args.fused_only else (False, True)):
            gen = GPTForGeneration(model, {"max_dec_len": args.tokens, "fused_decode": fused,
                                           "decode_strategy": "greedy_search"})
            gen.generate(prompt, max_length=8)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            gen.generate(prompt, max_length=1)
            torch.cuda.synchronize()
            t_pre = time.perf_counter() - t0
            t0 = time.perf_counter()
            ids, _ = gen.generate(prompt)
            torch.cuda.synchronize()
            t = time.perf_counter() - t0
            ms = 1e3 * (t - t_pre) / max(1, ids.shape[1] - 1)
            persistent = fused and B <= 4 and \
                os.environ.get("FLEETX_DECODE_PERSISTENT", "0") == "1"
            print(json.dumps({"model": args.model, "batch": B, "fused_decode": fused,
                              "persistent_layers": persistent,
                              "ms_per_token": round(ms, 3),
                              "tokens_per_s": round(B * 1e3 / ms, 1),
                              "weight_TB_s": round(nbytes / (ms * 1e-3) / 1e12, 2)}), flush=True)


if __name__ == "__main__":
    main()

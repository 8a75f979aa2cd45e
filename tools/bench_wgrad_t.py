"""16-bit weight gradient of GPT-3 6.7B's FC2 (dW[4096, 16384] over 8192
tokens) in the plain order and through the transposed product with the
transposed store (ops/gemm.py linear_wgrad, FLEETX_GEMM_WGRAD_T), interleaved."""
import json
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
import torch  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    from fleetx_amd.ops import gemm as G
    G.load_plan()
    for T, N, K in ((8192, 4096, 16384), (8192, 2048, 8192), (8192, 1024, 4096)):
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        sq = torch.zeros(G.sq_slots(N, K), device="cuda", dtype=torch.float32)
        fl = 2.0 * T * N * K
        res = {}
        for r in range(2):
            for on in (False, True):
                G.WGRAD_T = on
                ms = timeit(lambda: G.linear_wgrad(dy, x, out, False, sq=sq))
                res.setdefault("T" if on else "plain", []).append(round(fl / ms / 1e9, 1))
        print(json.dumps({"tokens": T, "N": N, "K": K, "TF": res}), flush=True)


if __name__ == "__main__":
    main()

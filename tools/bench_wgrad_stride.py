"""Weight-gradient GEMM of the FC2 shape with the activation's row stride
padded off the power of two (channel-conflict probe): dW[4096, 16384] = dy^T x
over 8192 tokens, x rows 16384 (32 KiB) vs 16384 + pad elements apart."""
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
    M, N, K = 8192, 4096, 16384
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    dw = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * M * N * K
    for pad in (0, 64, 128, 256):
        xb = torch.randn(M, K + pad, device="cuda", dtype=torch.bfloat16)
        x = xb[:, :K]
        ms = timeit(lambda: G.linear_wgrad(dy, x, dw, False))
        # and the FC1-like transpose of roles: dW[16384, 4096] = dy'^T x' (dy' rows 16384 + pad)
        dyb = torch.randn(M, K + pad, device="cuda", dtype=torch.bfloat16)
        x2 = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        dw2 = torch.empty(K, N, device="cuda", dtype=torch.bfloat16)
        ms2 = timeit(lambda: G.linear_wgrad(dyb[:, :K], x2, dw2, False))
        print(json.dumps({"pad": pad, "fc2_like_TF": round(fl / ms / 1e9, 1),
                          "fc1_like_TF": round(fl / ms2 / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()

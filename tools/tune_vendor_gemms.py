"""Add TunableOp picks for the vendor GEMMs of the BASELINE config-3 layouts
(GPT-3 6.7B with TP2: N = 2 at micro-batch 8, N = 4 / 8 at micro-batch 4) to
fleetx_amd/ops/tunableop_gfx950.csv.  Those runs need several GPUs, so the
per-rank GEMMs are issued here in the exact form the TP layers use
(F.linear, with the bias for the column-parallel QKV / FC1), one process,
tuning on.  Run with PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1
PYTORCH_TUNABLEOP_FILENAME=<file>: the file's existing rows are read first and
written back with the new ones."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main():
    h, tp, vocab = 4096, 2, 50304
    bf = torch.bfloat16
    for M in (8192, 4096):
        x = torch.randn(M, h, device="cuda", dtype=bf)
        for out, inp, bias in ((3 * h // tp, h, True), (4 * h // tp, h, True),
                               (h, h // tp, False), (h, 4 * h // tp, False),
                               (vocab // tp, h, False)):
            a = torch.randn(M, inp, device="cuda", dtype=bf) if inp != h else x
            w = torch.randn(out, inp, device="cuda", dtype=bf) * 0.02
            b = torch.randn(out, device="cuda", dtype=bf) if bias else None
            F.linear(a, w, b)
            if out == vocab // tp:  # LM head data gradient: F.linear(dlogits, W^T)
                F.linear(torch.randn(M, out, device="cuda", dtype=bf), w.t().contiguous())
        torch.cuda.synchronize()
        print("tuned M =", M, flush=True)


if __name__ == "__main__":
    main()

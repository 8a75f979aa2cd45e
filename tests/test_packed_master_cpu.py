"""The packed-master encoding (``loss_optim_embed.hip`` ``pk_encode`` /
``pk_decode``, mirrored here in integer torch ops): hi = x's high 16 bits
rounded to nearest on the low half (ties toward zero), lo = x's low 16 bits,
x = ((hi - (lo > 0x8000)) << 16) | lo.  Lossless for every finite fp32 value,
and hi is the round-to-nearest-even bf16 cast except at exact ties.  The
kernels themselves are checked on the GPU (tests/test_packed_master_gpu.py)."""
import torch


def _encode(x):
    b = x.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    lo = b & 0xFFFF
    hi = ((b >> 16) + (lo > 0x8000).to(torch.int64)) & 0xFFFF
    return hi, lo


def _decode(hi, lo):
    top = (hi - (lo > 0x8000).to(torch.int64)) & 0xFFFF
    b = (top << 16) | lo
    b = torch.where(b >= 2 ** 31, b - 2 ** 32, b)
    return b.to(torch.int32).view(torch.float32)


def test_encoding_is_lossless_and_round_to_nearest():
    g = torch.Generator().manual_seed(0)
    bits = torch.randint(-2 ** 31, 2 ** 31 - 1, (1 << 20,), generator=g, dtype=torch.int64)
    x = bits.to(torch.int32).view(torch.float32)
    x = x[torch.isfinite(x)]
    x = torch.cat([x, torch.tensor([0.0, -0.0, 1.0, -1.0, 1e-40, -3e38])])
    hi, lo = _encode(x)
    assert torch.equal(_decode(hi, lo).view(torch.int32), x.view(torch.int32))
    rne = x.to(torch.bfloat16).view(torch.int16).to(torch.int64) & 0xFFFF
    tie = lo == 0x8000
    finite = torch.isfinite(x.to(torch.bfloat16))
    ok = ~tie & finite
    assert torch.equal(hi[ok], rne[ok])
    # ties round toward zero: the high half unchanged
    b = x.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    assert torch.equal(hi[tie], (b[tie] >> 16) & 0xFFFF)

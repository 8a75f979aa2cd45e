"""CPU checks of the fused-softmax op API (the GPU kernels are in test_kernels_gpu.py)."""
import pytest
import torch

from fleetx_amd.ops.softmax import (_mask_div, softmax_mask_fuse,
                                    softmax_mask_fuse_upper_triangle)


def test_upper_triangle_matches_masked_softmax():
    x = torch.randn(2, 3, 16, 16)
    y = softmax_mask_fuse_upper_triangle(x)
    tri = torch.triu(torch.ones(16, 16, dtype=torch.bool), 1)
    assert torch.allclose(y, torch.softmax(x.masked_fill(tri, float("-inf")), -1))
    assert torch.allclose(y.sum(-1), torch.ones(2, 3, 16))


def test_additive_mask_and_fully_masked_rows():
    x = torch.randn(2, 2, 4, 8)
    mask = torch.zeros(2, 1, 4, 8)
    mask[:, :, 1] = float("-inf")
    y = softmax_mask_fuse(x, mask)
    assert (y[:, :, 1] == 0).all()
    assert torch.allclose(y[:, :, 0], torch.softmax(x[:, :, 0], -1))


def test_mask_row_divisor():
    x = torch.empty(2, 4, 8, 8)
    assert _mask_div(x, torch.empty(2, 1, 8, 8)) == 4
    assert _mask_div(x, torch.empty(1, 1, 8, 8)) == 8
    assert _mask_div(x, torch.empty(8, 8)) == 8
    assert _mask_div(x, torch.empty(2, 4, 8, 8)) == 1
    with pytest.raises(ValueError):
        _mask_div(x, torch.empty(1, 4, 8, 8))


def test_debug_modes(monkeypatch):
    import os
    from fleetx_amd.utils import env
    from fleetx_amd.utils.config import AttrDict
    monkeypatch.delenv("FLEETX_DETERMINISTIC", raising=False)
    cfg = AttrDict({"Global": AttrDict({"deterministic": True, "kernel_sync": False})})
    try:
        env.set_debug_modes(cfg)
        assert os.environ["FLEETX_DETERMINISTIC"] == "1"
        assert torch.are_deterministic_algorithms_enabled()
    finally:
        torch.use_deterministic_algorithms(False)
        os.environ.pop("FLEETX_DETERMINISTIC", None)

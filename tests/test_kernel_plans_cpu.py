"""Host-side launch plans of the HIP kernels, checked on the CPU (the plan
code runs without a GPU; the CU count falls back to MI355X's 256):

* gemm5 geometry / split-K for fp32 weight gradients (csrc/kernels/gemm5.hip
  ``g5_f32_nf`` + ``g5_split_plan``): 256-tiles cut into <= 4 slices for
  48-128 of them, 128-tile grids under 384 tiles cut to about one workgroup
  per CU, otherwise only a last wave at most a quarter full is split; the
  slab workspace is tiles x S slices x TILE^2 fp32;
* the one-pass LayerNorm backward (csrc/kernels/norm_eltwise.hip
  ``fx_ln_bwd_cols_blocks``): covered widths and partial-row counts."""
import os

import pytest

EPI_F32 = 3


def _k():
    try:
        from fleetx_amd._C import _kernels
    except ImportError:
        pytest.skip("HIP kernel library not built")
    if os.environ.get("FLEETX_GEMM_PF", "5") != "5" or os.environ.get("FLEETX_GEMM5_SPLITK", "1") == "0":
        pytest.skip("split-K plan pinned off by the environment")
    return _kernels


def test_splitk_plan():
    k = _k()
    # 528 128-tiles on 512 slots (short K: 256 K-tiles is the ViT rule below) -> 16 tiles x 32 slices
    assert k.gemm_ws_bytes(EPI_F32, 6144, 1408, 8192) == 16 * 32 * 128 * 128 * 4
    # ViT-g out-proj: 121 128-tiles -> round(256 / 121) = 2 slices
    assert k.gemm_ws_bytes(EPI_F32, 1408, 1408, 16448) == 121 * 2 * 128 * 128 * 4
    # 345M out-proj: 64 128-tiles -> 4 slices
    assert k.gemm_ws_bytes(EPI_F32, 1024, 1024, 8192) == 64 * 4 * 128 * 128 * 4
    # 345M QKV (48 256-tiles) -> 256-tiles in 4 slices; ViT-g QKV (102) -> 2
    assert k.gemm_ws_bytes(EPI_F32, 3072, 1024, 8192) == 48 * 4 * 256 * 256 * 4
    assert k.gemm_ws_bytes(EPI_F32, 4224, 1408, 8192) == 102 * 2 * 256 * 256 * 4
    # whole waves (6.7B: 256-tiles fill 256 slots) never split
    assert k.gemm_ws_bytes(EPI_F32, 4096, 4096, 8192) == 0
    assert k.gemm_ws_bytes(EPI_F32, 12288, 4096, 8192) == 0
    # 129-191 256-tiles: 128-tiles, unsplit at >= 384 of them (ViT-g FC1 at 8192 tokens) ...
    assert k.gemm_ws_bytes(EPI_F32, 5632, 1408, 8192) == 0
    # ... but 256-tiles in 3 slices over >= 192 K-tiles (ViT-g FC1 / FC2 at 16448 tokens)
    assert k.gemm_ws_bytes(EPI_F32, 6144, 1408, 16448) == 144 * 3 * 256 * 256 * 4
    assert k.gemm_ws_bytes(EPI_F32, 1408, 6144, 16448) == 144 * 3 * 256 * 256 * 4
    # short K: at least 8 K-tiles per slice
    assert k.gemm_ws_bytes(EPI_F32, 1024, 1024, 256) == 0
    # only the fp32 weight-gradient epilogue splits
    assert k.gemm_ws_bytes(0, 6144, 1408, 16448) == 0


def test_ln_bwd_cols_plan():
    k = _k()
    assert k.ln_bwd_cols_blocks(8192, 1024, 1536) == 512      # one wave per row, 4 rows per wave
    assert k.ln_bwd_cols_blocks(16448, 1408, 1536) > 0       # masked width (ViT-g)
    assert k.ln_bwd_cols_blocks(8192, 2048, 1536) == 0       # default limit: h <= 1536
    assert k.ln_bwd_cols_blocks(8192, 4096, 4096) == 512     # 4 waves per row when enabled
    assert k.ln_bwd_cols_blocks(8192, 4104, 4096) == 0       # wider than 4096
    assert k.ln_bwd_cols_blocks(8192, 1000, 1536) > 0        # h % 8 == 0 is enough at one wave
    assert k.ln_bwd_cols_blocks(3, 1024, 1536) == 1
    assert k.ln_bwd_cols_blocks(0, 1024, 1536) == 0

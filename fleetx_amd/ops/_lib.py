"""Loader for the in-tree HIP kernel library.

GPU tensors ALWAYS go through the HIP kernels: if the extension is missing
on a GPU box the op raises (no silent eager fallback).  CPU tensors use the
PyTorch reference math in each op module (same RNG hash, same formulas) --
that path exists for the CPU test-suite and the CPU float32 plumbing config.
"""
import os

import torch

_K = None
_ERR = None


def kernels():
    """Return the ``_kernels`` module or raise with the build hint."""
    global _K, _ERR
    if _K is not None:
        return _K
    try:
        lab = os.environ.get("FLEETX_KERNELS_LIB")
        if lab:
            # a lab build of the same library (tools/fa_lab/build.py)
            import importlib.util
            spec = importlib.util.spec_from_file_location("_kernels", lab)
            k = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(k)
        else:
            from .._C import _kernels as k  # noqa: WPS433
        _K = k
        return k
    except ImportError as e:  # pragma: no cover - exercised on broken installs
        _ERR = e
        raise RuntimeError(
            "FleetX-AMD HIP kernels are not built ({}). Run `python -m fleetx_amd._build` "
            "(hipcc --offload-arch=gfx950).".format(e)) from e


def available():
    try:
        kernels()
        return True
    except RuntimeError:
        return False


def dt_code(dtype):
    if dtype == torch.bfloat16:
        return 0
    if dtype == torch.float16:
        return 1
    raise NotImplementedError(
        "HIP kernels take bf16/fp16 tensors (got {}); train with mix_precision "
        "dtype bfloat16 or float16 on MI355X".format(dtype))


def stream():
    return torch.cuda.current_stream().cuda_stream


def ptr(t):
    return 0 if t is None else t.data_ptr()


def on_gpu(t):
    return t is not None and t.is_cuda


def check_contig(*ts):
    for t in ts:
        if t is not None and not t.is_contiguous():
            raise ValueError("expected a contiguous tensor")


DEBUG_SYNC = os.environ.get("FLEETX_KERNEL_SYNC", "0") == "1"


def maybe_sync():
    """``FLEETX_KERNEL_SYNC=1`` serialises after each launch (debug aid)."""
    if DEBUG_SYNC:
        torch.cuda.synchronize()

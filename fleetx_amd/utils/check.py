"""Environment checks (reference ``ppfleetx/utils/check.py:29-54`` and
``ppfleetx/utils/version.py:18-21``).

* :func:`check_gpu` -- the reference exits when Paddle was built without CUDA;
  here: PyTorch must be a ROCm build, a GPU must be visible, and (optionally)
  it must be gfx950 (MI355X), the only target the HIP kernels are built for;
* :func:`version_check` -- minimum PyTorch version (the RCCL collective forms
  used: ``all_gather_into_tensor`` / ``reduce_scatter_tensor`` /
  ``batch_isend_irecv``) and that the in-tree HIP extension matches the GPU.
Both log an error and ``sys.exit(1)`` like the reference (``exit=False``
raises instead, for library use).
"""
import sys

import torch

from .log import logger

MIN_TORCH = (2, 1)


def _fail(msg, exit):
    if exit:
        logger.error(msg)
        sys.exit(1)
    raise RuntimeError(msg)


def gpu_arch(device=0):
    props = torch.cuda.get_device_properties(device)
    return getattr(props, "gcnArchName", "") or ""


def check_gpu(require_gfx950=True, exit=True):
    if getattr(torch.version, "hip", None) is None:
        return _fail("PyTorch is not a ROCm build (torch.version.hip is None): "
                     "install the ROCm PyTorch to run on MI355X", exit)
    if not torch.cuda.is_available():
        return _fail("no AMD GPU is visible (HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES?)", exit)
    arch = gpu_arch()
    if require_gfx950 and not arch.startswith("gfx950"):
        return _fail("GPU architecture {!r}: the HIP kernels are built for gfx950 (MI355X)"
                     .format(arch), exit)
    return arch


def _ver(s):
    out = []
    for part in s.split("+")[0].split(".")[:2]:
        digits = "".join(ch for ch in part if ch.isdigit())
        out.append(int(digits or 0))
    return tuple(out)


def version_check(exit=True):
    v = _ver(torch.__version__)
    if v < MIN_TORCH:
        return _fail("PyTorch {} found; {}.{} or newer is required".format(
            torch.__version__, *MIN_TORCH), exit)
    for name in ("all_gather_into_tensor", "reduce_scatter_tensor", "batch_isend_irecv"):
        if not hasattr(torch.distributed, name):
            return _fail("torch.distributed.{} is missing".format(name), exit)
    return torch.__version__


check_version = version_check

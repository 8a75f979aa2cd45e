"""Process environment: seeding, distributed init, data-world geometry.

Parity: reference ``ppfleetx/utils/env.py:27-96`` (``set_seed``,
``init_dist_env``, ``get_local_rank``, ``get_data_world_size/rank``).
"""
import os
import random

import numpy as np
import torch

from ..parallel import topology as topo
from ..parallel.rng import model_parallel_random_seed


def get_local_rank():
    return int(os.environ.get("LOCAL_RANK", os.environ.get("PADDLE_RANK_IN_NODE", "0")))


def get_rank():
    return int(os.environ.get("RANK", "0"))


def get_world_size():
    return int(os.environ.get("WORLD_SIZE", "1"))


# Process-wide RCCL environment (Distributed.comm.rccl_env; the process
# environment always wins).  An 8-GPU MI355X node is a fully connected xGMI
# mesh (7 point-to-point links per GPU): a bandwidth-optimal collective needs
# enough channels that every link carries one, so the channel floor is
# raised to 32 for every communicator.  Per-communicator budgets
# (Distributed.comm.ctas, parallel/topology.py DEFAULT_CTAS) are opt-in until
# tools/bench_collectives.py --ctas has measured them on a node.
DEFAULT_RCCL_ENV = {"NCCL_MIN_NCHANNELS": "32"}


def apply_rccl_env(config=None):
    """Export the RCCL environment before the process group is created;
    returns the settings in effect."""
    env = dict(DEFAULT_RCCL_ENV)
    if config is not None:
        comm = (config.get("Distributed", {}) or {}).get("comm", {}) or {}
        extra = comm.get("rccl_env", None)
        if extra is False:  # Distributed.comm.rccl_env: False -> RCCL defaults
            env = {}
        elif extra:
            env.update({str(k): str(v) for k, v in dict(extra).items()})
    for k, v in env.items():
        os.environ.setdefault(k, v)
    return {k: os.environ[k] for k in env}


def init_dist_env(config, backend=None):
    """Create the process group and the hybrid topology from ``Distributed``."""
    set_debug_modes(config)
    d = config.Distributed
    # collective debugging (new vs. the reference): "fingerprint"
    # cross-checks every collective's op / sequence number / shape / dtype over
    # gloo mirrors and names the diverging rank; "detail" / "info" additionally
    # turn on torch's TORCH_DISTRIBUTED_DEBUG checks.
    dbg = str(d.get("debug", os.environ.get("FLEETX_COLLECTIVE_CHECK", "off")) or "off").lower()
    if dbg in ("1", "detail", "on", "true"):
        os.environ.setdefault("TORCH_DISTRIBUTED_DEBUG", "DETAIL")
    elif dbg == "info":
        os.environ.setdefault("TORCH_DISTRIBUTED_DEBUG", "INFO")
    _check_env(config)
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        apply_rccl_env(config)
    topo.init_distributed(backend=backend, timeout_s=int(d.get("timeout_s", 1800) or 1800))
    comm = d.get("comm", {}) or {}
    hcg = topo.init_hcg(dp=d.dp_degree, mp=d.mp_degree, pp=d.pp_degree,
                        sharding=d.sharding.sharding_degree,
                        pp_split_directions=bool(comm.get("pp_split_directions", False)),
                        ctas=comm.get("ctas", None))
    if dbg == "fingerprint":
        # per-collective op / sequence / shape / dtype cross-check over gloo
        # mirrors of every group (parallel/collective_check.py)
        from ..parallel import collective_check
        collective_check.enable(hcg)
    return hcg


def _check_env(config):
    """Reference ``config.py:242-245``: version check always, GPU check when
    ``Global.device`` is gpu (a missing GPU is reported, then the run falls
    back to CPU as ``env.device()`` does; a non-gfx950 GPU is reported)."""
    from . import check
    from .log import logger
    check.version_check(exit=False)
    if str((config.get("Global", {}) or {}).get("device", "gpu")).lower() in ("gpu", "cuda"):
        try:
            arch = check.check_gpu(require_gfx950=False, exit=False)
            if not str(arch).startswith("gfx950"):
                logger.warning("GPU %s is not gfx950 (MI355X): the HIP kernels will not load", arch)
        except RuntimeError as e:
            logger.warning("%s -- running on CPU", e)


def get_data_world_size():
    hcg = topo.get_hcg()
    return hcg.dp_degree * hcg.sharding_degree


def get_data_world_rank():
    hcg = topo.get_hcg()
    return hcg.dp_rank * hcg.sharding_degree + hcg.sharding_rank


def set_seed(seed):
    """Seed host RNGs with ``seed + data_rank`` and the dropout tracker."""
    hcg = topo.get_hcg()
    data_rank = get_data_world_rank()
    s = seed + data_rank
    random.seed(s)
    np.random.seed(s % (2 ** 32))
    torch.manual_seed(s)
    model_parallel_random_seed(seed, mp_rank=hcg.mp_rank, pp_rank=hcg.pp_rank,
                               data_rank=data_rank)
    # parameter-init seed for mp-sharded weights (reference env.py:67)
    return s


def set_debug_modes(config):
    """Debug / reproducibility switches (new vs. the reference):

    * ``Global.deterministic``: ``torch.use_deterministic_algorithms`` plus
      this framework's deterministic kernels (sorted-segment embedding
      backward instead of fp32 atomics) -- bitwise-reproducible steps for
      golden tests;
    * ``Global.kernel_sync``: synchronise after every HIP kernel launch of
      ours (``FLEETX_KERNEL_SYNC``) and serialise HIP launches
      (``AMD_SERIALIZE_KERNEL=3``), so a faulting kernel is reported at its
      own launch.  Both are read at process start, so they are set before
      the first kernel is loaded."""
    g = config.get("Global", {}) or {}
    if g.get("deterministic", False):
        os.environ["FLEETX_DETERMINISTIC"] = "1"
        torch.use_deterministic_algorithms(True, warn_only=True)
    if g.get("kernel_sync", False):
        os.environ.setdefault("AMD_SERIALIZE_KERNEL", "3")
        os.environ["FLEETX_KERNEL_SYNC"] = "1"
        from ..ops import _lib
        _lib.DEBUG_SYNC = True


def device():
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")

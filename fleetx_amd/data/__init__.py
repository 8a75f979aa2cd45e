"""Dataset / sampler / loader factory (reference ``ppfleetx/data/__init__.py:25-73``).

Names resolve through registries; the loader is ``torch.utils.data.DataLoader``
with a batch sampler and pinned host memory so the per-step H2D copy is async.
"""
import copy

import torch

from ..utils.log import logger
from .dataset import DATASETS
from .sampler import SAMPLERS
from .utils import COLLATE_FNS

__all__ = ["build_dataset", "build_dataloader"]


def build_dataset(config, mode):
    assert mode in ("Train", "Eval", "Test"), "Dataset mode should be Train, Eval, Test"
    if mode not in config or config[mode] is None:
        return None
    cfg = dict(copy.deepcopy(config[mode].dataset))
    name = cfg.pop("name")
    if name not in DATASETS:
        raise ValueError("unknown dataset {}".format(name))
    ds = DATASETS[name](**cfg)
    logger.debug("build dataset({}) success...".format(name))
    return ds


def build_dataloader(config, mode):
    if mode not in config or config[mode] is None:
        return None
    dataset = build_dataset(config, mode)
    batch_sampler = None
    if "sampler" in config[mode] and config[mode].sampler is not None:
        scfg = dict(copy.deepcopy(config[mode].sampler))
        sname = scfg.pop("name", "GPTBatchSampler")
        batch_sampler = SAMPLERS[sname](dataset, **scfg)
    collate = None
    lcfg = {}
    if "loader" in config[mode] and config[mode].loader is not None:
        lcfg = dict(copy.deepcopy(config[mode].loader))
        cname = lcfg.pop("collate_fn", None)
        collate = COLLATE_FNS[cname] if cname else None
    # Paddle-only loader keys
    for k in ("return_list", "use_shared_memory"):
        lcfg.pop(k, None)
    nw = int(lcfg.pop("num_workers", 0) or 0)
    kwargs = dict(num_workers=nw, collate_fn=collate,
                  pin_memory=torch.cuda.is_available())
    if nw > 0:
        kwargs["persistent_workers"] = True
        kwargs["prefetch_factor"] = 4
    if batch_sampler is not None:
        return torch.utils.data.DataLoader(dataset, batch_sampler=batch_sampler, **kwargs)
    return torch.utils.data.DataLoader(dataset, batch_size=lcfg.pop("batch_size", 1),
                                       shuffle=lcfg.pop("shuffle", False),
                                       drop_last=lcfg.pop("drop_last", False), **kwargs)

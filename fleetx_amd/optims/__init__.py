"""Optimizer / LR-scheduler builders (reference ``ppfleetx/optims/__init__.py:29-62``).

Names are resolved through registries instead of ``eval``.
"""
import copy

from .lr_scheduler import SCHEDULERS, LRScheduler  # noqa: F401
from .lr_scheduler import CosineAnnealingWithWarmupDecay, ViTLRScheduler  # noqa: F401
from .optimizer import OPTIMIZERS, CLIPS, FusedAdamW, AdamW, Adam, Momentum  # noqa: F401
from .optimizer import ClipGradByGlobalNorm  # noqa: F401
from ..utils.log import logger


def build_lr_scheduler(lr_config):
    cfg = dict(copy.deepcopy(lr_config))
    if "name" in cfg:
        name = cfg.pop("name")
        if name not in SCHEDULERS:
            raise ValueError("unknown lr scheduler {}".format(name))
        lr = SCHEDULERS[name](**cfg)
    else:
        lr = float(cfg.get("learning_rate", 1e-4))
    logger.debug("build lr ({}) success..".format(lr))
    return lr


def build_optimizer(config, buffer, lr_scheduler=None, **groups):
    """``buffer``: the model's FlatParamGradBuffer; ``groups``: mp/pp groups
    for the global-norm reduction."""
    cfg = dict(copy.deepcopy(config))
    lr_cfg = cfg.pop("lr", None)
    if lr_scheduler is None:
        lr_scheduler = build_lr_scheduler(lr_cfg) if lr_cfg is not None else 1e-4
    clip = None
    clip_cfg = cfg.pop("grad_clip", None)
    if clip_cfg is not None:
        clip_cfg = dict(clip_cfg)
        clip = CLIPS[clip_cfg.pop("name", "ClipGradByGlobalNorm")](**clip_cfg)
    name = cfg.pop("name")
    if name not in OPTIMIZERS:
        raise ValueError("unknown optimizer {}".format(name))
    cfg.update(groups)
    opt = OPTIMIZERS[name](learning_rate=lr_scheduler, buffer=buffer, grad_clip=clip, **cfg)
    logger.debug("build optimizer ({}) success..".format(type(opt).__name__))
    return opt

"""Auto-parallel engine.

Parity: reference ``core/engine/auto_engine.py:36-132`` (C16): constructed
from the config's ``Engine.strategy`` (built by ``get_auto_config``), ``fit``
/ ``evaluate`` / ``predict`` take *datasets* and batch them itself with
``batch_size = global_batch_size`` split over the data-parallel ranks,
``steps_per_epoch = max_steps``, ``valid_freq`` / ``valid_steps`` and the
``Data.collate_fn``; ``Data.sample_split`` is the number of leading sample
fields that are model inputs (the rest are labels); save / load use
``<dir>/auto``.

Execution: the strategy's degrees (given in the YAML for ``auto_mode: semi``,
or searched by :mod:`fleetx_amd.parallel.auto.planner` for ``auto_mode:
full``) drive the same hybrid runtime as the eager engine (TP layers, 1F1B,
flat-buffer DP/ZeRO, recompute, bf16 with fp32 master weights).
"""
import os

import torch

from ...data.utils import COLLATE_FNS as _COLLATE
from ...data.sampler import DistributedBatchSampler
from ...utils import env
from ...utils.log import logger
from ..module.basic_module import BasicModule
from .basic_engine import BasicEngine
from .eager_engine import EagerEngine


class AutoEngine(BasicEngine):
    def __init__(self, configs, module, optimizer=None, lr=None, mode="train"):
        super().__init__()
        if not isinstance(module, BasicModule):
            raise TypeError("'module' must be a BasicModule, got {}".format(type(module).__name__))
        if mode == "train" and module.loss_fn is not None and not callable(module.loss_fn):
            raise TypeError("'loss_fn' must be callable")
        self.mode = mode
        self._module = module
        self._cfg = configs
        e = configs.Engine
        self._max_steps = e.max_steps
        self._eval_freq = e.get("eval_freq", 1) or 1
        self._eval_iters = e.get("eval_iters", 10)
        self._test_iters = e.get("test_iters", 100)
        self._num_train_epochs = e.get("num_train_epochs", 1)
        self._strategy = e.get("strategy")
        sl = e.get("save_load", {}) or {}
        self._output_dir = sl.get("output_dir", "./output")
        self._ckpt_dir = sl.get("ckpt_dir")
        data = configs.get("Data", {}) or {}
        name = data.get("collate_fn")
        self.collate_fn = _COLLATE[name] if name else None
        self.sample_split = data.get("sample_split")
        self.batch_size = configs.Global.global_batch_size
        self._engine = EagerEngine(configs=configs, module=module, optimizer=optimizer, lr=lr,
                                   mode=mode)

    # ------------------------------------------------------------------ data
    def _loader(self, dataset):
        if dataset is None:
            return None
        nrep = env.get_data_world_size()
        sampler = DistributedBatchSampler(dataset, batch_size=self.batch_size // nrep,
                                          num_replicas=nrep, rank=env.get_data_world_rank(),
                                          shuffle=False, drop_last=True)
        return torch.utils.data.DataLoader(dataset, batch_sampler=sampler,
                                           collate_fn=self.collate_fn,
                                           pin_memory=torch.cuda.is_available())

    def _check_split(self, loader):
        if self.sample_split is None or loader is None:
            return
        first = next(iter(loader))
        if not 0 < self.sample_split < len(first):
            raise ValueError("sample_split={} but samples have {} fields".format(
                self.sample_split, len(first)))

    # ------------------------------------------------------------------ api
    def fit(self, epoch=1, train_dataset=None, valid_dataset=None):
        train = self._loader(train_dataset)
        valid = self._loader(valid_dataset)
        self._check_split(train)
        if self._strategy is not None:
            logger.info("auto strategy: %s" % dict(self._strategy))
        return self._engine.fit(epoch=epoch or self._num_train_epochs, train_data_loader=train,
                                valid_data_loader=valid)

    def evaluate(self, valid_dataset=None):
        return self._engine.evaluate(valid_data_loader=self._loader(valid_dataset))

    def predict(self, test_dataset=None):
        return self._engine.predict(test_data_loader=self._loader(test_dataset))

    def save(self, training=True, epoch=0, step=0):
        if not (self._output_dir and isinstance(self._output_dir, str)):
            raise TypeError("`save` requires a valid value of `output_dir`.")
        saved = self._engine._output_dir
        self._engine._output_dir = os.path.join(self._output_dir, "auto")
        try:
            opt = self._engine.optimizer
            if not training:
                self._engine.optimizer = None
            self._engine.save(epoch=epoch, step=step)
        finally:
            self._engine.optimizer = opt
            self._engine._output_dir = saved

    def load(self):
        if not (self._ckpt_dir and isinstance(self._ckpt_dir, str)):
            logger.warning("`load` requires a valid value of `ckpt_dir`.")
            return
        from ...utils import checkpoint as ckpt
        base = os.path.join(self._ckpt_dir, "auto")
        latest = ckpt.latest_checkpoint(base) or base
        self._engine.load(ckpt_dir=latest)

    @property
    def engine(self):
        return self._engine

"""Image-classification task module.

Parity: reference ``models/vision_model/general_classification_module.py:30-169``
(C22): model / loss / metric built by name from the ``Model`` config
(``model.name`` is a ViT preset), ``training_step`` -> loss,
``validation_step`` all-gathers logits and labels over the data-parallel world
before the top-k metric, epoch-end metric averaging with ``best_metric``
tracking, and images/sec in the log lines.
"""
import copy
from collections import defaultdict

import numpy as np
import torch
import torch.distributed as dist

from ...core.module.basic_module import BasicModule
from ...utils import env
from ...utils.log import logger
from . import loss as _loss
from . import metrics as _metrics
from . import vit as _vit


def build(cfg):
    cfg = dict(copy.deepcopy(cfg))
    name = cfg.pop("name")
    if name in _vit.PRESETS:
        return _vit.build_vit(name, **cfg)
    for mod in (_vit, _loss, _metrics):
        if hasattr(mod, name) and not name.startswith("_"):
            return getattr(mod, name)(**cfg)
    raise ValueError("unknown vision component {}".format(name))


def _all_gather_cat(t):
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return t
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t.contiguous())
    return torch.cat(parts, 0)


class GeneralClsModule(BasicModule):
    def __init__(self, configs):
        self.nranks = env.get_world_size()
        self.model_configs = copy.deepcopy(configs.Model)
        self.model_configs.pop("module", None)
        super().__init__(configs)
        assert "train" in self.model_configs.loss
        self.loss_fn = build(self.model_configs.loss.train)
        self.eval_loss_fn = build(self.model_configs.loss.eval) if "eval" in self.model_configs.loss \
            else self.loss_fn
        metric = self.model_configs.get("metric", {}) or {}
        self.train_metric_fn = build(metric["train"]) if "train" in metric else None
        self.eval_metric_fn = build(metric["eval"]) if "eval" in metric else None
        self.train_batch_size = None
        self.eval_batch_size = None
        self.best_metric = 0.0
        self.acc_list = []

    def get_model(self):
        cfg = dict(copy.deepcopy(self.model_configs.model))
        if self.model_configs.get("use_recompute", False):
            cfg.setdefault("use_recompute", True)
        return build(cfg)

    def forward(self, inputs):
        return self.model(inputs)

    def training_step(self, batch):
        inputs, labels = batch
        if self.train_batch_size is None:
            self.train_batch_size = inputs.shape[0] * self.nranks
        return self.loss_fn(self(inputs), labels)

    def training_step_end(self, log_dict):
        ips = (self.train_batch_size or 0) / log_dict["train_cost"]
        logger.info("[train] epoch: %d, step: [%d/%d], learning rate: %.7f, loss: %.9f, "
                    "batch_cost: %.5f sec, ips: %.2f images/sec"
                    % (log_dict["epoch"], log_dict["batch"], log_dict.get("total_batch", -1),
                       log_dict["lr"], log_dict["loss"], log_dict["train_cost"], ips))

    def validation_step(self, batch):
        inputs, labels = batch
        logits = self(inputs)
        loss = self.eval_loss_fn(logits, labels)
        labels = _all_gather_cat(labels)
        logits = _all_gather_cat(logits)
        if self.eval_batch_size is None:
            self.eval_batch_size = logits.shape[0]
        if self.eval_metric_fn is not None:
            self.acc_list.append(self.eval_metric_fn(logits, labels))
        return loss

    def validation_step_end(self, log_dict):
        ips = (self.eval_batch_size or 0) / max(log_dict["eval_cost"], 1e-9)
        logger.info("[eval] epoch: %d, step: [%d/%d], loss: %.9f, batch_cost: %.5f sec, "
                    "ips: %.2f images/sec"
                    % (log_dict["epoch"], log_dict["batch"], log_dict.get("total_batch", -1),
                       float(log_dict["loss"]), log_dict["eval_cost"], ips))

    def test_step(self, batch):
        return self.validation_step(batch)

    def training_epoch_end(self, log_dict):
        logger.info("[Training] epoch: %d, total time: %.5f sec"
                    % (log_dict["epoch"], log_dict["train_cost"]))

    def validation_epoch_end(self, log_dict):
        msg = ""
        self.last_results = {}
        if self.acc_list:
            ret = defaultdict(list)
            for item in self.acc_list:
                for k, v in item.items():
                    ret[k].append(v)
            ret = {k: float(np.mean(v)) for k, v in ret.items()}
            if "metric" in ret:
                self.best_metric = max(self.best_metric, ret["metric"])
                ret["best_metric"] = self.best_metric
            self.last_results = ret
            msg = ", " + ", ".join("%s = %.6f" % (k, v) for k, v in ret.items())
            self.acc_list.clear()
        logger.info("[Eval] epoch: %d, total time: %.5f sec%s"
                    % (log_dict["epoch"], log_dict.get("eval_cost", 0.0), msg))

    def input_spec(self):
        size = self.model.patch_embed.img_size
        return [("images", [None, 3, size, size], torch.float32)]

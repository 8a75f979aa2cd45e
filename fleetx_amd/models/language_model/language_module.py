"""Language-model task modules: GPT pretraining / eval / generation.

Parity: reference ``models/language_model/language_module.py:31-389``
(C19-C21): ``training_step`` over ``(tokens, position_ids, labels,
loss_mask)``, the reference train-log line (``ips_total`` / ``ips``),
model-size estimate, model choice by parallel layout (single/TP/SP vs
pipeline), pipeline batch format, export ``input_spec``; offline
WikiText/LAMBADA evaluation; sampling generation.
"""
import copy
import math

import torch

from ...core.module.basic_module import BasicModule
from ...parallel import topology as topo
from ...utils.log import logger
from ...utils import env
from .utils import process_configs
from .gpt.model import (GPTConfig, GPTForPretraining, GPTPretrainingCriterion, num_params)


def compute_dtype(configs):
    mp = configs.Engine.get("mix_precision", {}) or {}
    if not torch.cuda.is_available() or str(configs.Global.get("device", "gpu")) == "cpu":
        return torch.float32
    if mp.get("use_pure_fp16") and str(mp.get("dtype", "bfloat16")) in ("float16", "fp16"):
        return torch.float16
    return torch.bfloat16


class LanguageModule(BasicModule):
    def __init__(self, configs):
        self.nranks = env.get_world_size()
        self.data_world_size = env.get_data_world_size()
        super().__init__(configs)
        self.loss_fn = self.get_loss_fn()

    def process_configs(self, configs):
        return process_configs(configs)

    def forward(self, tokens, ids=None):
        return self.model(tokens, ids)

    def training_step(self, batch):
        tokens, position_ids, labels, loss_mask = batch
        preds = self(tokens, position_ids)
        return self.loss_fn(preds, labels, loss_mask)

    def training_step_end(self, log_dict):
        speed = 1.0 / log_dict["train_cost"]
        tokens = self.configs.Global.global_batch_size * self._seq_len()
        logger.info(
            "[train] epoch: %d, batch: %d, loss: %.9f, avg_batch_cost: %.5f sec, speed: %.2f step/s, "
            "ips_total: %.0f tokens/s, ips: %.0f tokens/s, learning rate: %.5e"
            % (log_dict["epoch"], log_dict["batch"], log_dict["loss"], log_dict["train_cost"], speed,
               speed * tokens, speed * tokens / self.data_world_size, log_dict["lr"]))

    def _seq_len(self):
        try:
            return self.configs.Data.Train.dataset.max_seq_len
        except (AttributeError, KeyError, TypeError):
            return self.configs.Model.get("max_position_embeddings", 1024)

    def validation_step(self, batch):
        tokens, position_ids, labels, loss_mask = batch
        preds = self(tokens, position_ids)
        return self.loss_fn(preds, labels, loss_mask)

    def validation_step_end(self, log_dict):
        speed = 1.0 / log_dict["eval_cost"]
        logger.info("[eval] epoch: %d, batch: %d, loss: %.9f, avg_eval_cost: %.5f sec, speed: %.2f step/s"
                    % (log_dict["epoch"], log_dict["batch"], log_dict["loss"], log_dict["eval_cost"], speed))

    def test_step(self, batch):
        return self.validation_step(batch)

    def test_step_end(self, log_dict):
        speed = 1.0 / log_dict["test_cost"]
        logger.info("[test] epoch: %d, batch: %d, loss: %.9f, avg_test_cost: %.5f sec, speed: %.2f step/s"
                    % (log_dict["epoch"], log_dict["batch"], log_dict["loss"], log_dict["test_cost"], speed))

    def get_model_size(self, l, h, v, s):
        P = 12 * l * h * h * (1 + 13 / (12 * h) + (v + s) / (12 * l * h))
        logger.info("Model Size: {:.2f} B".format(P / 1e9))

    def training_epoch_end(self, log_dict):
        logger.info("[Training] epoch: %d, total time: %.5f sec" % (log_dict["epoch"], log_dict["train_cost"]))


class GPTModule(LanguageModule):
    def get_model(self):
        m = copy.deepcopy(self.configs.Model)
        for k in ("module", "name"):
            m.pop(k, None)
        self.get_model_size(m["num_layers"], m["hidden_size"], m["vocab_size"],
                            m["max_position_embeddings"])
        hcg = topo.get_hcg()
        if hcg.mp_degree == 1:
            m["sequence_parallel"] = False
        self.gpt_config = GPTConfig.from_model_config(m, dtype=compute_dtype(self.configs))
        if hcg.pp_degree > 1:
            from .gpt.pipeline_model import GPTForPretrainingPipe
            model = GPTForPretrainingPipe(self.gpt_config, hcg,
                                          virtual_pp_degree=m.get("virtual_pp_degree", 1) or 1)
        else:
            model = GPTForPretraining(self.gpt_config)
        q = self.configs.get("Quantization")
        if q is not None and q.get("enable", False):
            from ...utils.qat import quantize_model
            model = quantize_model(model, q)
        return model

    def get_loss_fn(self):
        return GPTPretrainingCriterion(self.gpt_config)

    def pretreating_batch(self, batch):
        if topo.get_hcg().pp_degree > 1:
            tokens, position_ids, labels, loss_mask = batch
            return [(tokens, position_ids), (labels, loss_mask)]
        return batch

    def input_spec(self):
        return [("tokens", [None, None], torch.int64), ("ids", [None, None], torch.int64)]

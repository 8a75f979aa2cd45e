"""Multimodal task modules (Imagen).

Parity: reference ``models/multimodal_model/multimodal_module.py:28-120`` and
``utils.py:31-137`` (C25, C12): the model is built by name from the
``imagen`` builders with the remaining ``Model`` keys, the criterion from the
``Loss`` section, ``training_step`` on ``(images, text_embeds, text_masks)``
and the step/s log line.  The reference's validation / test steps are GPT
copies that cannot run on image batches; here validation
computes the same diffusion loss as training.
"""
import copy

import torch

from ...core.module.basic_module import BasicModule
from ...utils import env
from ...utils.log import logger
from . import imagen


def process_configs(configs):
    g, d = configs.Global, configs.Distributed
    dp = d.get("dp_degree") or 1
    sd = (d.get("sharding") or {}).get("sharding_degree", 1) or 1
    try:  # the Imagen loaders carry the per-rank batch size
        g["local_batch_size"] = int(configs.Data.Train.loader.batch_size)
        g["global_batch_size"] = g.local_batch_size * dp * sd
    except (AttributeError, KeyError, TypeError):
        pass
    if g.get("global_batch_size") is None and g.get("local_batch_size") is not None:
        g["global_batch_size"] = g.local_batch_size * dp * sd
    m = configs.Model
    if m.get("use_recompute") and not m.get("recompute_granularity"):
        m["recompute_granularity"] = "full"
    return configs


class MultiModalModule(BasicModule):
    def __init__(self, configs):
        self.nranks = env.get_world_size()
        super().__init__(configs)
        self.loss_fn = self.get_loss_fn()

    def process_configs(self, configs):
        return process_configs(configs)

    def forward(self, samples, text_embeds, text_masks):
        return self.model(samples, text_embeds=text_embeds, text_masks=text_masks)

    def training_step(self, batch):
        samples, text_embeds, text_masks = batch
        pred, target, log_snr, gamma = self(samples, text_embeds, text_masks)
        return self.loss_fn(pred, target, log_snr, gamma)

    def validation_step(self, batch):
        return self.training_step(batch)

    def test_step(self, batch):
        return self.training_step(batch)

    def training_step_end(self, log_dict):
        speed = 1.0 / log_dict["train_cost"]
        ips = speed * self.configs.Global.global_batch_size
        logger.info("[train] epoch: %d, batch: %d, loss: %.9f, avg_batch_cost: %.5f sec, "
                    "speed: %.2f step/s, ips: %.2f images/sec, learning rate: %.5e"
                    % (log_dict["epoch"], log_dict["batch"], log_dict["loss"],
                       log_dict["train_cost"], speed, ips, log_dict["lr"]))

    def validation_step_end(self, log_dict):
        logger.info("[eval] epoch: %d, batch: %d, loss: %.9f, avg_eval_cost: %.5f sec"
                    % (log_dict["epoch"], log_dict["batch"], float(log_dict["loss"]),
                       log_dict["eval_cost"]))

    def training_epoch_end(self, log_dict):
        logger.info("[Training] epoch: %d, total time: %.5f sec"
                    % (log_dict["epoch"], log_dict["train_cost"]))

    def input_spec(self):
        size = self.model.image_sizes[0]
        return [("images", [None, 3, size, size], torch.float32),
                ("text_embeds", [None, None, self.model.text_embed_dim], torch.float32),
                ("text_masks", [None, None], torch.bool)]


class ImagenModule(MultiModalModule):
    def get_model(self):
        m = copy.deepcopy(self.configs.Model)
        for k in ("module", "recompute_granularity"):
            m.pop(k, None)
        name = m.pop("name")
        if name not in imagen.BUILDERS:
            raise ValueError("unknown imagen model {} (known: {})".format(name,
                                                                           sorted(imagen.BUILDERS)))
        model = imagen.BUILDERS[name](**dict(m))
        q = self.configs.get("Quantization")
        if q is not None and q.get("enable", False):
            # reference multimodal_module.py:86-89 (QAT over Conv2D / Conv2DTranspose / Linear)
            from ...utils.qat import quantize_model
            model = quantize_model(model, q)
        return model

    def get_loss_fn(self):
        return imagen.ImagenCriterion(**dict(copy.deepcopy(self.configs.get("Loss", {}) or {})))

    def pretreating_batch(self, batch):
        return batch

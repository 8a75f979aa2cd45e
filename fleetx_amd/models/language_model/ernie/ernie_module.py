"""ERNIE pretraining task module.

Parity: reference ``models/language_model/ernie/ernie_module.py:28-102``
(C23): builds ``ErnieForPretraining(ErnieModel(**Model))`` from the config,
data processors identical to GPT's (``num_samples`` per split, sampler batch
size = ``local_batch_size``), the same ``ips_total`` train log line.

The reference ``training_step`` is a placeholder that scores random labels
(``ernie_module.py:79-91``).  Here it is a real masked-LM
objective on the GPT-format batch ``(tokens, position_ids, labels,
loss_mask)``: tokens are dynamically masked on the device (15%, 80/10/10,
``Model.mask_token_id`` default ``vocab_size - 1``), only masked positions go
through the LM head, and the loss is the mean CE over them (``ignore_index``
-1, NSP off as in the reference).
"""
import copy

import torch

from ....core.module.basic_module import BasicModule
from ....parallel import topology as topo
from ....utils import env
from ....utils.log import logger
from ..language_module import compute_dtype
from ..utils import process_data_configs, process_optim_configs
from .model import ErnieModel, ErnieForPretraining, ErniePretrainingCriterion, mlm_mask

_MODEL_KEYS = ("vocab_size", "hidden_size", "num_hidden_layers", "num_attention_heads",
               "intermediate_size", "hidden_act", "hidden_dropout_prob",
               "attention_probs_dropout_prob", "max_position_embeddings", "type_vocab_size",
               "initializer_range", "pad_token_id", "task_type_vocab_size", "task_id",
               "use_task_id", "use_recompute")


class ErnieModule(BasicModule):
    def __init__(self, configs):
        self.nranks = env.get_world_size()
        self.data_world_size = env.get_data_world_size()
        super().__init__(configs)
        # sentence-pair samples (ErnieDataset) train MLM + next-sentence prediction
        try:
            ds_name = self.configs.Data.Train.dataset.name
        except (AttributeError, KeyError):
            ds_name = None
        self.pair_data = ds_name == "ErnieDataset"
        self.criterion = ErniePretrainingCriterion(with_nsp_loss=self.pair_data)
        m = self.configs.Model
        self.mask_token_id = m.get("mask_token_id", m.vocab_size - 1)
        self.mask_prob = m.get("masked_lm_prob", 0.15)
        ds = {}
        try:
            ds = dict(self.configs.Data.Train.dataset)
        except (AttributeError, KeyError):
            pass
        self.special_ids = tuple({m.get("pad_token_id", 0), ds.get("cls_id", 1), ds.get("sep_id", 2)})

    def process_configs(self, configs):
        process_data_configs(configs)
        if "Optimizer" in configs:
            process_optim_configs(configs)
        return configs

    def get_loss_fn(self):
        return None

    def get_model(self):
        m = copy.deepcopy(self.configs.Model)
        kw = {k: m[k] for k in _MODEL_KEYS if k in m and m[k] is not None}
        if topo.get_hcg().pp_degree > 1:
            raise NotImplementedError("ERNIE supports data / tensor parallel (pp_degree must be 1)")
        return ErnieForPretraining(ErnieModel(dtype=compute_dtype(self.configs), **kw))

    def forward(self, tokens, masked_positions=None):
        return self.model(tokens, masked_positions=masked_positions)

    def _mlm_loss(self, batch):
        tokens = batch[0]
        vocab = self.configs.Model.vocab_size
        pad = self.configs.Model.get("pad_token_id", 0)
        special = self.special_ids if self.pair_data else (pad,)
        inputs, labels = mlm_mask(tokens, vocab, self.mask_token_id, self.mask_prob,
                                  special_ids=special)
        flat = labels.reshape(-1)
        pos = torch.nonzero(flat >= 0).reshape(-1)
        if self.pair_data:  # (tokens, token_type_ids, next_sentence_label, length)
            scores, rel = self.model(inputs, token_type_ids=batch[1], masked_positions=pos)
            mlm, nsp = self.criterion(scores, rel, flat[pos], batch[2])
            return mlm + nsp
        scores, rel = self.model(inputs, masked_positions=pos)
        return self.criterion(scores, rel, flat[pos])

    def training_step(self, batch):
        return self._mlm_loss(batch)

    def validation_step(self, batch):
        return self._mlm_loss(batch)

    def training_step_end(self, log_dict):
        speed = 1.0 / log_dict["train_cost"]
        tokens = self.configs.Global.global_batch_size * self.configs.Data.Train.dataset.max_seq_len
        logger.info(
            "[train] epoch: %d, batch: %d, loss: %.9f, avg_batch_cost: %.5f sec, speed: %.2f step/s, "
            "ips_total: %.0f tokens/s, ips: %.0f tokens/s, learning rate: %.5e"
            % (log_dict["epoch"], log_dict["batch"], log_dict["loss"], log_dict["train_cost"], speed,
               speed * tokens, speed * tokens / self.data_world_size, log_dict["lr"]))

    def validation_step_end(self, log_dict):
        logger.info("[eval] epoch: %d, batch: %d, loss: %.9f, avg_eval_cost: %.5f sec"
                    % (log_dict["epoch"], log_dict["batch"], float(log_dict["loss"]),
                       log_dict["eval_cost"]))

    def input_spec(self):
        return [("input_ids", [None, None], torch.int64)]

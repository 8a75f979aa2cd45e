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
            "ips_total: %.0f tokens/s, ips: %.0f tokens/s, learning rate: %.5e, mfu: %.1f%%"
            % (log_dict["epoch"], log_dict["batch"], log_dict["loss"], log_dict["train_cost"], speed,
               speed * tokens, speed * tokens / self.data_world_size, log_dict["lr"],
               100.0 * self.mfu(speed * tokens)))

    def mfu(self, tokens_per_s):
        """Model FLOPs utilisation of the whole job: useful
        training FLOPs (6N + attention, no recompute) / (GPUs x dense peak)."""
        from ...utils import hw
        from .gpt.model import flops_per_token
        try:
            fpt = flops_per_token(self.gpt_config, self._seq_len())
        except Exception:
            return 0.0
        n = max(1, env.get_world_size())
        dt = str(getattr(self.gpt_config, "dtype", "bfloat16") or "bfloat16")
        return tokens_per_s * fpt / (n * hw.peak_flops(dt))

    def tokens_per_step(self):
        """Tokens of one optimizer step over the whole job (the ips_total numerator)."""
        return self.configs.Global.global_batch_size * self._seq_len()

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


class GPTGenerationModule(BasicModule):
    """Zero-shot text generation (reference ``language_module.py:179-274``, C20)."""

    def __init__(self, configs):
        self.nranks = env.get_world_size()
        super().__init__(configs)

    def process_configs(self, configs):
        return process_configs(configs)

    def get_model(self):
        from .gpt.generation import GPTForGeneration
        m = copy.deepcopy(self.configs.Model)
        for k in ("module", "name"):
            m.pop(k, None)
        m["sequence_parallel"] = False
        m["hidden_dropout_prob"] = 0.0
        m["attention_probs_dropout_prob"] = 0.0
        self.gpt_config = GPTConfig.from_model_config(m, dtype=compute_dtype(self.configs))
        gen = dict(self.configs.get("Generation", {}) or {})
        gen["max_dec_len"] = min(gen.get("max_dec_len", 20) or 20, 512)  # reference clamp
        self.tokenizer = None
        try:
            from ...data.tokenizers import GPTTokenizer
            self.tokenizer = GPTTokenizer.from_pretrained(
                self.configs.get("Tokenizer", {}).get("dir", "gpt2")
                if self.configs.get("Tokenizer") else "gpt2")
            eos = self.tokenizer.eos_token_id
        except FileNotFoundError:
            eos = gen.get("eos_token_id", 50256)
        for k in ("bos_token_id", "eos_token_id", "pad_token_id"):
            gen.setdefault(k, eos)
        return GPTForGeneration(GPTForPretraining(self.gpt_config), gen)

    def left_padding(self, inputs, pad_id):
        """Kept for API parity; generation here right-pads with lengths."""
        maxlen = max(len(x) for x in inputs)
        return [[pad_id] * (maxlen - len(x)) + list(x) for x in inputs]

    def generate(self, input_text):
        return self(input_text)

    def forward(self, input_text):
        assert self.tokenizer is not None, "generation from text needs tokenizer files"
        texts = [input_text] if isinstance(input_text, str) else list(input_text)
        ids = [self.tokenizer.encode(t) for t in texts]
        lens = torch.tensor([len(x) for x in ids])
        maxlen = int(lens.max())
        pad = self.tokenizer.eos_token_id
        arr = torch.tensor([x + [pad] * (maxlen - len(x)) for x in ids])
        dev = next(self.model.parameters()).device
        out, _ = self.model.generate(arr.to(dev), lens.to(dev))
        res = []
        for row in out.tolist():
            if pad in row:
                row = row[:row.index(pad)]
            res.append(self.tokenizer.convert_ids_to_string(row))
        return res

    def input_spec(self):
        return [("input_ids", [None, None], torch.int64)]


class GPTEvalModule(LanguageModule):
    """Offline WikiText PPL / LAMBADA accuracy (reference ``language_module.py:277-389``)."""

    def __init__(self, configs):
        self.eval_cfg = configs.get("Offline_Eval", {})
        super().__init__(configs)
        self.first_step = True
        self.total_score = 0.0
        self.score_name = "loss" if not self.eval_cfg.get("cloze_eval", False) else "number correct"

    def process_configs(self, configs):
        configs = process_configs(configs)
        oe = configs.get("Offline_Eval", {})
        ds = "Lambada_Eval_Dataset" if oe.get("cloze_eval") else "LM_Eval_Dataset"
        from ...utils.config import AttrDict
        configs.Data["Eval"] = AttrDict(
            dataset=AttrDict(name=ds, input_dir=oe.get("eval_path"),
                             max_seq_len=oe.get("max_seq_len", 1024),
                             overlapping_eval=oe.get("overlapping_eval", 32)),
            loader=AttrDict(num_workers=0, collate_fn="gpt_eval_collate_fn",
                            batch_size=oe.get("batch_size", 8)))
        for k in ("Train", "Test"):
            configs.Data.pop(k, None)
        return configs

    def get_model(self):
        return GPTModule.get_model(self)

    def get_loss_fn(self):
        return None

    def validation_step(self, batch):
        tokens, loss_mask, attention_mask, position_ids, labels, info = batch
        logits = self.model(tokens, position_ids).float()
        if not self.eval_cfg.get("cloze_eval", False):
            if self.first_step:
                self.num_original_tokens = int(info[0][0])
                self.num_tokenized_tokens = int(info[0][1])
            lp = torch.nn.functional.cross_entropy(logits.transpose(1, 2), labels, reduction="none")
            return (lp * loss_mask).sum()
        if self.first_step:
            self.num_examples = int(info[0][0])
        pred = logits.argmax(-1)
        correct = ((pred == labels).float() * loss_mask + (1 - loss_mask)).prod(-1)
        return correct.sum()

    def validation_step_end(self, log_dict):
        self.first_step = False
        self.total_score += float(log_dict["loss"])
        logger.info("[eval] epoch: %d, batch: %d, %s: %.9f, speed: %.2f step/s"
                    % (log_dict["epoch"], log_dict["batch"], self.score_name,
                       float(log_dict["loss"]), 1.0 / max(log_dict["eval_cost"], 1e-9)))

    def validation_epoch_end(self, log_dict):
        if not self.eval_cfg.get("cloze_eval", False):
            total_loss = self.total_score / (self.num_tokenized_tokens - 1)
            ppl = math.exp(min(20, total_loss))
            token_ratio = (self.num_tokenized_tokens - 1) / (self.num_original_tokens - 1)
            adjusted_ppl = math.exp(min(20, total_loss * token_ratio))
            msg = ("validation results on {} | avg loss: {:.4E} | ppl: {:.4E} | adjusted ppl: "
                   "{:.4E} | token ratio: {}".format(self.eval_cfg.get("eval_path"), total_loss,
                                                      ppl, adjusted_ppl, token_ratio))
            self.results = {"loss": total_loss, "ppl": ppl, "adjusted_ppl": adjusted_ppl}
        else:
            acc = self.total_score / self.num_examples
            msg = ("validation results on {} | number correct: {:.4E} | total examples: {:.4E} | "
                   "avg accuracy: {:.4E}".format(self.eval_cfg.get("eval_path"), self.total_score,
                                                 self.num_examples, acc))
            self.results = {"acc": acc}
        logger.info(msg)

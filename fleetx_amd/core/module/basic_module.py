"""Lightning-style task adapter (reference ``core/module/basic_module.py:29-86``).

A module owns ``self.model`` (built in the constructor after
``process_configs``) and the per-task hooks the engine calls.
"""
import torch.nn as nn


class BasicModule(nn.Module):
    def __init__(self, configs, *args, **kwargs):
        super().__init__()
        self.configs = self.process_configs(configs)
        self.model = self.get_model()

    def process_configs(self, configs):
        return configs

    def get_model(self):
        raise NotImplementedError

    def get_loss_fn(self):
        return None

    def pretreating_batch(self, batch):
        return batch

    def forward(self, *args, **kwargs):
        return self.model(*args, **kwargs)

    def training_step(self, *args, **kwargs):
        raise NotImplementedError

    def training_step_end(self, *args, **kwargs):
        pass

    def validation_step(self, *args, **kwargs):
        pass

    def validation_step_end(self, *args, **kwargs):
        pass

    def test_step(self, *args, **kwargs):
        pass

    def test_step_end(self, *args, **kwargs):
        pass

    def backward(self, loss):
        loss.backward()

    def input_spec(self):
        raise NotImplementedError("Please redefine Module.input_spec for model export")

    def inference_end(self, outputs):
        pass

    def training_epoch_end(self, *args, **kwargs):
        pass

    def validation_epoch_end(self, *args, **kwargs):
        pass

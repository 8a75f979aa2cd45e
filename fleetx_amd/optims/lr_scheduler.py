"""Learning-rate schedules.

Parity: reference ``ppfleetx/optims/lr_scheduler.py:22-91``.  The step
semantics follow Paddle's ``LRScheduler``: the constructor performs one
``step()`` so ``last_epoch`` starts at ``last_epoch + 1``, and the engine
calls ``step()`` once per optimizer update.
"""
import math


class LRScheduler:
    def __init__(self, learning_rate=0.1, last_epoch=-1):
        self.base_lr = float(learning_rate)
        self.last_lr = float(learning_rate)
        self.last_epoch = last_epoch
        self.step()

    def get_lr(self):
        return self.base_lr

    def step(self, epoch=None):
        if epoch is None:
            self.last_epoch += 1
        else:
            self.last_epoch = epoch
        self.last_lr = self.get_lr()

    def __call__(self):
        return self.last_lr

    def state_dict(self):
        return {"last_epoch": self.last_epoch, "last_lr": self.last_lr}

    def set_state_dict(self, state):
        self.last_epoch = state["last_epoch"]
        self.last_lr = state.get("last_lr", self.get_lr())

    load_state_dict = set_state_dict


class ConstantLR(LRScheduler):
    pass


class CosineAnnealingWithWarmupDecay(LRScheduler):
    """Linear warmup over ``warmup_rate * decay_steps`` steps, cosine from
    ``max_lr`` to ``min_lr`` until ``decay_steps``, then ``min_lr``."""

    def __init__(self, max_lr, min_lr, warmup_rate, decay_steps, last_epoch=0, **kwargs):
        self.decay_steps = decay_steps
        self.warmup_step = warmup_rate * decay_steps
        self.max_lr = max_lr
        self.min_lr = min_lr
        super().__init__(max_lr, last_epoch)

    def get_lr(self):
        if self.warmup_step > 0 and self.last_epoch <= self.warmup_step:
            return float(self.max_lr) * self.last_epoch / self.warmup_step
        if self.last_epoch > self.decay_steps:
            return self.min_lr
        ratio = float(self.last_epoch - self.warmup_step) / float(self.decay_steps - self.warmup_step)
        coeff = 0.5 * (math.cos(math.pi * ratio) + 1.0)
        return self.min_lr + coeff * (self.max_lr - self.min_lr)


class LinearDecayWithWarmup(LRScheduler):
    def __init__(self, learning_rate, total_steps, warmup=0, last_epoch=-1, **kwargs):
        self.total_steps = total_steps
        self.warmup = int(warmup * total_steps) if isinstance(warmup, float) and warmup < 1 else int(warmup)
        super().__init__(learning_rate, last_epoch)

    def get_lr(self):
        if self.warmup > 0 and self.last_epoch < self.warmup:
            return self.base_lr * self.last_epoch / self.warmup
        return self.base_lr * max(0.0, (self.total_steps - self.last_epoch) /
                                  max(1, self.total_steps - self.warmup))


class ViTLRScheduler(LRScheduler):
    """Linear/cosine decay over ``epochs * step_each_epoch`` with warmup."""

    def __init__(self, learning_rate, step_each_epoch, epochs, decay_type="cosine",
                 linear_end=1e-5, warmup_steps=0, last_epoch=-1, **kwargs):
        self.linear_end = linear_end
        self.T_max = epochs * step_each_epoch
        self.warmup_steps = min(warmup_steps, self.T_max - 1) if self.T_max > 0 else warmup_steps
        self.decay_type = decay_type
        super().__init__(learning_rate, last_epoch)

    def get_lr(self):
        progress = (self.last_epoch - self.warmup_steps) / float(max(1, self.T_max - self.warmup_steps))
        progress = min(1.0, max(0.0, progress))
        if self.decay_type == "linear":
            lr = self.linear_end + (self.base_lr - self.linear_end) * (1.0 - progress)
        else:
            lr = 0.5 * self.base_lr * (1.0 + math.cos(math.pi * progress))
        if self.warmup_steps:
            lr = lr * min(1.0, self.last_epoch / self.warmup_steps)
        return lr


SCHEDULERS = {
    "CosineAnnealingWithWarmupDecay": CosineAnnealingWithWarmupDecay,
    "ViTLRScheduler": ViTLRScheduler,
    "LinearDecayWithWarmup": LinearDecayWithWarmup,
    "ConstantLR": ConstantLR,
}

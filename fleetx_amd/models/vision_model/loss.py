"""Classification losses (reference ``vision_model/loss/cross_entropy.py:23-91``).

``CELoss``: softmax CE with optional label smoothing (``(1-eps)*onehot +
eps/C``) and soft-label support.  ``ViTCELoss``: per-class sigmoid BCE summed
over classes, mean over the batch, with the reference's ViT-style smoothing
``label*(1-eps) + eps``.  Both compute in fp32 regardless of logits dtype.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


def _logits(x):
    return (x["logits"] if isinstance(x, dict) else x).float()


def _one_hot(label, c):
    if label.ndim == 1 or label.shape[-1] != c:
        return F.one_hot(label.reshape(-1).long(), c).float()
    return label.float()


class CELoss(nn.Module):
    def __init__(self, epsilon=None):
        super().__init__()
        if epsilon is not None:
            assert 0 <= epsilon <= 1, "epsilon must be in [0, 1]"
        self.epsilon = epsilon

    def forward(self, x, label):
        x = _logits(x)
        c = x.shape[-1]
        if self.epsilon is not None:
            soft = _one_hot(label, c) * (1 - self.epsilon) + self.epsilon / c
            loss = torch.sum(-F.log_softmax(x, -1) * soft, -1)
        elif label.ndim > 1 and label.shape[-1] == c:
            loss = torch.sum(-label.float() * F.log_softmax(x, -1), -1)
        else:
            loss = F.cross_entropy(x, label.reshape(-1).long(), reduction="none")
        return loss.mean()


class ViTCELoss(nn.Module):
    def __init__(self, epsilon=None):
        super().__init__()
        if epsilon is not None:
            assert 0 <= epsilon <= 1, "epsilon must be in [0, 1]"
        self.epsilon = epsilon

    def forward(self, x, label):
        x = _logits(x)
        target = _one_hot(label, x.shape[-1])
        if self.epsilon is not None:
            target = target * (1.0 - self.epsilon) + self.epsilon
        loss = F.binary_cross_entropy_with_logits(x, target, reduction="none")
        return loss.sum(-1).mean()

"""Top-k accuracy (reference ``vision_model/metrics/accuracy.py:19-47``)."""
import torch
import torch.nn as nn


class TopkAcc(nn.Module):
    def __init__(self, topk=(1, 5)):
        super().__init__()
        self.topk = [topk] if isinstance(topk, int) else list(topk)

    @torch.no_grad()
    def forward(self, x, label):
        x = x["logits"] if isinstance(x, dict) else x
        label = label.reshape(-1).long()
        k_max = min(max(self.topk), x.shape[-1])
        top = x.float().topk(k_max, -1).indices
        hit = top == label[:, None]
        out = {}
        for i, k in enumerate(self.topk):
            acc = hit[:, :min(k, k_max)].any(-1).float().mean().item()
            out["top{}".format(k)] = acc
            if i == 0:
                out["metric"] = acc
        return out

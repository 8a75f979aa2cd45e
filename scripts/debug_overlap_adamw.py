"""Debug: forward-overlapped AdamW vs serial after the caching allocator has
handed out dirty memory (fills a large block with NaN first)."""
import sys
import torch
sys.path.insert(0, ".")
from fleetx_amd.models.language_model.gpt.model import (GPTConfig, GPTForPretraining,
                                                        GPTPretrainingCriterion)
from fleetx_amd.parallel.grad_buffer import FlatParamGradBuffer
from fleetx_amd.optims.optimizer import FusedAdamW, ClipGradByGlobalNorm

DEV = "cuda"
dirty = torch.full((1 << 28,), float("nan"), device=DEV)
del dirty
runs = []
for overlap in (False, True):
    torch.manual_seed(0)
    cfg = GPTConfig(vocab_size=1024, hidden_size=256, num_layers=3, num_attention_heads=4,
                    max_position_embeddings=128, hidden_dropout_prob=0.0,
                    attention_probs_dropout_prob=0.0, dtype=torch.bfloat16)
    model = GPTForPretraining(cfg).cuda()
    crit = GPTPretrainingCriterion(cfg)
    buf = FlatParamGradBuffer(model.named_parameters())
    opt = FusedAdamW(1e-3, buf, grad_clip=ClipGradByGlobalNorm(1.0), weight_decay=0.01)
    if overlap:
        assert opt.enable_forward_overlap(model)
    g = torch.Generator(device=DEV).manual_seed(5)
    losses, gn = [], []
    for _ in range(4):
        toks = torch.randint(0, 1024, (4, 129), device=DEV, generator=g)
        loss = crit(model(toks[:, :-1]), toks[:, 1:], torch.ones(4, 128, device=DEV))
        loss.backward()
        buf.finish()
        opt.step()
        gn.append(float(getattr(opt, "_last_norm", torch.zeros(())).item()) if hasattr(opt, "_last_norm") else None)
        opt.clear_grad()
        losses.append(loss.item())
    opt.sync_state()
    torch.cuda.synchronize()
    runs.append((losses, {n: p.detach().float().clone() for n, p in model.named_parameters()},
                 [m.clone() for m in opt.master]))
print("losses", runs[0][0], runs[1][0])
bad = 0
for n in runs[0][1]:
    a, b = runs[0][1][n], runs[1][1][n]
    if not torch.equal(a, b):
        bad += 1
        d = (a - b).abs()
        print("MISMATCH", n, tuple(a.shape), "max", float(d.max()), "count", int((d > 0).sum()),
              "nan", bool(torch.isnan(a).any()), bool(torch.isnan(b).any()))
print("bad params", bad)
for i, (x, y) in enumerate(zip(runs[0][2], runs[1][2])):
    if not torch.equal(x, y):
        d = (x - y).abs()
        idx = torch.nonzero(d > 0).flatten()
        print("master range", i, "n", x.numel(), "diff count", idx.numel(), "first", idx[:10].tolist())

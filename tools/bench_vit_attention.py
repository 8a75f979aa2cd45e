"""ViT-g/14 attention shape (B 64, S 257, 16 heads, head dim 88 on the 96 tile,
packed [B, S, 3, H, D] QKV) forward / backward time over back-to-back launches.

    python tools/bench_vit_attention.py
"""
import json, sys, torch
sys.path.insert(0, '.')
from fleetx_amd import ops
B, S, H, D = 64, 257, 16, 88
qkv = (0.5 * torch.randn(B, S, 3, H, D, device="cuda")).bfloat16().requires_grad_()
g = torch.randn(B, S, H, D, device="cuda").bfloat16()
f = lambda: ops.flash_attention_qkvpacked(qkv, causal=False, pack_dim=2, scale=D ** -0.5)
for _ in range(3):
    torch.autograd.grad(f(), qkv, g)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    f()
e1.record(); torch.cuda.synchronize(); tf = e0.elapsed_time(e1) / 20
outs = [f() for _ in range(20)]; torch.cuda.synchronize()
e0.record()
for o in outs:
    torch.autograd.grad(o, qkv, g)
e1.record(); torch.cuda.synchronize(); tb = e0.elapsed_time(e1) / 20
print(json.dumps({"shape": "ViT-g B64 S257 H16 D88", "fwd_ms": round(tf, 4), "bwd_ms": round(tb, 4)}))

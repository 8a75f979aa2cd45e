import os, sys, torch
sys.path.insert(0, os.getcwd())
from fleetx_amd import ops
torch.manual_seed(0)
def rel(a, b): return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))
for (B, S, H, D, p) in [(4, 1024, 8, 64, 0.1), (4, 1024, 8, 64, 0.0), (8, 1024, 8, 64, 0.1), (2, 1024, 4, 128, 0.1), (4, 2048, 8, 64, 0.1), (1, 1024, 1, 64, 0.0)]:
    qkv = (0.5 * torch.randn(B, S, H, 3, D, device="cuda")).bfloat16().requires_grad_()
    out = ops.flash_attention_qkvpacked(qkv, causal=True, dropout_p=p, key=1234)
    g = torch.randn_like(out)
    out.backward(g)
    nan_o = bool(torch.isnan(out).any()); nan_g = bool(torch.isnan(qkv.grad).any())
    ref_in = qkv.detach().float().requires_grad_()
    ref = ops.attention_reference(ref_in[:, :, :, 0], ref_in[:, :, :, 1], ref_in[:, :, :, 2], causal=True, dropout_p=p, key=1234)
    ref.backward(g.float())
    print(B, S, H, D, p, "nan out", nan_o, "nan grad", nan_g, "rel out %.4f" % rel(out, ref),
          "rel dq %.4f dk %.4f dv %.4f" % tuple(rel(qkv.grad[:, :, :, i], ref_in.grad[:, :, :, i]) for i in range(3)), flush=True)
    # per-row check of unwritten rows: rows where out is exactly zero everywhere
    z = (out.detach().float().abs().sum(-1) == 0).sum().item()
    print("   zero rows", z, flush=True)

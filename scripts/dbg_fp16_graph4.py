import os, sys
sys.path.insert(0, os.getcwd())
os.environ["FLEETX_DETERMINISTIC"] = "1"
import torch
from tests import test_fp16_gpu as T


def run(graph, steps, extra=(), overlap=False):
    from fleetx_amd.ops import _lib
    _lib.kernels().set_dropout_salt(0)
    _lib.kernels().set_adamw_lr_ptr(0)
    eng = T._engine("float16", extra=(
        "Engine.cuda_graph=%s" % graph, "Engine.mix_precision.incr_every_n_steps=2",
        "Engine.mix_precision.decr_every_n_nan_or_inf=1",
        "Distributed.comm.overlap_optimizer=%s" % overlap) + tuple(extra))
    sc, opt = eng.scaler, eng.optimizer
    assert eng.buffer._fused_norm is not None
    losses, infs = [], []
    for s in range(steps):
        if s == 3:
            sc.scale.fill_(2.0 ** 40)
        elif s == 4:
            sc.scale.fill_(1024.0)
        losses.append(round(float(eng._fit_impl(T._batch(s))), 6))
        torch.cuda.synchronize()
        infs.append(int(opt.found_inf.item()))
    opt.sync_state()
    torch.cuda.synchronize()
    params = {n: p.detach().float().cpu() for n, p in eng._module.model.named_parameters()}
    return losses, infs, params


mode = sys.argv[1]
if mode == "zero":
    os.environ["FLEETX_DBG_ZERO_SQ"] = "1"
ex = ("Distributed.comm.fused_grad_norm=True",)
ov = mode == "overlap"
e = run(False, 9, ex, ov)
g = run(True, 9, ex, ov)
bad = [n for n in e[2] if not torch.equal(e[2][n], g[2][n])]
print(mode, "eager", e[0], e[1], "\n      graph", g[0], g[1], "\n params differ", len(bad), flush=True)

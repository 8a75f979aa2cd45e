import os, sys
sys.path.insert(0, os.getcwd())
os.environ["FLEETX_DETERMINISTIC"] = "1"
import torch
from tests import test_fp16_gpu as T


def run(graph, steps, reads, inject=True, extra=()):
    from fleetx_amd.ops import _lib
    _lib.kernels().set_dropout_salt(0)
    _lib.kernels().set_adamw_lr_ptr(0)
    eng = T._engine("float16", extra=(
        "Engine.cuda_graph=%s" % graph, "Engine.mix_precision.incr_every_n_steps=2",
        "Engine.mix_precision.decr_every_n_nan_or_inf=1",
        "Distributed.comm.overlap_optimizer=False") + tuple(extra))
    sc, opt = eng.scaler, eng.optimizer
    losses = []
    for s in range(steps):
        if s == 3 and inject:
            sc.scale.fill_(2.0 ** 40)
        elif s == 4 and inject:
            sc.scale.fill_(1024.0)
        losses.append(round(float(eng._fit_impl(T._batch(s))), 6))
        torch.cuda.synchronize()
        if reads:
            float(sc.scale), int(opt.found_inf.item())
    opt.sync_state()
    torch.cuda.synchronize()
    st = {"losses": losses, "scale": float(sc.scale), "good": int(sc.good), "bad": int(sc.bad),
          "step": int(opt.dev_step.item()), "fi": int(opt.found_inf.item())}
    params = {n: p.detach().float().cpu() for n, p in eng._module.model.named_parameters()}
    m = [x.float().cpu() for x in opt.m]
    return st, params, m


for name, extra in (("base", ()), ("nofusednorm", ("Distributed.comm.fused_grad_norm=False",)),
                    ("g32", ("Distributed.comm.grad_dtype=float32",)),
                    ("both", ("Distributed.comm.fused_grad_norm=False", "Distributed.comm.grad_dtype=float32"))):
    e = run(False, 6, True, True, extra)
    g = run(True, 6, True, True, extra)
    bad = [n for n in e[1] if not torch.equal(e[1][n], g[1][n])]
    print(name, "eager", e[0]["losses"][-2:], "graph", g[0]["losses"][-2:], "params differ", len(bad))

import os, sys
sys.path.insert(0, os.getcwd())
os.environ["FLEETX_DETERMINISTIC"] = "1"
import torch
from tests import test_fp16_gpu as T


def run(graph, probe, steps=7, inject=(3, 4)):
    from fleetx_amd.ops import _lib
    _lib.kernels().set_dropout_salt(0)
    _lib.kernels().set_adamw_lr_ptr(0)
    eng = T._engine("float16", extra=(
        "Engine.cuda_graph=%s" % graph, "Engine.mix_precision.incr_every_n_steps=2",
        "Engine.mix_precision.decr_every_n_nan_or_inf=1",
        "Distributed.comm.overlap_optimizer=False"))
    sc, opt = eng.scaler, eng.optimizer
    out = []
    for s in range(steps):
        if s == inject[0]:
            sc.scale.fill_(2.0 ** 40)
        elif s == inject[1]:
            sc.scale.fill_(1024.0)
        l = float(eng._fit_impl(T._batch(s)))
        torch.cuda.synchronize()
        if "norm" in probe:
            float(opt.last_grad_norm)
        if "gscale" in probe:
            float(opt.gscale.item())
        if "good" in probe:
            int(sc.good), int(sc.bad)
        if "step" in probe:
            int(opt.dev_step.item())
        if "params" in probe:
            {n: p.detach().double().sum().item() for n, p in eng._module.model.named_parameters()}
        out.append(round(l, 6))
    return out


for probe in ["", "norm", "gscale", "good,step", "params", "norm,gscale,good,step,params"]:
    print(repr(probe), "eager", run(False, probe), "graph", run(True, probe))

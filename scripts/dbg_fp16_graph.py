import os, sys
sys.path.insert(0, os.getcwd())
os.environ["FLEETX_DETERMINISTIC"] = "1"
import torch
from tests import test_fp16_gpu as T


def run(graph, overlap=False, steps=7, inject=(3, 4)):
    from fleetx_amd.ops import _lib
    _lib.kernels().set_dropout_salt(0)
    _lib.kernels().set_adamw_lr_ptr(0)
    eng = T._engine("float16", extra=(
        "Engine.cuda_graph=%s" % graph, "Engine.mix_precision.incr_every_n_steps=2",
        "Engine.mix_precision.decr_every_n_nan_or_inf=1",
        "Distributed.comm.overlap_optimizer=%s" % overlap))
    sc, opt = eng.scaler, eng.optimizer
    rows, snaps = [], []
    for s in range(steps):
        if s == inject[0]:
            sc.scale.fill_(2.0 ** 40)
        elif s == inject[1]:
            sc.scale.fill_(1024.0)
        l = float(eng._fit_impl(T._batch(s)))
        torch.cuda.synchronize()
        rows.append((s, l, float(sc.scale), int(opt.found_inf.item()), int(opt.dev_step.item())))
        snaps.append({n: p.detach().double().sum().item() for n, p in eng._module.model.named_parameters()})
    return rows, snaps


res = {}
for rep in range(int(os.environ.get("REPS", "2"))):
    for g in (False, True):
        res[(rep, g)] = run(g)
ref_rows, ref_snaps = res[(0, False)]
for key, (rows, snaps) in res.items():
    diff = [r[1] for r in rows] != [r[1] for r in ref_rows]
    print(key, "losses differ" if diff else "losses equal", [round(r[1], 6) for r in rows])
    for s, (a, b) in enumerate(zip(snaps, ref_snaps)):
        bad = [n for n in a if a[n] != b[n]]
        if bad:
            print("   step", s, "params differ:", bad[:6], len(bad))
            break

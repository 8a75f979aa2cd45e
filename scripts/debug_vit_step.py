"""Debug aid: a few ViT training steps through the engine with per-step
timing and a stack dump if a step stalls (faulthandler)."""
import faulthandler
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
faulthandler.dump_traceback_later(int(os.environ.get("DUMP_AFTER", "100")), exit=True)

from fleetx_amd.utils import config as C  # noqa: E402
from fleetx_amd.utils import env  # noqa: E402
from fleetx_amd.models import build_module  # noqa: E402
from fleetx_amd.core.engine.eager_engine import EagerEngine  # noqa: E402
import torch  # noqa: E402

if os.environ.get("VIT_UNFUSED") == "1":
    from fleetx_amd.models.vision_model import vit
    vit.Block._fusable = lambda self: False
cfg_file = sys.argv[1]
ov = sys.argv[2:]
cfg = C.get_config(cfg_file, overrides=ov, nranks=1)
cfg.Optimizer.lr = {"name": "ConstantLR", "learning_rate": 1e-3}
env.init_dist_env(cfg)
env.set_seed(cfg.Global.seed)
module = build_module(cfg)
eng = EagerEngine(configs=cfg, module=module, mode="train")
B = cfg.Data.Train.sampler.batch_size
img = torch.randn(B, 3, 224, 224, device="cuda")
lab = torch.randint(0, 1000, (B,), device="cuda")
for i in range(4):
    t0 = time.time()
    loss = eng._fit_impl([img, lab])
    torch.cuda.synchronize()
    print("step", i, float(loss), "%.3f s" % (time.time() - t0), flush=True)

import os, sys
sys.path.insert(0, os.getcwd())
os.environ["FLEETX_DETERMINISTIC"] = "1"
import torch
_G = torch.cuda.CUDAGraph


class DbgGraph(_G):
    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.enable_debug_mode()


torch.cuda.CUDAGraph = DbgGraph
from tests import test_fp16_gpu as T
from fleetx_amd.ops import _lib
_lib.kernels().set_dropout_salt(0)
_lib.kernels().set_adamw_lr_ptr(0)
eng = T._engine("float16", extra=(
    "Engine.cuda_graph=True", "Engine.mix_precision.incr_every_n_steps=2",
    "Engine.mix_precision.decr_every_n_nan_or_inf=1", "Distributed.comm.overlap_optimizer=False"))
for s in range(3):
    eng._fit_impl(T._batch(s))
torch.cuda.synchronize()
os.makedirs("gpurun_out/r6d", exist_ok=True)
eng._graph.debug_dump("gpurun_out/r6d/graph.dot")
print("dumped")

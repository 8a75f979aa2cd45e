"""Zero-shot text generation with a trained checkpoint (reference ``tasks/gpt/generation.py:34-62``).

    python tasks/gpt/generation.py -c fleetx_amd/configs/nlp/gpt/generation_gpt_345M_single_card.yaml \
        -o Engine.save_load.ckpt_dir=./output/epoch_0_step_1000
"""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

import torch  # noqa: E402

from fleetx_amd.utils import config as cfgmod  # noqa: E402
from fleetx_amd.utils import env  # noqa: E402
from fleetx_amd.utils import checkpoint as ckpt  # noqa: E402
from fleetx_amd.models import build_module  # noqa: E402


def main(argv=None, prompts=None):
    args = cfgmod.parse_args(argv)
    cfg = cfgmod.get_config(args.config, overrides=args.override)
    env.init_dist_env(cfg)
    env.set_seed(cfg.Global.seed)
    module = build_module(cfg)
    module.model.eval()
    d = cfg.Engine.save_load.get("ckpt_dir")
    if d:
        path = os.path.join(d, "model.pdparams")
        if not os.path.exists(path):
            path = os.path.join(d, ckpt.shard_dirname(0, 0, 0), "model.pdparams")
        sd = ckpt.load_payload(path)
        module.model.model.load_state_dict({k: v.float() for k, v in sd.items()}, strict=False)
    dev = env.device()
    module.model.to(dev)
    if dev.type == "cuda":
        module.model.to(torch.bfloat16)
    prompts = prompts or ["Hi, GPT2. Tell me who Jack Ma is."]
    for p in prompts:
        out = module.generate(p)
        print("Prompt:", p)
        print("Generation:", out[0])
    return module


if __name__ == "__main__":
    main()

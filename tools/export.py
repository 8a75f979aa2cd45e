"""Export a trained model for the inference engine (reference ``tools/export.py:32-49``).

    python tools/export.py -c .../inference_gpt_345M_single_card.yaml -o Engine.save_load.ckpt_dir=...
"""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

from fleetx_amd.utils import config as cfgmod  # noqa: E402
from fleetx_amd.utils import env  # noqa: E402
from fleetx_amd.models import build_module  # noqa: E402
from fleetx_amd.core.engine.eager_engine import EagerEngine  # noqa: E402


def main(argv=None):
    args = cfgmod.parse_args(argv)
    cfg = cfgmod.get_config(args.config, overrides=args.override)
    env.init_dist_env(cfg)
    env.set_seed(cfg.Global.seed)
    module = build_module(cfg)
    engine = EagerEngine(configs=cfg, module=module, mode="export")
    engine.load()
    engine.export()


if __name__ == "__main__":
    main()

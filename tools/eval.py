"""Offline evaluation entry (reference ``tools/eval.py:34-54``).

    python tools/eval.py -c fleetx_amd/configs/nlp/gpt/eval_gpt_345M_single_card.yaml \
        -o Offline_Eval.eval_path=./wikitext-103/wiki.valid.tokens
"""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

from fleetx_amd.utils import config as cfgmod  # noqa: E402
from fleetx_amd.utils import env  # noqa: E402
from fleetx_amd.data import build_dataloader  # noqa: E402
from fleetx_amd.models import build_module  # noqa: E402
from fleetx_amd.core.engine.eager_engine import EagerEngine  # noqa: E402


def main(argv=None):
    args = cfgmod.parse_args(argv)
    cfg = cfgmod.get_config(args.config, overrides=args.override)
    env.init_dist_env(cfg)
    env.set_seed(cfg.Global.seed)
    module = build_module(cfg)
    cfgmod.print_config(cfg)
    loader = build_dataloader(cfg.Data, "Eval")
    engine = EagerEngine(configs=cfg, module=module, mode="eval")
    engine.load()
    engine.evaluate(valid_data_loader=loader)
    return module


if __name__ == "__main__":
    main()

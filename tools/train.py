"""Pretraining entry point (reference ``tools/train.py:38-72``).

    python tools/train.py -c fleetx_amd/configs/nlp/gpt/pretrain_gpt_345M_single_card.yaml [-o k=v ...]
    torchrun --nproc-per-node 8 tools/train.py -c .../pretrain_gpt_6.7B_tp2_pp2_dp2.yaml
"""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

from fleetx_amd.utils import config as cfgmod  # noqa: E402
from fleetx_amd.utils import env  # noqa: E402
from fleetx_amd.utils.log import logger  # noqa: E402
from fleetx_amd.data import build_dataloader  # noqa: E402
from fleetx_amd.models import build_module  # noqa: E402
from fleetx_amd.core.engine.eager_engine import EagerEngine  # noqa: E402


def main(argv=None):
    args = cfgmod.parse_args(argv)
    cfg = cfgmod.get_config(args.config, overrides=args.override, show=False)
    env.init_dist_env(cfg)
    env.set_seed(cfg.Global.seed)
    module = build_module(cfg)
    cfgmod.print_config(cfg)
    train_loader = build_dataloader(cfg.Data, "Train")
    valid_loader = build_dataloader(cfg.Data, "Eval")
    if "lr" in cfg.Optimizer and cfg.Optimizer.lr.get("name") == "ViTLRScheduler":
        cfg.Optimizer.lr["step_each_epoch"] = len(train_loader)
        cfg.Optimizer.lr["epochs"] = cfg.Engine.num_train_epochs
    engine = EagerEngine(configs=cfg, module=module, mode="train")
    if cfg.Engine.save_load.get("ckpt_dir") is not None:
        engine.load()
    engine.fit(train_data_loader=train_loader, valid_data_loader=valid_loader,
               epoch=cfg.Engine.num_train_epochs)
    logger.info("training finished")
    return engine


if __name__ == "__main__":
    main()

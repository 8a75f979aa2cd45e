"""Run an exported model over the Test dataloader (reference ``tools/inference.py:37-59``)."""
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
    cfg = cfgmod.get_config(args.config, overrides=args.override)
    env.init_dist_env(cfg)
    module = build_module(cfg)
    engine = EagerEngine(configs=cfg, module=module, mode="inference")
    loader = build_dataloader(cfg.Data, "Test")
    outs = []
    for i, batch in enumerate(loader):
        if i >= cfg.Engine.test_iters:
            break
        data = [b.numpy() for b in batch]
        out = engine.inference(data)
        logger.info("inference batch %d -> %s" % (i, [o.shape for o in out]))
        outs.append(out)
    return outs


if __name__ == "__main__":
    main()

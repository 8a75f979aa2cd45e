"""Module-level config processors for the language models.

Parity: reference ``models/language_model/utils.py:39-150`` (data
``num_samples``/mode/seed/batch size, ``ffn_hidden_size = 4h``, recompute
default granularity, pipeline divisibility checks, ``multi_precision``,
tensor-fusion restriction, inference defaults).  ``fused_linear`` is accepted
and ignored: the bias is always fused into the HIP epilogue kernels.
"""
from ...utils.log import logger
from ...utils.config import get_world_size


def process_inference_configs(config):
    if "Inference" not in config:
        return
    inf = config["Inference"]
    if inf.get("model_dir") is None:
        inf["model_dir"] = config.Engine.save_load.output_dir
    if inf.get("mp_degree") is None:
        inf["mp_degree"] = config.Distributed.mp_degree


def process_model_configs(config):
    m = config.Model
    if m.get("ffn_hidden_size") is None:
        m["ffn_hidden_size"] = 4 * m.hidden_size
    if m.get("use_recompute") and not m.get("recompute_granularity"):
        m["recompute_granularity"] = "full"
    m.setdefault("fused_linear", False)
    pp = config.Distributed.pp_degree
    if pp > 1:
        vpp = m.get("virtual_pp_degree") or 1
        m["virtual_pp_degree"] = vpp
        assert m.num_layers % (vpp * pp) == 0, \
            "num_layers {} must be divisible by pp_degree * virtual_pp_degree ({} * {})".format(
                m.num_layers, pp, vpp)
        if vpp > 1:
            acc = config.Global.local_batch_size // config.Global.micro_batch_size
            assert acc % pp == 0, "num of microbatches {} should be divisible by pp_degree {} " \
                "when using interleave pipeline".format(acc, pp)
        if vpp > 2:
            logger.warning("Setting virtual_pp_degree > 2 may harm pipeline throughput.")
    elif m.get("virtual_pp_degree"):
        logger.warning("virtual_pp_degree is unused without pipeline parallel.")


def process_optim_configs(config):
    config.Optimizer["multi_precision"] = True
    if config.Optimizer.get("tensor_fusion"):
        assert get_world_size() == config.Distributed.dp_degree or get_world_size() == 1, \
            "tensor_fusion only supports single card or pure data parallel"


def process_data_configs(config):
    g, data, eng = config.Global, config.get("Data"), config.Engine
    if data is None:
        return
    max_steps = eng.get("max_steps", 1)
    eval_freq = max(1, eng.get("eval_freq", 1) or 1)
    num = {
        "Train": g.global_batch_size * max_steps,
        "Eval": g.global_batch_size * (max_steps // eval_freq + 1) * eng.get("eval_iters", 10),
        "Test": g.global_batch_size * eng.get("test_iters", 100),
    }
    for mode in ("Train", "Eval", "Test"):
        if mode in data and data[mode] is not None:
            data[mode].dataset["num_samples"] = num[mode]
            data[mode].dataset["mode"] = mode
            data[mode].dataset["seed"] = g.seed
            data[mode].setdefault("sampler", {})
            data[mode].sampler["batch_size"] = g.local_batch_size


def process_configs(config):
    process_data_configs(config)
    process_model_configs(config)
    process_optim_configs(config)
    process_inference_configs(config)
    return config

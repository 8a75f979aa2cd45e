"""YAML configuration system.

Behavioural parity with reference ``ppfleetx/utils/config.py``:

* ``_base_`` single inheritance resolved relative to the child file, dict
  values deep-merge, ``_inherited_: False`` replaces instead (``:163-202``);
* string leaves pass through ``ast.literal_eval`` (``:147-160``);
* ``-o a.b.0.c=v`` overrides create missing keys (``:248-310``);
* derived values: ``dp_degree`` from world size (``:30-65``), global/local
  batch (``:68-95``), ``accumulate_steps``/``save_steps``/``test_iters``
  (``:98-117``); the auto-parallel variants (``:332-464``).

Differences (MI355X-first): overrides are parsed with ``ast.literal_eval``
plus a tiny arithmetic evaluator instead of ``eval``; world size comes from
the torchrun env contract; mixed precision gains a ``dtype`` key (bf16
default) and ``Distributed`` gains ``comm`` tuning keys with defaults so that
reference YAMLs load unchanged.
"""
import argparse
import ast
import copy
import operator
import os
import sys

import yaml

from .log import logger, advertise

__all__ = ["AttrDict", "parse_config", "get_config", "get_auto_config",
           "override_config", "parse_args", "print_config"]


class AttrDict(dict):
    """dict with attribute access (reference ``config.py:120-144``)."""

    def __getattr__(self, key):
        try:
            return self[key]
        except KeyError as e:
            raise AttributeError(key) from e

    def __setattr__(self, key, value):
        self[key] = value

    def __deepcopy__(self, memo):
        out = AttrDict()
        memo[id(self)] = out
        for k, v in self.items():
            out[copy.deepcopy(k, memo)] = copy.deepcopy(v, memo)
        return out

    def __getstate__(self):
        return dict(self)

    def __setstate__(self, state):
        self.update(state)


def _to_attrdict(obj):
    if isinstance(obj, dict):
        out = AttrDict()
        for k, v in obj.items():
            out[k] = _to_attrdict(v)
        return out
    if isinstance(obj, list):
        return [_to_attrdict(v) for v in obj]
    if isinstance(obj, str):
        try:
            return ast.literal_eval(obj)
        except (ValueError, SyntaxError):
            return obj
    return obj


def _merge(child, base):
    """Deep merge ``child`` over ``base`` (both plain dicts)."""
    if not child.get("_inherited_", True):
        child = dict(child)
        child.pop("_inherited_")
        return child
    out = dict(base)
    for k, v in child.items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = _merge(v, out[k])
        else:
            out[k] = v
    return out


def _load_yaml(path):
    with open(path, "r", encoding="utf-8") as f:
        dic = yaml.load(f, Loader=yaml.SafeLoader) or {}
    if "_base_" in dic:
        base_path = os.path.join(os.path.dirname(path), dic.pop("_base_"))
        dic = _merge(dic, _load_yaml(base_path))
    return dic


def parse_config(cfg_file):
    """Load a YAML config (with ``_base_`` chain) into an :class:`AttrDict`."""
    return _to_attrdict(_load_yaml(cfg_file))


# --------------------------------------------------------------------------
# -o overrides
# --------------------------------------------------------------------------
_BINOPS = {ast.Add: operator.add, ast.Sub: operator.sub, ast.Mult: operator.mul,
           ast.Div: operator.truediv, ast.FloorDiv: operator.floordiv,
           ast.Pow: operator.pow, ast.Mod: operator.mod}


def _safe_eval(node):
    if isinstance(node, ast.Expression):
        return _safe_eval(node.body)
    if isinstance(node, ast.Constant):
        return node.value
    if isinstance(node, ast.UnaryOp) and isinstance(node.op, (ast.USub, ast.UAdd)):
        v = _safe_eval(node.operand)
        return -v if isinstance(node.op, ast.USub) else v
    if isinstance(node, ast.BinOp) and type(node.op) in _BINOPS:
        return _BINOPS[type(node.op)](_safe_eval(node.left), _safe_eval(node.right))
    if isinstance(node, (ast.List, ast.Tuple)):
        vals = [_safe_eval(e) for e in node.elts]
        return vals if isinstance(node, ast.List) else tuple(vals)
    if isinstance(node, ast.Dict):
        return {_safe_eval(k): _safe_eval(v) for k, v in zip(node.keys, node.values)}
    if isinstance(node, ast.Name) and node.id in ("True", "False", "None"):
        return {"True": True, "False": False, "None": None}[node.id]
    raise ValueError("unsupported expression")


def str2value(v):
    """Parse an override value: numbers, bools, lists, ``1.0/255.0``...

    Falls back to the raw string (reference ``config.py:259-263`` used eval).
    """
    try:
        return _safe_eval(ast.parse(v.strip(), mode="eval"))
    except (ValueError, SyntaxError, TypeError, ZeroDivisionError):
        return v


def _override(dl, keys, value):
    if isinstance(dl, list):
        idx = int(keys[0])
        if len(keys) == 1:
            assert idx < len(dl), "index {} out of range {}".format(idx, len(dl))
            dl[idx] = _to_attrdict(str2value(value))
        else:
            _override(dl[idx], keys[1:], value)
        return
    if len(keys) == 1:
        if keys[0] not in dl:
            logger.warning("A new field ({}) detected!".format(keys[0]))
        dl[keys[0]] = _to_attrdict(str2value(value))
        return
    if keys[0] not in dl or dl[keys[0]] is None:
        logger.warning("A new series field ({}) detected!".format(keys[0]))
        dl[keys[0]] = AttrDict()
    _override(dl[keys[0]], keys[1:], value)


def override_config(config, options=None):
    for opt in options or []:
        assert isinstance(opt, str) and "=" in opt, \
            "option {} should be key=value".format(opt)
        key, value = opt.split("=", 1)
        _override(config, key.split("."), value)
    return config


# --------------------------------------------------------------------------
# derived values
# --------------------------------------------------------------------------
def get_world_size():
    return int(os.environ.get("WORLD_SIZE", os.environ.get("PADDLE_TRAINERS_NUM", "1")))


def _fill_defaults(config):
    config.setdefault("Distributed", AttrDict())
    dist = config.Distributed
    if dist.get("sharding") is None:
        dist["sharding"] = AttrDict()
    dist.sharding.setdefault("sharding_degree", 1)
    dist.sharding.setdefault("sharding_stage", 1)
    dist.sharding.setdefault("sharding_offload", False)
    comm = dist.setdefault("comm", AttrDict())
    comm.setdefault("dp_bucket_mb", 256)        # few, large RCCL calls over xGMI
    comm.setdefault("overlap_grad_reduce", True)
    comm.setdefault("reduce_dtype", "float32")
    comm.setdefault("tp_overlap", True)         # async dX all-reduce / chunked row all-reduce
    comm.setdefault("tp_row_chunks", 2)
    comm.setdefault("sp_chunks", 2)             # SP all-gather / reduce-scatter chunks
    comm.setdefault("wgrad_stream", False)      # wgrad GEMMs on a side stream (opt-in, see eager_engine)
    comm.setdefault("overlap_optimizer_grid", 128)  # workgroups of the forward-overlapped AdamW
    eng = config.setdefault("Engine", AttrDict())
    eng.setdefault("cuda_graph", False)        # whole-step HIP graph (single rank)
    mp = eng.setdefault("mix_precision", AttrDict())
    mp.setdefault("use_pure_fp16", False)
    mp.setdefault("dtype", "bfloat16")
    mp.setdefault("scale_loss", 32768.0)
    config.setdefault("Global", AttrDict())
    config.Global.setdefault("seed", 1024)
    config.Global.setdefault("device", "gpu")
    config.Global.setdefault("global_batch_size", None)
    config.Global.setdefault("local_batch_size", None)
    config.Global.setdefault("micro_batch_size", 1)


def process_dist_config(dist, nranks=None):
    """Reference ``config.py:30-65``."""
    nranks = get_world_size() if nranks is None else nranks
    dist["mp_degree"] = dist.get("mp_degree") or 1
    dist["pp_degree"] = dist.get("pp_degree") or 1
    dist.sharding["sharding_degree"] = dist.sharding.get("sharding_degree") or 1
    other = dist.mp_degree * dist.pp_degree * dist.sharding.sharding_degree
    assert nranks % other == 0, "unreasonable config of dist_strategy: world {} " \
        "not divisible by mp*pp*sharding={}".format(nranks, other)
    if not dist.get("dp_degree"):
        dist["dp_degree"] = nranks // other
    elif dist.dp_degree * other != nranks:
        logger.warning("Mismatched config using {} cards with dp_degree[{}], mp_degree[{}], "
                       "pp_degree[{}] and sharding_degree[{}]; adjusting dp_degree to {}".format(
                           nranks, dist.dp_degree, dist.mp_degree, dist.pp_degree,
                           dist.sharding.sharding_degree, nranks // other))
        dist["dp_degree"] = nranks // other


def process_global_configs(config):
    """Reference ``config.py:68-95``."""
    dp = config.Distributed.dp_degree
    sd = config.Distributed.sharding.sharding_degree
    g = config.Global
    if g.global_batch_size is None and g.local_batch_size is None:
        raise ValueError("global_batch_size or local_batch_size should be set.")
    if g.global_batch_size is not None and g.local_batch_size is not None:
        assert g.global_batch_size // g.local_batch_size == dp * sd, \
            "global_batch_size[{}] should be local_batch_size[{}] * dp[{}] * sharding[{}]".format(
                g.global_batch_size, g.local_batch_size, dp, sd)
    elif g.global_batch_size is not None:
        assert g.global_batch_size % (dp * sd) == 0
        g["local_batch_size"] = g.global_batch_size // (dp * sd)
    else:
        g["global_batch_size"] = g.local_batch_size * dp * sd
    assert g.local_batch_size % g.micro_batch_size == 0, \
        "local_batch_size must be a multiple of micro_batch_size"


def process_engine_config(config):
    """Reference ``config.py:98-117``."""
    eng = config.Engine
    sl = eng.get("save_load")
    if sl:
        if sl.get("save_steps") in (None, -1):
            sl["save_steps"] = sys.maxsize
        if sl.get("save_epoch") in (None, -1):
            sl["save_epoch"] = 1
    eng.setdefault("eval_iters", 10)
    if eng.get("test_iters") is None:
        eng["test_iters"] = eng.eval_iters * 10
    eng["accumulate_steps"] = config.Global.local_batch_size // config.Global.micro_batch_size


def get_config(fname, overrides=None, show=False, nranks=None):
    assert os.path.exists(fname), "config file({}) does not exist".format(fname)
    config = parse_config(fname)
    override_config(config, overrides)
    _fill_defaults(config)
    process_dist_config(config.Distributed, nranks)
    process_global_configs(config)
    process_engine_config(config)
    if show:
        print_config(config)
    return config


# --------------------------------------------------------------------------
# auto-parallel variants (reference config.py:332-464)
# --------------------------------------------------------------------------
def process_auto_dist_configs(config, nranks=None):
    """Reference ``config.py:332-366``: ``dp = nranks / (mp * pp)`` and the
    sharding degree must divide it.  The reference counts sharding ranks inside
    dp; the hybrid topology here keeps sharding as its own axis, so the stored
    ``dp_degree`` is the number of pure replicas (``dp / sharding``)."""
    dist = config.Distributed
    nranks = get_world_size() if nranks is None else nranks
    dist["mp_degree"] = dist.get("mp_degree") or 1
    dist["pp_degree"] = dist.get("pp_degree") or 1
    sd = dist.sharding["sharding_degree"] = dist.sharding.get("sharding_degree") or 1
    other = dist.mp_degree * dist.pp_degree
    assert nranks % other == 0, "nranks should be divisible by mp_degree*pp_degree"
    data = nranks // other
    if dist.get("dp_degree") and dist.dp_degree * other != nranks:
        logger.warning("Mismatched config using {} cards with dp_degree[{}], mp_degree[{}], "
                       "pp_degree[{}]; adjusting dp_degree to {}".format(
                           nranks, dist.dp_degree, dist.mp_degree, dist.pp_degree, data))
    if sd > data:  # e.g. sharding16 on a smaller node: shard over what exists
        logger.warning("sharding_degree {} > data-parallel ranks {}; using {}".format(sd, data,
                                                                                    data))
        sd = dist.sharding["sharding_degree"] = data
    assert data % sd == 0, "dp_degree[{}] must be divisible by sharding_degree[{}]".format(data, sd)
    dist["dp_degree"] = data // sd


def process_auto_global_configs(config):
    d = config.Distributed
    data = d.dp_degree * d.sharding.sharding_degree
    g = config.Global
    if g.global_batch_size is None and g.local_batch_size is None:
        raise ValueError("global_batch_size or local_batch_size should be set.")
    if g.global_batch_size is not None and g.local_batch_size is not None:
        if g.global_batch_size // g.local_batch_size != data:
            g["local_batch_size"] = None
    if g.global_batch_size is not None and g.local_batch_size is None:
        assert g.global_batch_size % data == 0, \
            "global_batch_size[{}] should be divisible by data ranks[{}]".format(
                g.global_batch_size, data)
        g["local_batch_size"] = g.global_batch_size // data
    elif g.global_batch_size is None:
        g["global_batch_size"] = g.local_batch_size * data
    if g.local_batch_size % g.micro_batch_size:
        g["micro_batch_size"] = g.local_batch_size
    assert g.local_batch_size % g.micro_batch_size == 0


def process_auto_strategy(config):
    """Build the plain-dict strategy consumed by :class:`AutoEngine`."""
    eng = config.Engine
    amp = eng.get("mix_precision", AttrDict())
    sh = config.Distributed.sharding
    eng["strategy"] = AttrDict(
        auto_mode=eng.get("auto_mode", "semi"),
        seed=config.Global.seed,
        amp=AttrDict(enable=amp.get("enable", False),
                     level=amp.get("level", "o2"),
                     dtype=amp.get("dtype", "bfloat16"),
                     init_loss_scaling=amp.get("init_loss_scaling", 32768.0)),
        recompute=AttrDict(enable=eng.get("use_recompute", False)),
        sharding=AttrDict(enable=sh.sharding_degree > 1, degree=sh.sharding_degree,
                          stage=sh.get("sharding_stage", 1)),
    )


def get_auto_config(fname, overrides=None, show=False, nranks=None):
    assert os.path.exists(fname), "config file({}) does not exist".format(fname)
    config = parse_config(fname)
    override_config(config, overrides)
    _fill_defaults(config)
    process_auto_dist_configs(config, nranks)
    process_auto_global_configs(config)
    process_engine_config(config)
    process_auto_strategy(config)
    if show:
        print_config(config)
    return config


def print_dict(d, indent=0):
    for k, v in sorted(d.items(), key=lambda kv: str(kv[0])):
        if isinstance(v, dict):
            logger.info("{}{} : ".format(" " * indent, k))
            print_dict(v, indent + 4)
        elif isinstance(v, list) and v and isinstance(v[0], dict):
            logger.info("{}{} : ".format(" " * indent, k))
            for item in v:
                print_dict(item, indent + 4)
        else:
            logger.info("{}{} : {}".format(" " * indent, k, v))
        if isinstance(k, str) and k[:1].isupper() and indent == 0:
            logger.info("-" * 60)


def print_config(config):
    advertise()
    print_dict(config)


def parse_args(argv=None):
    parser = argparse.ArgumentParser("FleetX-AMD")
    parser.add_argument("-c", "--config", type=str, default="configs/config.yaml",
                        help="config file path")
    parser.add_argument("-o", "--override", action="append", default=[],
                        help="config options to be overridden, key.sub=value")
    return parser.parse_args(argv)

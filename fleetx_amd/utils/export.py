"""Model export for the inference engine.

Parity: reference ``ppfleetx/utils/export.py:24-59`` + ``eager_engine.py:662-669``
(``to_static`` -> prune -> ``jit.save`` to ``output_dir/rank_{r}/model.pdmodel
+ model.pdiparams``).

MI355X-native design: there is no tracing compiler in the loop.  An exported
model is a self-describing directory per rank:

    rank_{r}/model.json        module name, Model/Generation config, input spec
    rank_{r}/model.pdparams    weights (tensor dict, ``torch.load(weights_only)``)

and :class:`~fleetx_amd.core.engine.inference_engine.InferenceEngine`
rebuilds the network on the HIP kernels and replays its fixed-shape forward
through a captured HIP graph.
"""
import json
import os

import torch

from . import checkpoint as ckpt


def _plain(obj):
    if isinstance(obj, dict):
        return {str(k): _plain(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [_plain(v) for v in obj]
    if isinstance(obj, (int, float, str, bool)) or obj is None:
        return obj
    return str(obj)


def export_inference_model(module, output_dir, mp_degree=1):
    """``mp_degree > 1``: ``output_dir`` is this tensor-parallel rank's
    ``rank_{mp_rank}`` directory and the weights are its shard."""
    os.makedirs(output_dir, exist_ok=True)
    cfg = module.configs
    try:
        spec = module.input_spec()
    except NotImplementedError:
        spec = []
    meta = {
        "module": cfg.Model.get("module", "GPTModule"),
        "Model": _plain(dict(cfg.Model)),
        "Generation": _plain(dict(cfg.get("Generation", {}) or {})),
        "Global": _plain(dict(cfg.Global)),
        "input_spec": [[n, s, str(d).replace("torch.", "")] for n, s, d in spec],
        "mp_degree": int(mp_degree),
        "format": "fleetx-amd-export-v1",
    }
    with open(os.path.join(output_dir, "model.json"), "w") as f:
        json.dump(meta, f, indent=2)
    sd = {k: v.detach().to("cpu", copy=True) for k, v in module.model.state_dict().items()}
    torch.save(sd, os.path.join(output_dir, "model.pdparams"))
    return output_dir


def load_exported(model_dir):
    with open(os.path.join(model_dir, "model.json")) as f:
        meta = json.load(f)
    sd = ckpt.load_payload(os.path.join(model_dir, "model.pdparams"))
    return meta, sd

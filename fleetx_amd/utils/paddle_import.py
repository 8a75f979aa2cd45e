"""Import reference (PaddleFleetX) GPT checkpoints.

SURVEY §5.4: "an optional importer for reference ``.pdparams`` files (pickled
numpy dicts; Paddle ``Linear`` weights are ``[in, out]``, so transpose for
``[out, in]`` layouts) enables PPL parity checks against the published 345M
checkpoint".  The reference writes them with ``paddle.save(state_dict)``
(``eager_engine.py:589-612``): a pickle of ``{structured_name: ndarray}``
plus a ``StructuredToParameterName@@`` table.

Safety: the file is read by a restricted unpickler that resolves ONLY the
numpy array / dtype reconstructors and plain containers -- any other global
(code execution gadgets included) raises ``UnpicklingError``.  Nothing in the
file is executed.

Name map (``single_model.py:43-653`` -> ``fleetx_amd/models/language_model/gpt/model.py``)::

    gpt.embeddings.word_embeddings.weight        -> gpt.embeddings.word_embeddings.weight
    gpt.embeddings.position_embeddings.weight    -> gpt.embeddings.position_embeddings
    gpt.decoder.layers.{i}.norm1.{weight,bias}   -> gpt.layers.{i}.ln1.*
    gpt.decoder.layers.{i}.self_attn.qkv_proj.*  -> gpt.layers.{i}.attn.qkv_proj.*   (W^T)
    gpt.decoder.layers.{i}.self_attn.out_proj.*  -> gpt.layers.{i}.attn.out_proj.*   (W^T)
    gpt.decoder.layers.{i}.norm2.*               -> gpt.layers.{i}.ln2.*
    gpt.decoder.layers.{i}.linear1.*             -> gpt.layers.{i}.mlp.fc1.*          (W^T)
    gpt.decoder.layers.{i}.linear2.*             -> gpt.layers.{i}.mlp.fc2.*          (W^T)
    gpt.decoder.norm.{weight,bias}               -> gpt.final_ln.*

The fused QKV column order is the same in both (per head ``[q_h | k_h | v_h]``,
``single_model.py:99-103``), so only the ``[in, out] -> [out, in]`` transpose
is needed.  Split q/k/v projections (``fuse_attn_qkv=False``) are packed into
that per-head layout.
"""
import io
import pickle
import re

import numpy as np
import torch

_ALLOWED = {
    ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
    ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
    ("numpy", "ndarray"), ("numpy", "dtype"),
    ("collections", "OrderedDict"),
    ("builtins", "dict"), ("builtins", "list"), ("builtins", "tuple"), ("builtins", "bytes"),
    ("_codecs", "encode"),
}


class _SafeUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError("refusing to load global {}.{} from a checkpoint".format(
            module, name))


def load_paddle_state(path_or_bytes):
    """``{name: np.ndarray}`` from a reference ``.pdparams`` (restricted unpickling)."""
    if isinstance(path_or_bytes, (bytes, bytearray)):
        f = io.BytesIO(path_or_bytes)
        obj = _SafeUnpickler(f).load()
    else:
        with open(path_or_bytes, "rb") as f:
            obj = _SafeUnpickler(f).load()
    if not isinstance(obj, dict):
        raise ValueError("expected a state dict, got {}".format(type(obj).__name__))
    return {k: v for k, v in obj.items()
            if isinstance(v, np.ndarray) and not k.startswith("StructuredToParameterName")}


_LAYER = re.compile(r"^(?:gpt\.)?decoder\.layers\.(\d+)\.(.+)$")
_SUB = {
    "norm1.weight": ("ln1.weight", False), "norm1.bias": ("ln1.bias", False),
    "norm2.weight": ("ln2.weight", False), "norm2.bias": ("ln2.bias", False),
    "self_attn.qkv_proj.weight": ("attn.qkv_proj.weight", True),
    "self_attn.qkv_proj.bias": ("attn.qkv_proj.bias", False),
    "self_attn.out_proj.weight": ("attn.out_proj.weight", True),
    "self_attn.out_proj.bias": ("attn.out_proj.bias", False),
    "linear1.weight": ("mlp.fc1.weight", True), "linear1.bias": ("mlp.fc1.bias", False),
    "linear2.weight": ("mlp.fc2.weight", True), "linear2.bias": ("mlp.fc2.bias", False),
}
_TOP = {
    "embeddings.word_embeddings.weight": "gpt.embeddings.word_embeddings.weight",
    "embeddings.position_embeddings.weight": "gpt.embeddings.position_embeddings",
    "decoder.norm.weight": "gpt.final_ln.weight",
    "decoder.norm.bias": "gpt.final_ln.bias",
}


def _pack_split_qkv(sd, num_heads):
    """``fuse_attn_qkv=False`` checkpoints: q/k/v ``[h, h]`` -> fused per-head ``[h, 3h]``."""
    out = dict(sd)
    for k in list(sd):
        m = re.match(r"^(.*self_attn\.)q_proj\.(weight|bias)$", k)
        if not m:
            continue
        pre, kind = m.groups()
        q, kk, v = (sd[pre + n + "_proj." + kind] for n in ("q", "k", "v"))
        h = q.shape[-1]
        d = h // num_heads
        parts = [x.reshape(*x.shape[:-1], num_heads, d) for x in (q, kk, v)]
        fused = np.stack(parts, axis=-2).reshape(*q.shape[:-1], 3 * h)  # [.., heads, 3, d]
        out[pre + "qkv_proj." + kind] = fused
        for n in ("q", "k", "v"):
            del out[pre + n + "_proj." + kind]
    return out


def convert_gpt_state(paddle_sd, num_heads=None):
    """Reference GPT names/layouts -> this framework's ``GPTForPretraining`` state dict."""
    if num_heads is not None:
        paddle_sd = _pack_split_qkv(paddle_sd, num_heads)
    out = {}
    for k, v in paddle_sd.items():
        key = k[len("gpt."):] if k.startswith("gpt.") else k
        t = torch.from_numpy(np.ascontiguousarray(v))
        if key in _TOP:
            out[_TOP[key]] = t
            continue
        m = _LAYER.match(k)
        if m and m.group(2) in _SUB:
            name, transpose = _SUB[m.group(2)]
            out["gpt.layers.{}.{}".format(m.group(1), name)] = t.t().contiguous() if transpose else t
            continue
        raise KeyError("unmapped reference parameter: {}".format(k))
    return out


def _find_heads(model):
    for mod in model.modules():
        for obj in (mod, getattr(mod, "config", None), getattr(mod, "gpt_config", None)):
            h = getattr(obj, "num_attention_heads", None) if obj is not None else None
            if isinstance(h, int):
                return h
    return None


def load_into_model(model, path, strict=True, num_heads=None):
    """Load a reference ``.pdparams`` into ``model`` (cast to the model's dtypes).
    ``num_heads`` is only needed for split q/k/v checkpoints (found on the model
    config when omitted)."""
    heads = num_heads if num_heads is not None else _find_heads(model)
    sd = convert_gpt_state(load_paddle_state(path), num_heads=heads)
    own = model.state_dict()
    missing = [k for k in own if k not in sd]
    if strict and missing:
        raise KeyError("checkpoint lacks {} parameters, e.g. {}".format(len(missing), missing[:3]))
    for k, v in sd.items():
        if k not in own:
            if strict:
                raise KeyError("model has no parameter {}".format(k))
            continue
        if tuple(own[k].shape) != tuple(v.shape):
            raise ValueError("{}: checkpoint {} vs model {}".format(k, tuple(v.shape),
                                                                   tuple(own[k].shape)))
        with torch.no_grad():
            own[k].copy_(v.to(own[k].dtype))
    return model


__all__ = ["load_paddle_state", "convert_gpt_state", "load_into_model"]

"""Lower shard annotations of a serial network into the distributed model.

Parity: reference P10 / C32 — the semi-auto engine's completion + partition
passes (``core/engine/auto_engine.py:86-100``; the annotated GPT of
``gpt/auto/auto_model.py:109-110,238-239,601-610``): the user writes the
SERIAL network, annotates tensors with ``shard_tensor(w, mesh, spec)`` and the
engine turns that into per-rank shards.

MI355X-first lowering (no graph partitioner / program rewriting):

1. the serial network is built once with every weight whole
   (``topology.serial_scope``: layers see a one-rank model-parallel world);
   every rank builds the identical serial weights from the per-name seeds;
2. :func:`complete` turns the annotations into a storage-layout spec for EVERY
   parameter (annotations use the reference's ``[in, out]`` convention for
   linear weights; biases inherit the output split of their weight; anything
   unannotated is replicated) and derives the layout they imply: which mesh
   dimension carries the tensor parallelism and with which degree, and the
   pipeline stage of every decoder layer (``Mesh.stages``);
3. :func:`lower` fills the materialised hybrid model (TP layers / 1F1B
   stages) from the serial weights, slicing each tensor by ITS completed spec
   and this rank's mesh coordinates.  A parallel parameter whose shape is not
   the slice its spec implies -- an annotation that disagrees with the
   runtime's partitioning -- is an error, as is a tensor-parallel degree with
   no tensor sharded on it.

The result equals the serial model split by the annotations, so a semi-auto
run starts from bit-identical weights to the single-rank run.
"""
import re

import torch

from .. import topology as topo
from .mesh import get_dist_attr


def _linear_like(mod):
    from .. import layers as L
    return isinstance(mod, (L.ColumnParallelLinear, L.RowParallelLinear, torch.nn.Linear))


def complete(serial, mesh):
    """Storage-layout spec of every parameter of ``serial`` (name -> list of
    mesh dim names / None), plus the implied layout ``{"tp_dim", "tp_degree",
    "stages"}``."""
    specs = {}
    mods = dict(serial.named_modules())
    tp_dims = set()
    for mname, mod in mods.items():
        w = getattr(mod, "weight", None)
        if not isinstance(w, torch.nn.Parameter):
            continue
        attr = get_dist_attr(w)
        if attr is None:
            continue
        _, spec = attr
        spec = list(spec)
        if _linear_like(mod):
            spec = spec[::-1]  # [in, out] annotation -> [out, in] storage
        specs[(mname + "." if mname else "") + "weight"] = spec
        tp_dims.update(s for s in spec if s is not None)
        b = getattr(mod, "bias", None)
        if isinstance(b, torch.nn.Parameter) and _linear_like(mod):
            specs[(mname + "." if mname else "") + "bias"] = [spec[0]]
    for name, p in serial.named_parameters():
        specs.setdefault(name, [None] * p.dim())
    if len(tp_dims) > 1:
        raise ValueError("tensors are sharded over several mesh dims %s; one tensor-parallel "
                         "dim is supported" % sorted(tp_dims))
    tp_dim = next(iter(tp_dims)) if tp_dims else None
    pm = mesh.process_mesh
    layout = {"tp_dim": tp_dim, "tp_degree": pm.size(tp_dim) if tp_dim else 1}
    stages = {}
    for mname, mod in mods.items():
        st = getattr(mod, "_fx_stage", None)
        if st is not None:
            stages[mname] = st
    layout["stages"] = stages
    return specs, layout


def _coords(hcg):
    return {"mp": hcg.mp_rank, "pp": hcg.pp_rank,
            "dp": hcg.dp_rank * hcg.sharding_degree + hcg.sharding_rank}


def shard_slice(full, spec, mesh, coords):
    """The part of ``full`` this rank owns under ``spec``."""
    out = full
    for d, name in enumerate(spec):
        if name is None:
            continue
        n = mesh.process_mesh.size(name)
        if out.shape[d] % n:
            raise ValueError("dim %d of size %d is not divisible by mesh dim %s=%d"
                             % (d, out.shape[d], name, n))
        out = out.chunk(n, dim=d)[coords[name]]
    return out


_PIPE_LAYER = re.compile(r"^chunks\.(\d+)\.layers\.(\d+)\.(.*)$")


def serial_name(name, model, hcg):
    """Serial-network name of a parameter of the materialised model."""
    if not hasattr(model, "chunks"):
        return name
    if name == "shared_word_embeddings":
        return "gpt.embeddings.word_embeddings.weight"
    m = _PIPE_LAYER.match(name)
    if m:
        c, j, rest = int(m.group(1)), int(m.group(2)), m.group(3)
        per = model.cfg.num_layers // (model.P * model.V)
        v = c * model.P + hcg.pp_rank
        return "gpt.layers.%d.%s" % (v * per + j, rest)
    m = re.match(r"^chunks\.\d+\.(embeddings|final_ln)\.(.*)$", name)
    if m:
        return "gpt.%s.%s" % (m.group(1), m.group(2))
    raise KeyError(name)


def lower(serial, model, mesh, hcg=None):
    """Copy the annotation-sliced serial weights into ``model``; returns the
    completed layout (see :func:`complete`)."""
    hcg = hcg or topo.get_hcg()
    specs, layout = complete(serial, mesh)
    if layout["tp_degree"] != hcg.mp_degree:
        raise ValueError("annotations shard over %s=%d but the runtime has mp_degree=%d"
                         % (layout["tp_dim"], layout["tp_degree"], hcg.mp_degree))
    if hcg.mp_degree > 1 and layout["tp_dim"] != "mp":
        raise ValueError("tensor parallelism must use the mesh dim 'mp'")
    # stage annotations must match the runtime's placement of decoder layers
    if hcg.pp_degree > 1 and getattr(model, "V", 1) == 1:
        per = model.cfg.num_layers // hcg.pp_degree
        for mname, st in layout["stages"].items():
            m = re.match(r"^gpt\.layers\.(\d+)$", mname)
            if m and int(m.group(1)) // per != st:
                raise ValueError("%s is annotated for stage %d but runs on stage %d"
                                 % (mname, st, int(m.group(1)) // per))
    coords = _coords(hcg)
    full = dict(serial.named_parameters())
    n = 0
    with torch.no_grad():
        for name, p in model.named_parameters():
            sname = serial_name(name, model, hcg)
            src = shard_slice(full[sname], specs[sname], mesh, coords)
            if tuple(src.shape) != tuple(p.shape):
                raise ValueError("%s: annotation %s gives a %s shard but the runtime holds %s"
                                 % (name, specs[sname], tuple(src.shape), tuple(p.shape)))
            p.copy_(src.to(p.dtype))
            n += 1
    layout["lowered"] = n
    return layout

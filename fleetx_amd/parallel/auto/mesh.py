"""Process meshes and sharding annotations (semi-auto parallel front end).

Parity: reference P10 / C32 — ``auto.ProcessMesh`` with named dims, the
``Mesh`` helper of ``gpt/auto/auto_utils.py:24-108`` (mesh dims ``[pp, dp,
mp]`` with degree-1 axes dropped, ``mesh[stage]`` sub-meshes,
``stages(num_layers)``), and ``auto.shard_tensor`` / ``auto.shard_op``
annotations (``auto_model.py:109-110,143-146,238-239,384-387,464-465,601-610``).

Annotations are recorded on tensors as ``_fx_dist = (mesh, spec)``: a spec
``[None, "mp"]`` on a ``[in, out]`` weight means a column-parallel split,
``["mp", None]`` a row-parallel split.  :mod:`.partition` completes the specs
of a serial network and lowers them: every tensor of the materialised hybrid
model (TP layers, 1F1B stages, flat-buffer DP/ZeRO) is the slice of the
serial tensor its spec names.  :func:`verify_annotations` checks annotations
made directly on an already-parallel model (the QAT path).
"""
import numpy as np


class ProcessMesh:
    def __init__(self, mesh, dim_names=None):
        arr = np.asarray(mesh, dtype=np.int64)
        if arr.ndim == 0:
            arr = arr.reshape(1)
        self.mesh = arr
        self.dim_names = list(dim_names) if dim_names is not None else \
            ["d%d" % i for i in range(arr.ndim)]
        assert len(self.dim_names) == arr.ndim, "dim_names must match the mesh rank"

    @property
    def shape(self):
        return list(self.mesh.shape)

    @property
    def process_ids(self):
        return self.mesh.reshape(-1).tolist()

    @property
    def ndim(self):
        return self.mesh.ndim

    def size(self, name):
        return self.mesh.shape[self.dim_names.index(name)] if name in self.dim_names else 1

    def __getitem__(self, idx):
        sub = self.mesh[idx]
        if np.ndim(sub) == 0:  # a single process: a one-process mesh
            return ProcessMesh([int(sub)], ["serial"])
        return ProcessMesh(sub, self.dim_names[1:] if np.ndim(sub) == self.mesh.ndim - 1
                           else self.dim_names)

    def __contains__(self, rank):
        return int(rank) in self.process_ids

    def __eq__(self, other):
        return isinstance(other, ProcessMesh) and self.dim_names == other.dim_names and \
            np.array_equal(self.mesh, other.mesh)

    def __repr__(self):
        return "ProcessMesh(shape={}, dim_names={})".format(self.shape, self.dim_names)


class Mesh:
    """Topology helper built from the ``Distributed`` config (pp, dp, mp order)."""

    def __init__(self, dist_cfg):
        pp, dp, mp = dist_cfg["pp_degree"], dist_cfg["dp_degree"], dist_cfg["mp_degree"]
        self.config = dict(pp_degree=pp, dp_degree=dp, mp_degree=mp)
        dims = [(n, d) for n, d in (("pp", pp), ("dp", dp), ("mp", mp)) if d > 1]
        n = int(np.prod([d for _, d in dims])) if dims else 1
        procs = np.arange(n)
        if dims:
            self.process_mesh = ProcessMesh(procs.reshape([d for _, d in dims]),
                                            [nm for nm, _ in dims])
        else:
            self.process_mesh = ProcessMesh(procs, ["serial"])
        names = self.process_mesh.dim_names
        self.dp_dim = "dp" if "dp" in names else None
        self.mp_dim = "mp" if "mp" in names else None

    def __getitem__(self, idx):
        if "pp" in self.process_mesh.dim_names:
            return self.process_mesh[idx]
        return self.process_mesh

    def stages(self, num_layers):
        per = num_layers // self.config["pp_degree"]
        return [i // per for i in range(num_layers)]

    @property
    def dp(self):
        return self.dp_dim

    @property
    def mp(self):
        return self.mp_dim


def shard_tensor(tensor, mesh, spec):
    """Record that ``tensor`` is distributed over ``mesh`` as ``spec`` (one
    entry per tensor dim: a mesh dim name or None)."""
    assert len(spec) == tensor.dim(), "spec {} does not match rank {}".format(spec, tensor.dim())
    for s in spec:
        assert s is None or s in mesh.dim_names, "unknown mesh dim {}".format(s)
    tensor._fx_dist = (mesh, list(spec))
    return tensor


def shard_op(fn, mesh, in_specs=None, out_specs=None):
    """Wrap ``fn`` so its outputs carry ``out_specs`` annotations."""
    def wrapped(*args, **kwargs):
        out = fn(*args, **kwargs)
        if out_specs:
            outs = out if isinstance(out, (tuple, list)) else (out,)
            for o, spec in zip(outs, out_specs):
                if spec is not None and hasattr(o, "dim") and len(spec) == o.dim():
                    o._fx_dist = (mesh, list(spec))
        return out
    return wrapped


def get_dist_attr(tensor):
    return getattr(tensor, "_fx_dist", None)


def verify_annotations(model):
    """Check every annotated parameter against its actual TP partitioning.

    Returns the number of annotated parameters; raises on a mismatch."""
    from .. import layers as L
    n = 0
    for mod in model.modules():
        kind = None
        if isinstance(mod, L.ColumnParallelLinear):
            kind = "col"
        elif isinstance(mod, L.RowParallelLinear):
            kind = "row"
        elif isinstance(mod, L.VocabParallelEmbedding):
            kind = "vocab"
        w = getattr(mod, "weight", None)
        attr = get_dist_attr(w) if w is not None else None
        if attr is None or kind is None:
            continue
        n += 1
        mesh, spec = attr
        # weights are stored [out, in]; annotations use the reference's [in, out]
        want = {"col": [None, "mp"], "row": ["mp", None], "vocab": ["mp", None]}[kind]
        if "mp" not in mesh.dim_names:
            want = [None, None]
        if spec != want and not (kind == "vocab" and spec == ["mp", None]):
            raise ValueError("annotation {} on a {} layer; expected {}".format(spec, kind, want))
    return n

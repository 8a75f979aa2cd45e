"""Hybrid-parallel process topology and communication groups.

Capability parity: Paddle ``HybridCommunicateGroup`` reached from
reference ``tools/train.py:42-43`` / ``ppfleetx/utils/env.py:49-96`` and
consumed at ``eager_engine.py:173-188``, ``hybrid_model.py:48-51``.

MI355X-first design:

* one process per GPU, ``torch.distributed`` with backend ``nccl`` (= RCCL on
  ROCm) for device collectives and a side ``gloo`` group for host barriers;
* axis order ``[dp, pp, sharding, mp]`` with mp innermost so that the
  latency-critical TP collectives of a group sit on adjacent GPUs (on an MI355X
  node every GPU pair has a direct xGMI link, so adjacency only matters across
  nodes, where mp/pp must stay intra-node);
* groups are created once, eagerly, for every axis (``new_group`` is
  collective, so all ranks create all groups in the same order).
"""
import itertools
import os

import torch
import torch.distributed as dist

_HCG = None

# Per-communicator RCCL CTA budget (``Distributed.comm.ctas.<key>``): every
# RCCL channel is one workgroup resident on a CU for the whole collective, so
# the budget is set per group by what the group overlaps with, not by one
# process-wide NCCL_MIN_NCHANNELS:
#  * mp (TP all-reduce / SP gather-scatter): on the critical path -> many
#    channels when the group spans several links; a TP-2 pair is ONE xGMI
#    link, which a few channels fill, so its budget is small
#    (every extra channel is a CU taken from the GEMM chunk the all-reduce
#    overlaps; RCCL's topology search picks the rest) -- see model_ctas();
#  * dp / sharding / data_world (gradient buckets, ZeRO gathers): overlapped
#    with backward GEMMs that want all 256 CUs -> capped;
#  * pp (activation p2p) and the tied-embedding pair: medium;
#  * check (norm / found-inf scalars): latency-bound -> few.
# ``(min_ctas, max_ctas)``; ``None`` leaves the bound to RCCL.
# OPT-IN (``Distributed.comm.ctas: preset`` or a dict of overrides): the
# budgets have not been measured on a multi-GPU xGMI node yet, and a data-group
# cap of 16 channels could leave links of the 7-link mesh idle, so by default
# no group carries options and the process-wide ``NCCL_MIN_NCHANNELS=32``
# floor (utils/env.py) applies to every communicator.
CTA_KEYS = {"dp": "data", "mp": "model", "pp": "pipe", "sharding": "sharding",
            "data_world": "data_world", "check": "check", "embedding": "embedding"}
DEFAULT_CTAS = {"model": (32, 64), "data": (8, 16), "sharding": (8, 16),
                "data_world": (8, 16), "pipe": (4, 16), "check": (1, 4),
                "embedding": (8, 32)}


def model_ctas(t):
    """Default TP-group budget for a group of ``t`` GPUs: ``t - 1`` links,
    about 8 channels per link (unmeasured across GPUs: a floor so one link is
    kept busy, a cap so the overlapped GEMM keeps its CUs)."""
    if t <= 2:
        return (8, 16)
    if t <= 4:
        return (16, 32)
    return DEFAULT_CTAS["model"]


def parse_ctas(cfg):
    """``Distributed.comm.ctas`` -> ``{group name: (min, max)}``.

    ``None`` / ``{}`` / ``False``: no per-group budget (RCCL's own choice over
    the process-wide channel floor).  ``"preset"`` / ``True``: the
    DEFAULT_CTAS table.  A dict: the table with these overrides -- values
    ``"min,max"``, ``[min, max]`` or an int (max only); ``None`` / ``False``
    for a key drops that group's bound."""
    if cfg is False or cfg is None or (isinstance(cfg, dict) and not cfg):
        return {}
    if cfg is True or cfg == "preset":
        cfg = {}
    out = dict(DEFAULT_CTAS)
    for k, v in dict(cfg or {}).items():
        name = CTA_KEYS.get(k, k)
        if name not in DEFAULT_CTAS:
            raise ValueError("Distributed.comm.ctas: unknown group %r (keys: %s)"
                             % (k, ", ".join(sorted(CTA_KEYS))))
        if v in (None, False):
            out.pop(name, None)
            continue
        if isinstance(v, str):
            v = [int(x) for x in v.split(",")]
            v = v[0] if len(v) == 1 else v
        if isinstance(v, int):
            v = (None, v)
        lo, hi = v
        if lo is not None and hi is not None and lo > hi:
            raise ValueError("Distributed.comm.ctas.%s: min %d > max %d" % (k, lo, hi))
        out[name] = (lo, hi)
    out["pipe_bwd"] = out.get("pipe")
    if out["pipe_bwd"] is None:
        out.pop("pipe_bwd")
    return out


def nccl_options(ctas):
    """``ProcessGroupNCCL.Options`` carrying ``(min_ctas, max_ctas)``."""
    if ctas is None:
        return None
    opts = dist.ProcessGroupNCCL.Options()
    lo, hi = ctas
    if lo is not None:
        opts.config.min_ctas = int(lo)
    if hi is not None:
        opts.config.max_ctas = int(hi)
    return opts


class ParallelMode:
    DATA_PARALLEL = 0
    TENSOR_PARALLEL = 1
    PIPELINE_PARALLEL = 2
    SHARDING_PARALLEL = 3


class CommGroup:
    """A process group plus its rank list and this process' position in it."""

    def __init__(self, ranks, group, gloo_group=None):
        self.ranks = list(ranks)
        self.group = group
        self.gloo_group = gloo_group
        me = dist.get_rank() if dist.is_initialized() else 0
        self.rank = self.ranks.index(me) if me in self.ranks else -1
        self.nranks = len(self.ranks)

    @property
    def world_size(self):
        return self.nranks

    def __repr__(self):
        return "CommGroup(ranks={}, rank={})".format(self.ranks, self.rank)


class HybridTopology:
    """Rank <-> coordinate map for axes ``(dp, pp, sharding, mp)``."""

    AXES = ("data", "pipe", "sharding", "model")

    def __init__(self, dp=1, pp=1, sharding=1, mp=1):
        self.dims = (dp, pp, sharding, mp)
        self.world_size = dp * pp * sharding * mp
        self._coord_to_rank = {}
        self._rank_to_coord = {}
        for r, coord in enumerate(itertools.product(*[range(d) for d in self.dims])):
            self._coord_to_rank[coord] = r
            self._rank_to_coord[r] = coord

    def get_coord(self, rank):
        return self._rank_to_coord[rank]

    def get_rank(self, **kw):
        coord = tuple(kw[a] for a in self.AXES)
        return self._coord_to_rank[coord]

    def axis_groups(self, axis):
        """All rank lists that vary only along ``axis``."""
        ai = self.AXES.index(axis)
        others = [range(d) for i, d in enumerate(self.dims) if i != ai]
        groups = []
        for fixed in itertools.product(*others):
            ranks = []
            for v in range(self.dims[ai]):
                coord = list(fixed)
                coord.insert(ai, v)
                ranks.append(self._coord_to_rank[tuple(coord)])
            groups.append(ranks)
        return groups


class HybridCommunicateGroup:
    """Holds every communicator of the hybrid layout for this rank."""

    def __init__(self, dp=1, mp=1, pp=1, sharding=1, pp_split_directions=False, ctas=None):
        self.topo = HybridTopology(dp=dp, pp=pp, sharding=sharding, mp=mp)
        self.initialized = dist.is_initialized()
        self.global_rank = dist.get_rank() if self.initialized else 0
        ws = dist.get_world_size() if self.initialized else 1
        assert ws == self.topo.world_size, \
            "world size {} != dp{}*pp{}*sharding{}*mp{}".format(ws, dp, pp, sharding, mp)
        self.dp_degree, self.mp_degree, self.pp_degree, self.sharding_degree = dp, mp, pp, sharding
        coord = self.topo.get_coord(self.global_rank)
        self.dp_rank, self.pp_rank, self.sharding_rank, self.mp_rank = coord
        self.stage_id = self.pp_rank
        self._nccl = self.initialized and dist.get_backend() == "nccl"
        self.ctas = parse_ctas(ctas) if ctas is not False else {}
        self._model_ctas_set = isinstance(ctas, dict) and any(CTA_KEYS.get(k, k) == "model"
                                                              for k in ctas)

        self._groups = {}
        for axis in HybridTopology.AXES:
            self._groups[axis] = self._build(self.topo.axis_groups(axis), axis)
        # data world = dp x sharding (reference env.py:76-96)
        self._groups["data_world"] = self._build(self._data_world_groups(), "data_world")
        # "check" group: mp x pp x sharding for global-norm / found-inf reductions
        self._groups["check"] = self._build(self._check_groups(), "check")
        # first/last pipeline stage pairs for the tied embedding
        self._groups["embedding"] = self._build(self._embedding_groups(), "embedding")
        # Optional second communicator over each pipe group
        # (Distributed.comm.pp_split_directions): backward-direction p2p gets
        # its own RCCL stream.  Off by default: with more peer-waiting streams
        # than GPU_MAX_HW_QUEUES two directions can land in one in-order
        # hardware queue in opposite orders on neighbouring stages
        # (utils/streams.py); one communicator is deadlock-free whatever the
        # mapping.
        self._groups["pipe_bwd"] = self._build(self.topo.axis_groups("pipe"), "pipe_bwd") \
            if pp > 1 and pp_split_directions else self._groups["pipe"]

    def ctas_for(self, name):
        """Effective ``(min, max)`` CTA budget of group ``name`` (or None)."""
        c = self.ctas.get(name)
        if name == "model" and c is not None and not self._model_ctas_set:
            c = model_ctas(self.mp_degree)
        return c

    def pg_options(self, name):
        """RCCL options of group ``name`` (None on gloo or without a budget)."""
        return nccl_options(self.ctas_for(name)) if self._nccl else None

    def _build(self, rank_lists, name):
        mine = None
        opts = self.pg_options(name)
        for ranks in rank_lists:
            if self.initialized and len(ranks) > 1:
                g = dist.new_group(ranks=ranks, pg_options=opts) if opts is not None \
                    else dist.new_group(ranks=ranks)
                gg = dist.new_group(ranks=ranks, backend="gloo") if _want_gloo() else None
            else:
                g, gg = None, None
            if self.global_rank in ranks:
                mine = CommGroup(ranks, g, gg)
        return mine

    def _data_world_groups(self):
        t = self.topo
        groups = []
        for p in range(self.pp_degree):
            for m in range(self.mp_degree):
                ranks = [t.get_rank(data=d, pipe=p, sharding=s, model=m)
                         for d in range(self.dp_degree) for s in range(self.sharding_degree)]
                groups.append(ranks)
        return groups

    def _check_groups(self):
        t = self.topo
        groups = []
        for d in range(self.dp_degree):
            ranks = [t.get_rank(data=d, pipe=p, sharding=s, model=m)
                     for p in range(self.pp_degree) for s in range(self.sharding_degree)
                     for m in range(self.mp_degree)]
            groups.append(ranks)
        return groups

    def _embedding_groups(self):
        t = self.topo
        groups = []
        for d in range(self.dp_degree):
            for s in range(self.sharding_degree):
                for m in range(self.mp_degree):
                    first = t.get_rank(data=d, pipe=0, sharding=s, model=m)
                    last = t.get_rank(data=d, pipe=self.pp_degree - 1, sharding=s, model=m)
                    groups.append(sorted({first, last}))
        return groups

    # --- Paddle-like accessors -------------------------------------------
    def get_data_parallel_group(self):
        return self._groups["data"]

    def get_model_parallel_group(self):
        return self._groups["model"]

    def get_pipe_parallel_group(self):
        return self._groups["pipe"]

    def get_pipe_bwd_group(self):
        return self._groups["pipe_bwd"]

    def get_sharding_parallel_group(self):
        return self._groups["sharding"]

    def get_data_world_group(self):
        return self._groups["data_world"]

    def get_check_parallel_group(self):
        return self._groups["check"]

    def get_embedding_group(self):
        return self._groups["embedding"]

    def get_data_parallel_rank(self):
        return self.dp_rank

    def get_model_parallel_rank(self):
        return self.mp_rank

    def get_stage_id(self):
        return self.pp_rank

    def get_sharding_parallel_rank(self):
        return self.sharding_rank

    def get_data_parallel_world_size(self):
        return self.dp_degree

    def get_model_parallel_world_size(self):
        return self.mp_degree

    def get_pipe_parallel_world_size(self):
        return self.pp_degree

    def get_sharding_parallel_world_size(self):
        return self.sharding_degree

    def is_first_stage(self):
        return self.pp_rank == 0

    def is_last_stage(self):
        return self.pp_rank == self.pp_degree - 1

    def get_rank_from_stage(self, stage_id):
        return self.topo.get_rank(data=self.dp_rank, pipe=stage_id,
                                  sharding=self.sharding_rank, model=self.mp_rank)

    def __repr__(self):
        return ("HybridParallelInfo: rank_id: {}, dp_degree: {}, mp_degree: {}, pp_degree: {}, "
                "sharding_degree: {}, dp_group: {}, mp_group: {}, pp_group: {}, "
                "sharding_group: {}".format(
                    self.global_rank, self.dp_degree, self.mp_degree, self.pp_degree,
                    self.sharding_degree, self._groups["data"].ranks, self._groups["model"].ranks,
                    self._groups["pipe"].ranks, self._groups["sharding"].ranks))


def _want_gloo():
    return os.environ.get("FLEETX_GLOO_SIDE_GROUPS", "0") == "1"


def init_hcg(dp=1, mp=1, pp=1, sharding=1, pp_split_directions=False, ctas=None):
    global _HCG
    _HCG = HybridCommunicateGroup(dp=dp, mp=mp, pp=pp, sharding=sharding,
                                  pp_split_directions=pp_split_directions, ctas=ctas)
    return _HCG


def get_hcg():
    """Returns the active hybrid group, or a trivial single-rank one."""
    global _HCG
    if _HCG is None:
        ws = dist.get_world_size() if dist.is_initialized() else 1
        _HCG = HybridCommunicateGroup(dp=ws)
    return _HCG


def set_hcg(hcg):
    global _HCG
    _HCG = hcg


def reset_hcg():
    global _HCG
    _HCG = None
    from . import comm
    comm.reset()


_SERIAL = [0]


class serial_scope:
    """Layers built inside see a single-rank model-parallel world (full,
    unsplit weights): the semi-auto front end builds the serial network this
    way and partitions it from its shard annotations (parallel/auto/partition.py)."""

    def __enter__(self):
        _SERIAL[0] += 1
        return self

    def __exit__(self, *exc):
        _SERIAL[0] -= 1
        return False


def mp_group():
    return None if _SERIAL[0] else get_hcg().get_model_parallel_group()


def mp_world_size():
    return get_hcg().mp_degree if _HCG is not None and not _SERIAL[0] else 1


def mp_rank():
    return get_hcg().mp_rank if _HCG is not None and not _SERIAL[0] else 0


def init_distributed(backend=None, timeout_s=1800):
    """Initialise ``torch.distributed`` from the torchrun env contract.

    Backend defaults to ``nccl`` (RCCL) when a GPU is visible, else ``gloo``.
    The device for this rank is ``LOCAL_RANK``.
    """
    import datetime
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1 or dist.is_initialized():
        if torch.cuda.is_available():
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        return dist.is_initialized()
    if backend is None:
        # FLEETX_DIST_BACKEND=gloo rehearses multi-rank GPU code paths with
        # several ranks sharing one device (RCCL refuses duplicate GPUs)
        backend = os.environ.get("FLEETX_DIST_BACKEND") or \
            ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    kw = {}
    if backend == "nccl":
        kw["device_id"] = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return True

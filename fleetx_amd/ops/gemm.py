"""Linear-layer GEMMs on the hand-written gfx950 MFMA kernel (csrc/kernels/gemm.hip).

Three entry points cover the three GEMMs of a linear layer ``y = x W^T (+b)``
with the weight stored ``[out, in]``, each in its NATIVE layout (no transposed
copies):

* :func:`linear_fwd`   ``y = x W^T (+ b)``, optionally with the tanh/erf GeLU
  epilogue (returns ``(gelu(h), h)``; ``h`` is the pre-activation kept for the
  backward pass).  A = x ``[M][K]`` (k-contiguous), B = W ``[N][K]``.
* :func:`linear_dgrad` ``dx = dy W``, optionally times ``gelu'(h)`` in the
  epilogue (FC2's data gradient becomes FC1's dH directly).  A = dy
  ``[M][N]``, B = W read as ``[K=N][n=in]`` (mn-contiguous, hardware
  transposed LDS reads).
* :func:`linear_wgrad` ``main_grad (+)= dy^T x`` in fp32 (beta 0/1).  Both
  operands token-major (mn-contiguous).

Each returns ``None`` when the kernel does not cover the shape (K not a
multiple of 64, odd extents, non-unit inner strides, fp32 tensors); the
caller then uses hipBLASLt.  ``FLEETX_GEMM=hip`` routes every covered GEMM
here, ``blas`` none, ``auto`` (default) the kinds in ``FLEETX_GEMM_AUTO``.

Parity: the reference's ``FusedLinear`` / ``fused_gemm_epilogue``
(``gpt/dygraph/single_model.py:29,81,375``; ``language_model/utils.py:30-36``).
"""
import os

import torch

from . import _lib

LAY_KC, LAY_MC = 0, 1
EPI_STORE, EPI_BIAS_GELU, EPI_DGELU, EPI_F32, EPI_BIAS_GELU_ERF, EPI_DGELU_ERF, EPI_F32B, \
    EPI_F32BT = range(8)

_MODE = os.environ.get("FLEETX_GEMM", "auto")


def enabled():
    return _MODE != "blas"


def set_mode(mode):
    """'hip' (default), 'blas' (hipBLASLt everywhere) or 'auto' (per-kind table)."""
    global _MODE
    _MODE = mode


# GEMM kinds routed to the MFMA kernel under FLEETX_GEMM=auto.  The
# hand-scheduled 4-wave kernel (csrc/kernels/gemm5.hip) takes
#  * wgrad: the fp32-accumulating weight gradient in its native token-major
#    layout -- 1.23-1.43 PF against 1.01-1.18 PF for hipBLASLt's TN path plus
#    the two transposes it needs (profiles/r3_gemm/);
#  * dgrad (opt-in): the data gradient with the weight read in place
#    (hardware transposed LDS reads) -- 1.37-1.54 PF against 1.41-1.48 PF for
#    the TN path with its weight transpose in isolation, but 4 ms/step slower
#    in the 6.7B step on the same box (profiles/r3_step/routing_ab.txt);
#  * dgrad_act / fwd_act (opt-in): the GEMMs with a fused GeLU' / bias+GeLU
#    epilogue.  Measured in the 6.7B step they lose: the GeLU math runs with
#    the matrix pipe idle at one workgroup per CU (0.97 ms vs 0.77 ms for the
#    plain GEMM on FC2's data gradient, more than the 0.16 ms elementwise
#    pass they retire), and a forward GEMM that holds whole CUs starves the
#    forward-overlapped AdamW (profiles/r3_step/);
# forward GEMMs stay on hipBLASLt, whose TN kernels tie or lead there.
# Only shapes whose output fills the chip go to the kernel: >= 192 tiles of
# 128 x 128 (the kernel itself runs 256 x 256 tiles when there are >= 192 of
# those, else 128 x 128 tiles at two workgroups per CU, which is what the
# hidden 1024-2048 models and ViT-g use); FLEETX_GEMM_AUTO="kind,kind"
# replaces the set.
_DEFAULT_AUTO = "wgrad"


def default_auto_kinds():
    """The process default: ``FLEETX_GEMM_AUTO`` or the built-in table."""
    return os.environ.get("FLEETX_GEMM_AUTO", _DEFAULT_AUTO)


AUTO_KINDS = set(k for k in default_auto_kinds().split(",") if k)
MIN_TILES = int(os.environ.get("FLEETX_GEMM_MIN_TILES", "192"))
# weight gradients whose tiles underfill the chip run split along K
# (gemm5.hip g5_split_plan), so they may take smaller shapes
WGRAD_MIN_TILES = int(os.environ.get("FLEETX_GEMM_WGRAD_MIN_TILES", "64"))


def set_auto_kinds(kinds):
    """Replace the kinds routed under ``auto`` ('wgrad,dgrad' or a list)."""
    if isinstance(kinds, str):
        kinds = [k.strip() for k in kinds.split(",")]
    AUTO_KINDS.clear()
    AUTO_KINDS.update(k for k in kinds if k)


def _tiles(r, c, t=128):
    return ((r + t - 1) // t) * ((c + t - 1) // t)


def out_tiles(kind, a, b, t=128):
    """t x t output tiles of GEMM ``kind`` on operands (a, b) as passed to
    :func:`use`: fwd (x, w) -> [M, N]; dgrad (dy, w) -> [M, K]; wgrad (dy, x)
    -> [N, K]."""
    M = a.numel() // a.shape[-1]
    if kind.startswith("fwd"):
        return _tiles(M, b.shape[0], t)
    if kind.startswith("dgrad"):
        return _tiles(M, b.shape[1], t)
    return _tiles(a.shape[-1], b.shape[-1], t)


# Per-shape routing of the plain data-gradient GEMMs
# (FLEETX_GEMM_ROUTE=tune, the default; "off" keeps the kind table alone).
# Which of the MFMA kernel and hipBLASLt is faster depends on the shape
# (GPT-3 6.7B with the tuned tile order: QKV forward 1466 vs 1331 TF/s, FC1
# forward 1414 vs 1521; data gradients of QKV / out / FC1 lead, FC2 trails;
# profiles/r4_gm/).  The first call of a (kind, shape) outside stream capture
# times both paths (interleaved, a few launches each, on the caller's
# stream) and the kernel takes the shape only when it wins by ROUTE_MARGIN,
# so near-ties stay on one side from run to run.  The vendor path of a kind
# is registered by its caller (VENDOR).
# Forward GEMMs are not raced: their isolated timing misleads in the step.
# Beside the forward-overlapped AdamW a gemm5 wave takes its SIMD's whole
# register file, so the update cannot share those CUs: with the
# QKV forward on gemm5 (10 % faster alone) the 6.7B step takes 316-317 ms
# vs 293-295 (three interleaved runs each; ViT-g 461 vs 465 img/s;
# profiles/r4_route/fwd_race_ab.txt).  Even without the overlapped update
# (345M in its graph) the race's picks (out-proj, FC2 forward) made the step
# 0.1-0.3 ms slower (profiles/r4_route/fwd_race_345m.txt).
ROUTE_TUNE = os.environ.get("FLEETX_GEMM_ROUTE", "tune") == "tune"
TUNE_KINDS = ("dgrad",)
# Forward GEMMs follow the plan only (never raced): "plan" = an entry's
# "route" field; "faster" = also entries without one whose planned kernel time
# beats the vendor's by ROUTE_MARGIN (lab A/Bs); "off" = hipBLASLt.
FWD_ROUTE = os.environ.get("FLEETX_GEMM_FWD_ROUTE", "plan")
ROUTE_MARGIN = 0.03
VENDOR = {}
_ROUTE = {}
_ROUTE_SRC = {}  # key -> "plan" | "race" | "default"
PLAN_KINDS = ("fwd", "fwd_act", "dgrad", "dgrad_act", "wgrad")

# ----------------------------------------------------------------------------
# Shipped GEMM plan (reproducible routing; reference parity: the fused path is
# chosen at config time, ``models/language_model/utils.py:30-36,67-71``).
# ``gemm_plan_gfx950.json`` (tools/gemm_plan.py: many interleaved launches per
# candidate on an MI355X) holds, per (kind, dtype, M, N, K) of the model zoo's
# layer shapes, the route (MFMA kernel or vendor) and the tile-order M-group
# height.  Shapes in the plan are never raced or re-tuned, so one tree runs the
# same kernels with the same tile orders on every box and under a profiler;
# the first-call race / tune remains only for shapes the plan lacks, and not
# at all under FLEETX_DETERMINISTIC=1 (missing shapes: vendor path, gm 8).
# Key convention: M = rows of the activation (tokens), N = output columns,
# K = reduction; wgrad: M = tokens, N = out features, K = in features.
# ----------------------------------------------------------------------------
PLAN_FILE = os.environ.get("FLEETX_GEMM_PLAN",
                           os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                        "gemm_plan_gfx950.json"))
_PLAN = None  # {(kind, dtype, M, N, K): entry}


def _deterministic():
    return os.environ.get("FLEETX_DETERMINISTIC", "0") == "1"


_KIND_LAYOUT = {"fwd": (LAY_KC, LAY_KC, 0), "fwd_act": (LAY_KC, LAY_KC, 0),
                "dgrad": (LAY_KC, LAY_MC, 0), "dgrad_act": (LAY_KC, LAY_MC, 0),
                "wgrad": (LAY_MC, LAY_MC, 1)}


def kernel_shape(kind, M, N, K):
    """(la, lb, fp32 out, M, N, K) of the kernel launch for a plan key."""
    la, lb, f32 = _KIND_LAYOUT[kind]
    if kind == "wgrad":
        return la, lb, f32, N, K, M
    return la, lb, f32, M, N, K


# Vendor-GEMM solutions (hipBLASLt / rocBLAS, the forward and TN data-gradient
# GEMMs that stay on the library) picked per shape by PyTorch TunableOp on an
# MI355X for the single-GPU model zoo (scripts/gpu_r5_ar.sh).  Loaded read-only:
# shapes missing from the file run the library default.
# Opt-in (FLEETX_VENDOR_TUNE=on): its A/B is neutral at the 6.7B headline
# (288.17 vs 288.16 ms, profiles/r5_vendor_tune/) and it turns TunableOp on
# for every torch GEMM of the process; PYTORCH_TUNABLEOP_* set by the user win.
VENDOR_TUNE_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                "tunableop_gfx950.csv")


def enable_vendor_tuning():
    if os.environ.get("FLEETX_VENDOR_TUNE", "off") != "on" \
            or any(k.startswith("PYTORCH_TUNABLEOP") for k in os.environ) \
            or not torch.cuda.is_available() or not os.path.exists(VENDOR_TUNE_FILE):
        return False
    import torch.cuda.tunable as tunable
    tunable.enable(True)
    tunable.tuning_enable(False)
    tunable.record_untuned_enable(False)
    if not tunable.read_file(VENDOR_TUNE_FILE):
        tunable.enable(False)
        return False
    return True


def load_plan(path=None, force=False):
    """Read the plan (once) and preload its tile orders into the kernel
    library; returns {key: entry}.  A missing / foreign-arch plan is empty."""
    global _PLAN
    if _PLAN is not None and not force:
        return _PLAN
    enable_vendor_tuning()
    import json
    plan = {}
    path = path or PLAN_FILE
    try:
        with open(path) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        doc = {}
    arch = doc.get("arch", "gfx950")
    ok_arch = True
    if torch.cuda.is_available():
        name = getattr(torch.cuda.get_device_properties(0), "gcnArchName", "") or ""
        ok_arch = not name or name.split(":")[0] == arch
    if ok_arch:
        for e in doc.get("entries", []):
            key = (e["kind"], e.get("dtype", "bf16"), int(e["M"]), int(e["N"]), int(e["K"]))
            plan[key] = e
    _PLAN = plan
    if plan and _lib.available() and torch.cuda.is_available():
        k = _lib.kernels()
        for (kind, dt, M, N, K), e in plan.items():
            if e.get("gm"):
                k.gemm_set_tuned(*kernel_shape(kind, M, N, K), int(e["gm"]))
    if _deterministic() and _lib.available():
        _lib.kernels().gemm_set_tune(0)
    return plan


def _dt_name(dtype):
    return "bf16" if dtype == torch.bfloat16 else "fp16"


def _plan_entry(kind, dtype, M, N, K):
    """The plan entry of a shape; fp16 shapes the plan lacks take the bf16
    entry (same kernels, same MFMA cycle counts, same tile orders: the fp16
    O2 step otherwise raced the QKV data gradient onto hipBLASLt plus a
    transpose, +16 ms per 6.7B step, profiles/r6_fp16/)."""
    plan = load_plan()
    e = plan.get((kind, _dt_name(dtype), M, N, K))
    if e is None and dtype == torch.float16:
        e = plan.get((kind, "bf16", M, N, K))
    return e


def plan_route(kind, M, N, K, dtype):
    """True / False when the plan fixes the route of this shape, else None."""
    e = _plan_entry(kind, dtype, M, N, K)
    if e is None or "route" not in e:
        return None
    return e["route"] == "kernel"


def route_table():
    """{(kind, M, N, K): True if the MFMA kernel takes it} decided so far."""
    return {k[:4]: v for k, v in _ROUTE.items()}


def kernel_routes():
    """{"kind MxNxK": source} of every shape routed to the MFMA kernel so far
    (data gradients: "plan" / "race"; forwards: "plan"), for the bench line."""
    out = {}
    for k, v in _ROUTE.items():
        if v:
            out["%s %dx%dx%d" % k[:4]] = _ROUTE_SRC.get(k, "default")
    for k, v in _FWD_ROUTE.items():
        if v:
            out["%s %dx%dx%d" % k[:4]] = "plan"
    return dict(sorted(out.items()))


def route_sources():
    """{"plan": n, "race": n, "default": n}: where the routes came from."""
    out = {"plan": 0, "race": 0, "default": 0}
    for v in _ROUTE_SRC.values():
        out[v] += 1
    return out


def _race(f_hip, f_vendor, iters=3):
    if f_hip() is None:
        return False
    f_vendor()
    t = []
    for f in (f_hip, f_vendor, f_hip, f_vendor):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            f()
        e1.record()
        e1.synchronize()
        t.append(e0.elapsed_time(e1))
    return min(t[0], t[2]) < (1.0 - ROUTE_MARGIN) * min(t[1], t[3])


def _tuned_route(kind, a, b):
    a2 = a.reshape(-1, a.shape[-1])
    M = a2.shape[0]
    if kind == "fwd":
        N, K = b.shape[0], b.shape[1]
    else:
        N, K = b.shape[1], b.shape[0]
    key = (kind, M, N, K, a.dtype)
    r = _ROUTE.get(key)
    if r is not None:
        return r
    p = plan_route(kind, M, N, K, a.dtype)
    if p is not None:
        _ROUTE[key], _ROUTE_SRC[key] = p and _ok(a2, b), "plan"
        return _ROUTE[key]
    if out_tiles(kind, a, b) < MIN_TILES or kind not in VENDOR or not _ok(a2, b) \
            or _deterministic():
        _ROUTE[key], _ROUTE_SRC[key] = False, "default"
        return False
    if torch.cuda.is_current_stream_capturing():
        return False
    if kind == "fwd":
        r = _race(lambda: linear_fwd(a2, b), lambda: VENDOR["fwd"](a2, b))
    else:
        r = _race(lambda: linear_dgrad(a2, b), lambda: VENDOR["dgrad"](a2, b))
    _ROUTE[key], _ROUTE_SRC[key] = r, "race"
    return r


_FWD_ROUTE = {}  # forward routes from the plan (kept apart from the raced table)


def _planned_fwd_route(a, b):
    key = ("fwd", a.numel() // a.shape[-1], b.shape[0], b.shape[1], a.dtype)
    r = _FWD_ROUTE.get(key)
    if r is not None:
        return r
    e = _plan_entry("fwd", a.dtype, *key[1:4])
    r = False
    if e is not None:
        if "route" in e:
            r = e["route"] == "kernel"
        elif FWD_ROUTE == "faster" and e.get("vendor_ms") and e.get("kernel_ms"):
            r = e["kernel_ms"] < (1.0 - ROUTE_MARGIN) * e["vendor_ms"]
        r = r and _ok(a.reshape(-1, a.shape[-1]), b)
    _FWD_ROUTE[key] = r
    return r


def use(kind, a, b=None):
    """Whether GEMM ``kind`` ('fwd' | 'fwd_act' | 'dgrad' | 'dgrad_act' |
    'wgrad'; ``_act`` = with the GeLU / GeLU' epilogue) on these operands goes
    to the MFMA kernel (the kernel itself may still decline the shape)."""
    if _MODE == "blas" or not a.is_cuda or a.dtype not in (torch.bfloat16, torch.float16):
        return False
    if _MODE == "auto":
        if b is None:
            return False
        if kind in PLAN_KINDS and (kind in TUNE_KINDS or kind in AUTO_KINDS):
            load_plan()
        if kind in AUTO_KINDS:
            return out_tiles(kind, a, b) >= (WGRAD_MIN_TILES if kind == "wgrad" else MIN_TILES)
        if ROUTE_TUNE and kind in TUNE_KINDS:
            return _tuned_route(kind, a, b)
        if kind == "fwd" and FWD_ROUTE != "off":
            return _planned_fwd_route(a, b)
        return False
    return True


def _ok(*ts):
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda or t.dtype not in (torch.bfloat16, torch.float16) or t.dim() != 2 \
                or t.stride(1) != 1 or t.data_ptr() % 16 or t.stride(0) % 8:
            return False
    return True


def _launch(dt, la, lb, epi, M, N, K, A, lda, B, ldb, C, ldc, bias=None, aux=None, ldaux=0,
            beta=0, sq=None, ws=None):
    return _lib.kernels().gemm(dt, la, lb, epi, M, N, K, A.data_ptr(), lda, B.data_ptr(), ldb,
                               C.data_ptr(), ldc, _lib.ptr(bias), _lib.ptr(aux), ldaux, int(beta),
                               _lib.stream(), _lib.ptr(sq), _lib.ptr(ws))


def _splitk_ws(M, N, K, device):
    """Scratch for the split-K slices of an fp32 weight-gradient GEMM whose
    tiles do not fill whole waves of the chip (gemm5.hip ``g5_split_plan``:
    the leftover tiles are cut along K and summed in slice order by a combine
    launch); None when the shape runs unsplit."""
    n = _lib.kernels().gemm_ws_bytes(EPI_F32, M, N, K)
    return torch.empty(n // 4, device=device, dtype=torch.float32) if n else None


def sq_slots(n, k):
    """fp32 slots :func:`linear_wgrad` may write with ``sq`` for an [n, k]
    weight gradient: one per wave of every 128 x 128 tile (the 256-tile
    geometry uses the first quarter; slots it does not write keep their
    zero)."""
    return 4 * ((n + 127) // 128) * ((k + 127) // 128)


def linear_fwd(x2, w, bias=None, act=None, out=None):
    """``x2 [M,K] @ w[N,K]^T (+ bias)``; ``act`` in (None, 'gelu', 'gelu_erf').
    Returns ``y`` or ``(gelu(h), h)``; ``None`` if not covered."""
    if not enabled() or not _ok(x2, w) or w.dtype != x2.dtype:
        return None
    if bias is not None and (bias.dtype != x2.dtype or not bias.is_contiguous()):
        return None
    M, K = x2.shape
    N = w.shape[0]
    if w.shape[1] != K:
        raise ValueError("linear_fwd: shape mismatch {} x {}".format(tuple(x2.shape), tuple(w.shape)))
    y = out if out is not None else torch.empty(M, N, device=x2.device, dtype=x2.dtype)
    h = None
    if act is None:
        epi = EPI_STORE
    else:
        epi = EPI_BIAS_GELU if act == "gelu" else EPI_BIAS_GELU_ERF
        h = torch.empty(M, N, device=x2.device, dtype=x2.dtype)
    rc = _launch(_lib.dt_code(x2.dtype), LAY_KC, LAY_KC, epi, M, N, K, x2, x2.stride(0), w,
                 w.stride(0), y, N, bias, h, N)
    if rc != 0:
        return None
    _lib.maybe_sync()
    return y if act is None else (y, h)


def linear_dgrad(dy2, w, act_input=None, act="gelu", out=None):
    """``dy2 [M,N] @ w [N,K]`` (times ``gelu'(act_input)`` when given), into
    ``out`` (a contiguous [M, K] block) when given."""
    if not enabled() or not _ok(dy2, w, act_input) or w.dtype != dy2.dtype:
        return None
    M, N = dy2.shape
    K = w.shape[1]
    if w.shape[0] != N:
        raise ValueError("linear_dgrad: shape mismatch")
    if out is not None and (out.shape != (M, K) or not out.is_contiguous()
                            or out.dtype != dy2.dtype or out.data_ptr() % 16):
        return None
    dx = out if out is not None else torch.empty(M, K, device=dy2.device, dtype=dy2.dtype)
    epi = EPI_STORE
    ld_aux = 0
    if act_input is not None:
        epi = EPI_DGELU if act == "gelu" else EPI_DGELU_ERF
        ld_aux = act_input.stride(0)
    # C[M, K] = sum_n A[m, n] B[n, k]: A = dy (k-contig over n), B = w stored [n][k]
    rc = _launch(_lib.dt_code(dy2.dtype), LAY_KC, LAY_MC, epi, M, K, N, dy2, dy2.stride(0), w,
                 w.stride(0), dx, K, None, act_input, ld_aux)
    if rc != 0:
        return None
    _lib.maybe_sync()
    return dx


# 16-bit weight gradients wider than tall through the transposed product
# (linear_wgrad): 6.7B FC2 1365 -> 1460-1474 TF/s, step -1.1 to -2.3 ms,
# bitwise the plain order (profiles/r5_wgrad_t/).  FLEETX_GEMM_WGRAD_T=0 keeps
# the plain order.
WGRAD_T = os.environ.get("FLEETX_GEMM_WGRAD_T", "1") == "1"


def covers_wgrad(dy2, x2):
    """Whether :func:`linear_wgrad` takes ``dy2^T x2`` (same checks as the
    kernel: 16-bit token-major operands, tokens a multiple of 64, extents of
    8)."""
    if not enabled() or not _ok(dy2, x2) or dy2.dtype != x2.dtype:
        return False
    M, N = dy2.shape
    return M % 64 == 0 and M >= 64 and N % 8 == 0 and x2.shape[1] % 8 == 0 and N >= 8 \
        and x2.shape[1] >= 8


def linear_wgrad(dy2, x2, out32, accumulate, sq=None):
    """``out32[N,K] (+)= dy2[M,N]^T @ x2[M,K]`` in fp32.  Returns True if done.

    ``out32`` may also be 16-bit (the bf16 / fp16 gradient storage of
    ``Distributed.comm.grad_dtype``): fp32 accumulation, one rounding in the
    epilogue; with ``accumulate`` (micro-batches, pipeline schedules) the
    stored value joins the fp32 sum before that rounding.

    ``sq`` (fp32, :func:`sq_slots` long): the epilogue also writes the sums of
    squares of the values it stores (of the fp32 values for a 16-bit output),
    so the global gradient norm needs no second pass over this weight's
    gradient (parallel/grad_buffer.py, ``enable_fused_norm``).  Returns False
    when the kernel cannot (the caller then computes without it)."""
    if not enabled() or not _ok(dy2, x2) or dy2.dtype != x2.dtype:
        return False
    out16 = out32.dtype == dy2.dtype
    if (out32.dtype != torch.float32 and not out16) or not out32.is_contiguous():
        return False
    M, N = dy2.shape
    K = x2.shape[1]
    if out32.shape != (N, K):
        raise ValueError("linear_wgrad: out shape {} != {}".format(tuple(out32.shape), (N, K)))
    # C[N, K] = sum_m A[n, m] B[m, k]: A = dy stored [m][n], B = x stored [m][k]
    if sq is not None and (sq.dtype != torch.float32 or sq.numel() < sq_slots(N, K)):
        raise ValueError("linear_wgrad: sq needs {} fp32 slots".format(sq_slots(N, K)))
    rc = -1
    if out16 and N < K and WGRAD_T and not accumulate:
        # wide gradient (FC2: [4096, 16384]): run the transposed product
        # x^T dy, the FC1 operand order, and store it transposed.  The FC2 order
        # takes 46 % more L2 misses (profiles/r5_gemm_pmc/); -7 = the shape
        # would split along K, where only the plain order exists
        rc = _launch(_lib.dt_code(dy2.dtype), LAY_MC, LAY_MC, EPI_F32BT, K, N, M, x2,
                     x2.stride(0), dy2, dy2.stride(0), out32, K, sq=sq,
                     ws=_splitk_ws(K, N, M, dy2.device))
    if rc != 0:
        rc = _launch(_lib.dt_code(dy2.dtype), LAY_MC, LAY_MC, EPI_F32B if out16 else EPI_F32, N,
                     K, M, dy2, dy2.stride(0), x2, x2.stride(0), out32, K, beta=accumulate, sq=sq,
                     ws=_splitk_ws(N, K, M, dy2.device))
    if rc == 0:
        _lib.maybe_sync()
    return rc == 0


def wgrad_16(dy2, x2):
    """``dy2^T @ x2`` returned in the 16-bit input dtype (no main_grad)."""
    if not enabled() or not _ok(dy2, x2) or dy2.dtype != x2.dtype:
        return None
    M, N = dy2.shape
    K = x2.shape[1]
    out = torch.empty(N, K, device=dy2.device, dtype=dy2.dtype)
    rc = _launch(_lib.dt_code(dy2.dtype), LAY_MC, LAY_MC, EPI_STORE, N, K, M, dy2, dy2.stride(0),
                 x2, x2.stride(0), out, K)
    return out if rc == 0 else None


# ----------------------------------------------------------------------------
# decode-time skinny GEMM (csrc/kernels/decode_gemv.hip)
# ----------------------------------------------------------------------------
GV_BIAS, GV_GELU, GV_RES, GV_QKV = range(4)


def decode_linear(x, weight, bias=None, epi=GV_BIAS, res=None, qkv_cache=None, ln=None):
    """``x [M, K] @ weight[N, K]^T`` for M <= 16 rows on the weight-streaming
    MFMA GEMV, with the epilogue ``epi``: GV_BIAS (+b), GV_GELU (gelu_tanh(+b)),
    GV_RES (+b + res[M, N]) or GV_QKV (``qkv_cache = (k_cache, v_cache, pos)``:
    the packed [heads][3][head_dim] output is scattered -- q returned as [M, H*D],
    k/v written into the caches [M, maxlen, H, D] at ``pos`` [M]).

    ``ln = (weight, bias, eps)`` (GV_GELU / GV_QKV): ``x`` is the residual
    stream and its LayerNorm is fused into the GEMV as a prologue (the
    decoder layer's LN1 / LN2 then cost no launch of their own).

    Returns the output, or None when the kernel does not cover the shape (the
    caller then uses the general GEMM)."""
    if not x.is_cuda or x.dim() != 2 or x.shape[0] > 16 or x.dtype not in (torch.bfloat16,
                                                                            torch.float16):
        return None
    M, K = x.shape
    N = weight.shape[0]
    if weight.dtype != x.dtype or weight.stride(1) != 1 or x.stride(1) != 1 or K % 1024:
        return None
    if ln is not None and (ln[0].dtype != x.dtype or ln[1] is None or ln[1].dtype != x.dtype
                           or not ln[0].is_contiguous() or not ln[1].is_contiguous()
                           or epi not in (GV_GELU, GV_QKV)):
        return None
    k = _lib.kernels()
    kc = vc = pos = None
    heads = hd = maxlen = 0
    if epi == GV_QKV:
        kc, vc, pos = qkv_cache
        maxlen, heads, hd = kc.shape[1], kc.shape[2], kc.shape[3]
        assert N == 3 * heads * hd and kc.is_contiguous() and vc.is_contiguous()
        assert pos.dtype == torch.int64 and pos.numel() == M
        y = torch.empty(M, heads * hd, device=x.device, dtype=x.dtype)
    else:
        y = torch.empty(M, N, device=x.device, dtype=x.dtype)
    if res is not None:
        assert res.shape == (M, N) and res.stride(1) == 1
    nb = k.decode_gemv(_lib.dt_code(x.dtype), int(epi), M, N, K, x.data_ptr(), x.stride(0),
                       weight.data_ptr(), weight.stride(0), _lib.ptr(bias), _lib.ptr(res),
                       res.stride(0) if res is not None else 0, y.data_ptr(), y.stride(0),
                       _lib.ptr(kc), _lib.ptr(vc), _lib.ptr(pos), heads, hd, maxlen,
                       _lib.ptr(ln[0]) if ln is not None else 0,
                       _lib.ptr(ln[1]) if ln is not None else 0,
                       float(ln[2]) if ln is not None else 0.0, _lib.stream())
    if nb == 0:
        return None
    _lib.maybe_sync()
    return y

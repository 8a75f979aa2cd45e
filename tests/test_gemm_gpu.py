"""Numerics of the hand-written MFMA GEMM (csrc/kernels/gemm.hip) against a
plain PyTorch fp32 reference of the same op, every layout x epilogue, bf16 and
fp16, including edge tiles (M, N not multiples of 256) and K-tails."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(256, 256, 128), (512, 768, 1024), (296, 520, 192), (1024, 1000, 320), (64, 256, 128),
          (384, 260, 256),  # N % 8 == 4: the direct (unstaged) epilogue
          (4096, 3072, 512)]  # >= 192 256-tiles: the 256 x 256 geometry


def _rel(out, ref):
    return float((out.float() - ref).abs().max() / ref.abs().max().clamp_min(1e-6))


def _gelu(x, erf):
    return torch.nn.functional.gelu(x, approximate="none" if erf else "tanh")


def _gelu_grad(x, erf):
    x = x.detach().requires_grad_(True)
    y = _gelu(x, erf)
    (g,) = torch.autograd.grad(y.sum(), x)
    return g


@pytest.fixture(scope="module")
def gemm():
    from fleetx_amd.ops import gemm as G
    from fleetx_amd.ops import _lib
    _lib.kernels()
    old = G._MODE
    G.set_mode("hip")
    yield G
    G.set_mode(old)  # later modules pick their GEMM routing on purpose


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_fwd_store_bias(gemm, M, N, K, dtype):
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda", dtype=dtype)
    w = torch.randn(N, K, device="cuda", dtype=dtype) * 0.05
    b = torch.randn(N, device="cuda", dtype=dtype)
    ref = x.float() @ w.float().t()
    y = gemm.linear_fwd(x, w)
    assert y is not None
    assert _rel(y, ref) < 1e-2
    yb = gemm.linear_fwd(x, w, b)
    assert _rel(yb, ref + b.float()) < 1e-2


@pytest.mark.parametrize("erf", [False, True])
@pytest.mark.parametrize("M,N,K", SHAPES[:3])
def test_fwd_bias_gelu(gemm, M, N, K, erf):
    torch.manual_seed(1)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    h_ref = x.float() @ w.float().t() + b.float()
    y, h = gemm.linear_fwd(x, w, b, act="gelu_erf" if erf else "gelu")
    assert _rel(h, h_ref) < 1e-2
    assert _rel(y, _gelu(h_ref, erf)) < 1e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_dgrad(gemm, M, N, K, dtype):
    # dx[M, K] = dy[M, N] @ w[N, K]
    torch.manual_seed(2)
    dy = torch.randn(M, N, device="cuda", dtype=dtype)
    w = torch.randn(N, K, device="cuda", dtype=dtype) * 0.05
    if N % 64 or K % 8:
        assert gemm.linear_dgrad(dy, w) is None
        return
    dx = gemm.linear_dgrad(dy, w)
    assert dx is not None
    assert _rel(dx, dy.float() @ w.float()) < 1e-2


@pytest.mark.parametrize("erf", [False, True])
def test_dgrad_dgelu(gemm, erf):
    torch.manual_seed(3)
    M, N, K = 512, 1024, 768
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    h = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    dx = gemm.linear_dgrad(dy, w, act_input=h, act="gelu_erf" if erf else "gelu")
    ref = (dy.float() @ w.float()) * _gelu_grad(h.float(), erf)
    assert _rel(dx, ref) < 1e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (1024, 768, 512), (320, 520, 296),
                                   (2048, 1000, 256)])
def test_wgrad_f32(gemm, M, N, K, dtype):
    # out[N, K] (+)= dy[M, N]^T x[M, K]  -- reduction over the M tokens
    torch.manual_seed(4)
    dy = torch.randn(M, N, device="cuda", dtype=dtype)
    x = torch.randn(M, K, device="cuda", dtype=dtype)
    out = torch.randn(N, K, device="cuda", dtype=torch.float32)
    base = out.clone()
    ref = dy.float().t() @ x.float()
    if M % 64:
        assert not gemm.linear_wgrad(dy, x, out, False)
        return
    assert gemm.linear_wgrad(dy, x, out, False)
    assert _rel(out, ref) < 1e-4
    out.copy_(base)
    assert gemm.linear_wgrad(dy, x, out, True)
    assert _rel(out, ref + base) < 1e-4


@pytest.mark.parametrize("M,N,K", [(1024, 768, 512), (2048, 1000, 256), (256, 4096, 4096)])
def test_wgrad_norm_partials(gemm, M, N, K):
    # the fp32 epilogue's per-wave sums of squares add up to |out|^2 of the
    # values it stored, for beta 0 and beta 1; slots it does not own stay 0
    # ((256, 4096, 4096) runs the 256-tile geometry, the others 128-tiles)
    torch.manual_seed(5)
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    out = torch.randn(N, K, device="cuda", dtype=torch.float32)
    sq = torch.zeros(gemm.sq_slots(N, K) + 16, device="cuda")
    sq[-16:] = 7.0  # guard: never written
    assert gemm.linear_wgrad(dy, x, out, True, sq=sq[:-16])
    ref = out.double().pow(2).sum()
    assert abs(float(sq[:-16].double().sum()) - float(ref)) < 1e-5 * float(ref)
    assert torch.all(sq[-16:] == 7.0)
    assert gemm.linear_wgrad(dy, x, out, False, sq=sq[:-16])
    ref = out.double().pow(2).sum()
    assert abs(float(sq[:-16].double().sum()) - float(ref)) < 1e-5 * float(ref)
    with pytest.raises(ValueError):
        gemm.linear_wgrad(dy, x, out, False, sq=sq[:8])


@pytest.mark.parametrize("M,N,K", [(16448, 6144, 1408), (16448, 1408, 1408), (8192, 1024, 1024)])
def test_wgrad_splitk(gemm, M, N, K):
    """fp32 weight gradients whose tiles leave the last wave of the chip
    mostly empty run their leftover tiles split along K (gemm5.hip
    g5_split_plan; ViT-g FC1: 528 tiles on 512 slots -> 16 tiles x 32 slices)
    and sum the slices in slice order: against fp32 torch for beta 0 / 1,
    norm partials included, and bitwise repeatable."""
    from fleetx_amd.ops import _lib
    assert _lib.kernels().gemm_ws_bytes(gemm.EPI_F32, N, K, M) > 0
    torch.manual_seed(7)
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    ref = dy.float().t() @ x.float()
    base = torch.randn(N, K, device="cuda", dtype=torch.float32)
    out = base.clone()
    sq = torch.zeros(gemm.sq_slots(N, K), device="cuda")
    assert gemm.linear_wgrad(dy, x, out, True, sq=sq)
    assert _rel(out, base + ref) < 1e-4
    assert abs(float(sq.double().sum()) - float(out.double().pow(2).sum())) < 1e-5 * float(out.double().pow(2).sum())
    out2 = torch.empty_like(out)
    assert gemm.linear_wgrad(dy, x, out2, False)
    assert _rel(out2, ref) < 1e-4
    out3 = torch.empty_like(out)
    assert gemm.linear_wgrad(dy, x, out3, False)
    assert torch.equal(out2, out3)


def test_strided_rows(gemm):
    """Row-strided activations (a column slice of a wider buffer) are read in place."""
    torch.manual_seed(5)
    big = torch.randn(512, 1024, device="cuda", dtype=torch.bfloat16)
    x = big[:, 256:768]
    w = torch.randn(384, 512, device="cuda", dtype=torch.bfloat16) * 0.05
    y = gemm.linear_fwd(x, w)
    assert _rel(y, x.float() @ w.float().t()) < 1e-2


def test_uncovered_shapes_fall_back(gemm):
    x = torch.randn(64, 100, device="cuda", dtype=torch.bfloat16)   # K % 64 != 0
    w = torch.randn(128, 100, device="cuda", dtype=torch.bfloat16)
    assert gemm.linear_fwd(x, w) is None
    xf = torch.randn(64, 128, device="cuda")
    assert gemm.linear_fwd(xf, xf) is None


def test_gelu_without_bias(gemm):
    torch.manual_seed(6)
    x = torch.randn(512, 256, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(768, 256, device="cuda", dtype=torch.bfloat16) * 0.05
    h_ref = x.float() @ w.float().t()
    y, h = gemm.linear_fwd(x, w, None, act="gelu")
    assert _rel(h, h_ref) < 1e-2
    assert _rel(y, _gelu(h_ref, False)) < 1e-2


@pytest.mark.parametrize("K", [128, 192])
def test_persistent_many_tiles(gemm, K):
    """More tiles than CUs: each workgroup walks several tiles with the staging
    stream running across tile boundaries (odd and even K-tile counts)."""
    torch.manual_seed(7)
    M, N = 4608, 4352                     # 18 x 17 = 306 tiles of 256x256
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    ref = x.float() @ w.float().t() + b.float()
    assert _rel(gemm.linear_fwd(x, w, b), ref) < 1e-2
    y, h = gemm.linear_fwd(x, w, b, act="gelu")
    assert _rel(h, ref) < 1e-2 and _rel(y, _gelu(ref, False)) < 1e-2
    # dgrad over the same sizes: dx[M, K2] = dy[M, N] w2[N, K2] with N % 64 == 0
    w2 = torch.randn(N, 4352, device="cuda", dtype=torch.bfloat16) * 0.05
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    hh = torch.randn(M, 4352, device="cuda", dtype=torch.bfloat16)
    dx = gemm.linear_dgrad(dy, w2, act_input=hh)
    assert _rel(dx, (dy.float() @ w2.float()) * _gelu_grad(hh.float(), False)) < 1e-2
    # wgrad with accumulate: out[N, K] += dy^T x over M tokens
    out = torch.randn(N, K, device="cuda", dtype=torch.float32)
    base = out.clone()
    assert gemm.linear_wgrad(dy, x, out, True)
    assert _rel(out, dy.float().t() @ x.float() + base) < 1e-4


def test_tile_order_autotune_is_bitwise_neutral(gemm):
    """The tuned tile-order M-group (csrc/kernels/gemm.hip gemm_tuned_gm)
    changes only which workgroup computes which tile: outputs are bitwise
    those of the default order, and the shape lands in the tuned table."""
    from fleetx_amd.ops import _lib
    k = _lib.kernels()
    torch.manual_seed(11)
    M, N, K = 4096, 3072, 1024
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    outs = []
    for gm in (8, 0, 1):          # forced default, tuned, forced 1
        k.gemm_set_gm(gm)
        o32 = torch.zeros(N, K, device="cuda", dtype=torch.float32)
        assert gemm.linear_wgrad(dy, x, o32, False)
        outs.append((gemm.linear_fwd(x, w), gemm.linear_dgrad(dy, w), o32))
    k.gemm_set_gm(0)
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    for a, b in zip(outs[0], outs[2]):
        assert torch.equal(a, b)
    tuned = {(r[0], r[1], r[2], r[3], r[4], r[5]): r[6] for r in k.gemm_tuned()}
    assert (1, 1, 1, N, K, M) in tuned and tuned[(1, 1, 1, N, K, M)] in (1, 2, 4, 8, 16)


def test_route_tuner_picks_a_path_and_both_agree():
    """Per-shape routing of plain data-gradient GEMMs (ops/gemm.py
    _tuned_route): the first call of a shape races the MFMA kernel against the
    registered vendor path, caches the winner, and either path matches fp32."""
    from fleetx_amd.ops import gemm as G
    from fleetx_amd.parallel import linear as L
    old = (G._MODE, G.ROUTE_TUNE, set(G.AUTO_KINDS))
    try:
        G.set_mode("auto")
        G.ROUTE_TUNE = True
        G.set_auto_kinds("wgrad")
        torch.manual_seed(12)
        M, N, K = 4096, 6144, 1024
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
        dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        y = L.fwd_gemm(x, w)
        dx = L.dgrad_gemm(dy, w)
        table = G.route_table()
        # data gradients race; forward GEMMs do not (see ops/gemm.py)
        assert ("dgrad", M, K, N) in table and ("fwd", M, N, K) not in table
        assert _rel(y, x.float() @ w.float().t()) < 1e-2
        assert _rel(dx, dy.float() @ w.float()) < 1e-2
        # small outputs never race (under MIN_TILES): vendor path, cached False
        dys = torch.randn(256, 512, device="cuda", dtype=torch.bfloat16)
        L.dgrad_gemm(dys, w[:512])
        assert G.route_table()[("dgrad", 256, K, 512)] is False
    finally:
        G.set_mode(old[0])
        G.ROUTE_TUNE = old[1]
        G.set_auto_kinds(old[2])


@pytest.mark.parametrize("nf,split", [(4, 1), (4, 3), (8, 2), (8, 1)])
def test_wgrad_forced_geometry(gemm, nf, split):
    """The lab geometry / split-K override (fx_gemm_set_geom) used by
    tools/bench_gemm.py --geom: every forced plan computes the same product."""
    from fleetx_amd.ops import _lib
    k = _lib.kernels()
    torch.manual_seed(13)
    M, N, K = 2048, 1024, 768
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    base = torch.randn(N, K, device="cuda", dtype=torch.float32)
    try:
        k.gemm_set_geom(nf, split)
        out = base.clone()
        assert gemm.linear_wgrad(dy, x, out, True)
    finally:
        k.gemm_set_geom(0, 0)
    assert _rel(out, base + dy.float().t() @ x.float()) < 1e-4


# Persistent 16-bit launches (gemm5 ``P.qslot``): more tiles than resident
# workgroups, pulled from per-XCD queues.  (4096, 6144, 256): 384 tiles of
# 256 on 256 workgroups; (2560, 4608, 256): 720 tiles of 128 on 512.
PERSIST_SHAPES = [(4096, 6144, 256), (2560, 4608, 256)]


@pytest.fixture
def persist_mode(gemm):
    from fleetx_amd.ops import _lib
    yield _lib.kernels().gemm_set_persist
    _lib.kernels().gemm_set_persist(-1)


@pytest.mark.parametrize("M,N,K", PERSIST_SHAPES)
def test_persistent_matches_one_tile_per_workgroup(gemm, persist_mode, M, N, K):
    """Every tile is computed exactly once whichever workgroup pulls it: the
    persistent launch is bitwise the one-workgroup-per-tile launch, for the
    forward (bias + GeLU epilogue too) and the data gradient."""
    torch.manual_seed(6)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    w2 = torch.randn(N, 512, device="cuda", dtype=torch.bfloat16) * 0.05
    outs = {}
    for mode in (0, 1):
        persist_mode(mode)
        y = gemm.linear_fwd(x, w, b)
        g, h = gemm.linear_fwd(x, w, b, act="gelu")
        dx = gemm.linear_dgrad(dy, w2)
        outs[mode] = (y, g, h, dx)
    for a, c in zip(outs[0], outs[1]):
        assert torch.equal(a, c)
    ref = x.float() @ w.float().t() + b.float()
    assert _rel(outs[1][0], ref) < 1e-2
    assert _rel(outs[1][3], dy.float() @ w2.float()) < 1e-2


def test_persistent_queue_slots_recycle(gemm, persist_mode):
    """More launches than queue slots (4096): each launch re-zeroes its slot,
    so a reused slot starts from an empty queue (a stale count would skip
    tiles and leave the output partly unwritten)."""
    persist_mode(1)
    torch.manual_seed(7)
    M, N, K = 2560, 4608, 128
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    ref = gemm.linear_fwd(x, w)
    out = torch.empty_like(ref)
    for i in range(4200):
        if i % 700 == 0:
            out.fill_(float("nan"))
        gemm.linear_fwd(x, w, out=out)
        if i % 700 == 699:
            assert torch.equal(out, ref), i
    torch.cuda.synchronize()


def test_persistent_two_streams(gemm, persist_mode):
    """Two persistent GEMMs in flight on two streams use different slots."""
    persist_mode(1)
    torch.manual_seed(8)
    M, N, K = 4096, 6144, 256
    xs = [torch.randn(M, K, device="cuda", dtype=torch.bfloat16) for _ in range(2)]
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    refs = [x.float() @ w.float().t() for x in xs]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    ys = [None, None]
    for _ in range(20):
        with torch.cuda.stream(s):
            ys[1] = gemm.linear_fwd(xs[1], w)
        ys[0] = gemm.linear_fwd(xs[0], w)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    for y, r in zip(ys, refs):
        assert _rel(y, r) < 1e-2


@pytest.mark.parametrize("act", [None, "gelu"])
def test_persistent_under_memory_pressure(gemm, persist_mode, act):
    """Persistent launches while another stream saturates HBM (as the
    forward-overlapped AdamW does in the step): the next tile's K-tiles are
    issued before the current tile's epilogue and MAIN waits for them with a
    counted vmcnt; under long load latencies a wrong count reads stale LDS.
    Bitwise against one-workgroup-per-tile, repeated."""
    torch.manual_seed(9)
    M, N, K = 8192, 6144, 4096
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    persist_mode(0)
    ref = gemm.linear_fwd(x, w, b, act=act)
    ref = ref if act is None else ref[0]
    persist_mode(1)
    big = torch.empty(1 << 29, device="cuda", dtype=torch.float32)  # 2 GiB
    dst = torch.empty_like(big)
    s = torch.cuda.Stream()
    for _ in range(6):
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(4):
                dst.copy_(big)
        y = gemm.linear_fwd(x, w, b, act=act)
        y = y if act is None else y[0]
        torch.cuda.current_stream().wait_stream(s)
        assert torch.equal(y, ref)
    torch.cuda.synchronize()


@pytest.mark.parametrize("M,N,K", [(1024, 768, 512), (8192, 1024, 1024), (16448, 1408, 1408),
                                   (256, 4096, 4096), (2048, 1024, 4096)])
def test_wgrad_16bit_out(gemm, M, N, K):
    """EPI_F32B: the weight gradient written in bf16 from the fp32
    accumulators (16-bit gradient storage), split-K shapes included; the norm
    partials are the sums of squares of the fp32 values; with accumulate the
    stored value is added before the rounding."""
    torch.manual_seed(10)
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    ref = dy.float().t() @ x.float()
    out = torch.full((N, K), float("nan"), device="cuda", dtype=torch.bfloat16)
    sq = torch.zeros(gemm.sq_slots(N, K), device="cuda")
    assert gemm.linear_wgrad(dy, x, out, False, sq=sq)
    assert _rel(out, ref) < 1e-2
    # one rounding of the fp32 result: as close to it as bf16 allows
    assert torch.equal(out, ref.to(torch.bfloat16)) or \
        float((out.float() - ref).abs().max()) <= float(ref.abs().max()) * 2 ** -7
    assert abs(float(sq.double().sum()) - float(ref.double().pow(2).sum())) < \
        1e-4 * float(ref.double().pow(2).sum())
    # accumulation (micro-batches / pipeline schedules): the stored gradient
    # joins the fp32 sum, one rounding per write
    prev = out.clone()
    assert gemm.linear_wgrad(dy, x, out, True)
    want = (prev.float() + ref).to(torch.bfloat16)
    assert float((out.float() - want.float()).abs().max()) <= \
        float(want.float().abs().max()) * 2 ** -7


# XCD rectangles (gemm5 ``P.xm``, FLEETX_GEMM_XRECT): each XCD's range of tile
# ids is one rectangle of the tile grid.  A permutation of which workgroup
# computes which tile: bitwise the plain order for every kind (persistent and
# one-per-tile forwards, data gradients, split-K fp32 and 16-bit weight
# gradients).  Shapes whose 256- / 128-tile grids cut into 8 equal rectangles.
@pytest.fixture
def xrect_mode(gemm):
    from fleetx_amd.ops import _lib
    yield _lib.kernels().gemm_set_xrect
    _lib.kernels().gemm_set_xrect(-1)


@pytest.mark.parametrize("M,N,K", [(4096, 6144, 512), (2048, 2048, 1024), (8192, 1024, 1024)])
def test_xcd_rectangles_are_bitwise_the_plain_order(gemm, persist_mode, xrect_mode, M, N, K):
    torch.manual_seed(11)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    outs = {}
    for xr in (2, 1):  # forced off / on
        xrect_mode(xr)
        res = []
        for pm in (0, 1):
            persist_mode(pm)
            res.append(gemm.linear_fwd(x, w, b))
        res.append(gemm.linear_fwd(x, w, b, act="gelu")[0])
        res.append(gemm.linear_dgrad(dy, w))
        dw = torch.empty(N, K, device="cuda", dtype=torch.float32)
        assert gemm.linear_wgrad(dy, x, dw, False)
        res.append(dw)
        dw16 = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        assert gemm.linear_wgrad(dy, x, dw16, False)
        res.append(dw16)
        outs[xr] = res
    for a, c in zip(outs[2], outs[1]):
        assert torch.equal(a, c)
    assert _rel(outs[1][0], x.float() @ w.float().t() + b.float()) < 1e-2
    assert _rel(outs[1][4], dy.float().t() @ x.float()) < 1e-3


@pytest.mark.parametrize("M,N,K", [(4096, 16384, 512), (2048, 8192, 1024)])
def test_tile_order_codes_are_bitwise_equal(gemm, M, N, K):
    """Every tile-order code (M-group height, XCD rectangles, the runner-up
    rectangle cut) computes each tile with the same arithmetic."""
    from fleetx_amd.ops import _lib
    k = _lib.kernels()
    torch.manual_seed(12)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    outs = []
    try:
        for code in (1, 4, 33, 36, 97, 100):
            k.gemm_set_gm(code)
            dw = torch.empty(N, K, device="cuda", dtype=torch.float32)
            assert gemm.linear_wgrad(dy, x, dw, False)
            outs.append((gemm.linear_fwd(x, w), gemm.linear_dgrad(dy, w), dw))
    finally:
        k.gemm_set_gm(0)
    for o in outs[1:]:
        for a, c in zip(outs[0], o):
            assert torch.equal(a, c)


@pytest.mark.parametrize("shape", [(1024, 3072, 4096), (512, 512, 2048)])
def test_wgrad_transposed_store_matches_plain(shape):
    """A 16-bit weight gradient wider than tall (N < K) through the transposed
    product x^T dy with the transposed store (EPI_F32BT, ops/gemm.py
    linear_wgrad under FLEETX_GEMM_WGRAD_T) equals the plain order bitwise,
    and its norm partials sum to the same total.  The second shape would split
    along K, so the kernel declines (-7) and the plain order runs."""
    from fleetx_amd.ops import gemm as G
    T, N, K = shape
    torch.manual_seed(3)
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    outs, sqs = [], []
    old = G.WGRAD_T
    try:
        for on in (False, True):
            G.WGRAD_T = on
            out = torch.full((N, K), float("nan"), device="cuda", dtype=torch.bfloat16)
            sq = torch.zeros(G.sq_slots(N, K), device="cuda", dtype=torch.float32)
            assert G.linear_wgrad(dy, x, out, False, sq=sq)
            outs.append(out)
            sqs.append(sq)
    finally:
        G.WGRAD_T = old
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref = (dy.float().t() @ x.float())
    assert _rel(outs[1], ref) < 1e-2
    s0, s1 = float(sqs[0].double().sum()), float(sqs[1].double().sum())
    assert abs(s0 - s1) <= 1e-5 * s0, (s0, s1)

"""Generates csrc/kernels/gemm_asm.inc: the hand-scheduled K-loop of the
4-wave gfx950 GEMM (``gemm5_kernel`` in csrc/kernels/gemm.hip).

Why a generator: the loop is one inline-asm statement (hipcc cannot be told to
keep 16 LDS-DMA loads, 32-64 LDS fragment reads, 4 barriers and counted
vmcnt/lgkmcnt waits spread between 128 MFMAs per K-tile -- it clusters them,
and a cluster of LDS-DMA issues starves the matrix pipe at one wave per SIMD).
The instruction stream is written out here with the waits computed by a small
scoreboard, so a schedule edit is a parameter change, not a hand edit.

Structure (per workgroup: 256 threads = 4 waves as 2 x 2, each wave owns a
128 x 128 block of C as 8 x 8 v_mfma_f32_16x16x32 tiles = 256 AGPRs):

* K-tile = 64: A 256 x 64 and B 256 x 64 staged HBM -> LDS by
  ``buffer_load_dwordx4 ... lds`` (32 KiB each, 8 per wave per operand), two
  LDS buffers of 64 KiB; tile t+2 is staged into the buffer of tile t as soon
  as each half of it has been read into registers.
* fragments are double-buffered in VGPRs (k-step 0 / 1 of 32): the k-step 1
  fragments of tile t are read under k-step 0's MFMAs, the k-step 0
  fragments of tile t+1 under k-step 1's.
* four segments of 32 MFMAs per K-tile, each closed by ``s_barrier`` issued
  right behind an MFMA (the matrix pipe runs through the barrier):
    S1  k0 rows 0-3   + B k1 reads            -> B half of the buffer free
    S2  k0 rows 4-7   + A k1 reads, B(t+2) DMA -> A half free
    S3  k1 rows 0-3   + A(t+2) DMA             -> vmcnt: B(t+1) landed
    S4  k1 rows 4-7   + B(t+1) k0 reads | vmcnt: A(t+1) landed | A(t+1) k0 reads

Layouts (per operand, 256 rows of the tile x 64 k):
  KC (k-contiguous, [rows][K]): LDS [row][128 B], 16-B chunk c of row r holds
     global chunk c ^ ((r >> 1) & 7) -> ds_read_b128 conflict-free.
  MC (mn-contiguous, [K][rows]): LDS [mq 4][khi 8][mr 4][pos 8][32 B] with
     m-block 4 mq + mr of 16 columns, k = 8 khi + klo, pos = klo ^ (khi & 1) * 4;
     one DMA = 8 k-rows x 64 columns (128-B global rows), fragments by
     ds_read_b64_tr_b16 (conflict-free, every fragment an immediate offset).

    python tools/gen_gemm_asm.py          (rewrites csrc/kernels/gemm_asm.inc)
"""
import os
import sys

KC, MC = 0, 1
# schedule knobs (per generated stream): dma_off = this wave's DMA slot shift
CFG = {"dma_off": 0, "dma_start": 0, "stagger": 1}
# Geometry of the stream being generated (set_geometry):
#   T256: 256 x 256 workgroup tile, 4 waves of 128 x 128 (8 x 8 fragments),
#         fragments in v[128:255], two 64 KiB LDS buffers, 1 workgroup per CU;
#   T128: 128 x 128 tile, 4 waves of 64 x 64 (4 x 4 fragments), fragments in
#         v[64:127], two 32 KiB buffers, 2 workgroups per CU (their waves
#         cover each other's LDS-DMA issue).
GEO = {}


def set_geometry(tag):
    nf = 8 if tag == "T256" else 4
    fb = 128 if nf == 8 else 64
    n = 4 * nf  # registers per (operand, k-step) fragment set
    GEO.clear()
    GEO.update(tag=tag, nf=nf, buf=2 * (32 * nf) * 128,
               frag_base={("A", 0): fb, ("A", 1): fb + n, ("B", 0): fb + 2 * n,
                          ("B", 1): fb + 3 * n})


def FRAG(op, s):
    return GEO["frag_base"][(op, s)]


class Stream:
    """Instruction list with an LDS-read scoreboard (lgkmcnt)."""

    def __init__(self):
        self.lines = []
        self.pending = []  # frag keys of outstanding LDS reads, oldest first

    def emit(self, s):
        self.lines.append(s)

    def read(self, key, text):
        self.lines.append(text)
        self.pending.append(key)

    def need(self, keys):
        idx = -1
        for pos, k in enumerate(self.pending):
            if k in keys:
                idx = pos
        if idx < 0:
            return
        n = len(self.pending) - 1 - idx
        n = min(n, 15)
        self.lines.append("s_waitcnt lgkmcnt(%d)" % n)
        self.pending = self.pending[len(self.pending) - n:] if n else []

    def drain(self):
        if self.pending:
            self.lines.append("s_waitcnt lgkmcnt(0)")
        self.pending = []


def vreg(base, n):
    return "v[%d:%d]" % (base, base + n - 1)


def read_ops(lay, op, s, i, which):
    """LDS reads of fragment i (k-step s) of operand op ('A'/'B') from the
    buffer addressed by base set `which` ('cur' / 'nxt')."""
    dst = FRAG(op, s) + 4 * i
    key = (op, s, i)
    if lay == KC:
        base = "%%[r%s_%s]" % (op, which)   # KC bases: cur = k-step 1, nxt = k-step 0
        return [(key, "ds_read_b128 %s, %s offset:%d" % (vreg(dst, 4), base, 2048 * i))]
    off = (i >> 2) * 8192 + (i & 3) * 256 + s * 4096
    lo = "%%[r%s_%slo]" % (op, which)
    hi = "%%[r%s_%shi]" % (op, which)
    return [(key, "ds_read_b64_tr_b16 %s, %s offset:%d" % (vreg(dst, 2), lo, off)),
            (key, "ds_read_b64_tr_b16 %s, %s offset:%d" % (vreg(dst + 2, 2), hi, off))]


def dma_ops(op, nop=False):
    """nf LDS-DMA loads of operand op for the next-but-one K-tile (M0 = this
    wave's nf KiB slice of the operand's region in the buffer being refilled).
    Returns (m0_setup, [[load, m0 advance], ...]).  An SALU write of M0 needs
    one wait state before an LDS-DMA reads it: in the loop the advance is
    followed by MFMAs; `nop` pads it for back-to-back issue."""
    pad = ["s_nop 0"] if nop else []
    groups = []
    nu = GEO["nf"]
    for u in range(nu):
        g = ["buffer_load_dwordx4 %%[vo%s%d], %%[rs%s], %%[so%s] offen lds" % (op, u, op, op)]
        if u < nu - 1:
            g += ["s_add_u32 m0, m0, 1024"] + pad
        groups.append(g)
    return ["s_mov_b32 m0, %%[m%s]" % op, "s_nop 0"], groups


def mfma(dt, st, s, i, j):
    st.need({("A", s, i), ("B", s, j)})
    k = GEO["nf"] * i + j
    mn = "v_mfma_f32_16x16x32_bf16" if dt == "bf16" else "v_mfma_f32_16x16x32_f16"
    st.emit("%s %%%d, %s, %s, %%%d" % (mn, k, vreg(FRAG("B", s) + 4 * j, 4),
                                       vreg(FRAG("A", s) + 4 * i, 4), k))


def segment(dt, st, s, rows, extras, read_gap, dma_gap, close=None, mf=None):
    """MFMAs of k-step s for fragment rows `rows` (x nf columns) -- or the
    explicit (s, i, j) list `mf` -- with `extras` (list of ('read', [(key,
    text)...]) / ('dma', (setup, groups))) interleaved: reads one per
    `read_gap` MFMAs from the start, DMA loads one per `dma_gap` MFMAs.
    `close` = wait line ('lgkm0' = drain the scoreboard) emitted before the
    last MFMA, followed by s_barrier after it."""
    if mf is None:
        mf = [(s, i, j) for i in rows for j in range(GEO["nf"])]
    reads = [x for kind, xs in extras if kind == "read" for x in xs]
    setup, groups = [], []
    for kind, xs in extras:
        if kind == "dma":
            setup += xs[0]
            groups += xs[1]
    plan = {p: [] for p in range(len(mf))}
    for n, r in enumerate(reads):
        plan[min(len(mf) - 2, n * read_gap)].append(("read", r))
    # DMA slots: one per dma_gap MFMAs, shifted by this wave's offset so the
    # four waves of a workgroup (in step between barriers) do not queue their
    # LDS-DMA issues at the CU's address unit at the same time
    start = CFG["dma_start"] + CFG["dma_off"]
    for n, g in enumerate(groups):
        plan[min(len(mf) - 2, start + n * dma_gap)].append(("dma", g))
    for t in setup:
        st.emit(t)
    for p, (ss, i, j) in enumerate(mf):
        if close is not None and p == len(mf) - 1:
            if close == "lgkm0":
                st.drain()
            elif close:
                st.emit(close)
        mfma(dt, st, ss, i, j)
        for kind, x in plan[p]:
            if kind == "read":
                st.read(x[0], x[1])
            else:
                for t in x:
                    st.emit(t)
    if close is not None:
        st.emit("s_barrier")


def generate(la, lb, dt, read_gap=1, dma_gap=3):
    lay = {"A": la, "B": lb}
    out = []
    nf, X = GEO["nf"], "0x%x" % GEO["buf"]
    out.append("s_mov_b32 %[keep], m0")
    # prologue: tiles 0 and 1 (B then A each), tile 0's k0 fragments
    for t in range(2):
        for op in "BA":
            setup, groups = dma_ops(op, nop=True)
            out += setup
            for g in groups:
                out += g
            out.append("s_add_u32 %%[so%s], %%[so%s], %%[ks%s]" % (op, op, op))
            out.append("s_xor_b32 %%[m%s], %%[m%s], %s" % (op, op, X))
    out.append("s_waitcnt vmcnt(%d)" % (2 * nf))
    out.append("s_barrier")
    pro = Stream()
    for op in "BA":
        for i in range(nf):
            for key, text in read_ops(lay[op], op, 0, i, "nxt"):
                pro.read(key, text)
    out += pro.lines
    for op in "AB":
        if lay[op] == KC:
            out.append("v_xor_b32 %%[r%s_nxt], %s, %%[r%s_nxt]" % (op, X, op))
        else:
            out.append("v_xor_b32 %%[r%s_nxtlo], %s, %%[r%s_nxtlo]" % (op, X, op))
            out.append("v_xor_b32 %%[r%s_nxthi], %s, %%[r%s_nxthi]" % (op, X, op))
    # The fragments of k-step 0 of the coming tile are the last reads issued
    # before every body (prologue or previous body); each body starts from
    # that scoreboard.
    carried = list(pro.pending)

    def emit_body(kind):
        st = Stream()
        st.pending = list(carried)
        return body_with(st, la, lb, dt, kind, read_gap, dma_gap)

    out.append("s_cmp_eq_u32 %[cnt], 0")
    out.append("s_cbranch_scc1 L_tail_%=")
    nw = 4 if CFG["stagger"] else 1
    if nw > 1:
        for w in range(1, nw):
            out.append("s_cmp_eq_u32 %%[wid], %d" % w)
            out.append("s_cbranch_scc1 L_w%d_%%=" % w)
    for w in range(nw):
        CFG["dma_off"] = w if nw > 1 else 0
        full_lines, full_pend = emit_body("full")
        assert full_pend == carried, "loop body must leave the scoreboard it expects"
        out.append("L_w%d_%%=:" % w)
        out += full_lines
        out.append("s_sub_u32 %[cnt], %[cnt], 1")
        out.append("s_cmp_lg_u32 %[cnt], 0")
        out.append("s_cbranch_scc1 L_w%d_%%=" % w)
        if w + 1 < nw:
            out.append("s_branch L_tail_%=")
    CFG["dma_off"] = 0
    out.append("L_tail_%=:")
    nod_lines, nod_pend = emit_body("nodma")
    out += nod_lines
    last_lines, _ = emit_body("last")
    out += last_lines
    out.append("s_mov_b32 m0, %[keep]")
    return out


def body_with(st, la, lb, dt, kind, read_gap, dma_gap):
    if CFG.get("sched") == "2bar":
        return body_2bar(st, la, lb, dt, kind, read_gap, dma_gap)
    return body_4bar(st, la, lb, dt, kind, read_gap, dma_gap)


def body_2bar(st, la, lb, dt, kind, read_gap, dma_gap):
    """One K-tile iteration with TWO barriers (FX_GEN_SCHED=2bar):
      P1  k0 rows 0..p1-1        + every k1 fragment read (A then B)
          -> lgkm0, barrier: the whole buffer of tile t is in registers
      P2  k0 rows p1..nf-1, k1 rows 0..nf-p3-1 + B(t+2) then A(t+2) DMA
          -> vmcnt(2 nf): tile t+1 landed, barrier
      P3  k1 rows nf-p3..nf-1    + tile t+1's k0 reads (B then A)
    The k0 and k1 fragment sets of tile t are both live during P1/P2 (the
    same 4 x 4 nf registers as the 4-barrier body)."""
    lay = {"A": la, "B": lb}

    def reads(op, s, which, idxs):
        return [r for i in idxs for r in read_ops(lay[op], op, s, i, which)]

    full, last = kind == "full", kind == "last"
    nf, X = GEO["nf"], "0x%x" % GEO["buf"]
    p1 = CFG.get("p1", (5 * nf) // 8)
    mc = lay["A"] == MC or lay["B"] == MC
    p3 = CFG.get("p3", nf // 2 if mc else (3 * nf) // 8)
    allmf = [(0, i, j) for i in range(nf) for j in range(nf)] + \
            [(1, i, j) for i in range(nf) for j in range(nf)]
    n1, n3 = p1 * nf, p3 * nf
    mf1, mf2, mf3 = allmf[:n1], allmf[n1:len(allmf) - n3], allmf[len(allmf) - n3:]
    segment(dt, st, 0, None, [("read", reads("A", 1, "cur", range(nf)) +
                                reads("B", 1, "cur", range(nf)))],
            read_gap, dma_gap, close=None if last else "lgkm0", mf=mf1)
    ex = []
    if full:
        sB, gB = dma_ops("B")
        sA, gA = dma_ops("A")
        ex.append(("dma", (sB, gB + [sA + gA[0]] + gA[1:])))
    if last:
        segment(dt, st, 0, None, ex, read_gap, dma_gap, mf=mf2 + mf3)
        st.emit("s_nop 15")
        st.emit("s_nop 15")
        return st.lines, st.pending
    segment(dt, st, 0, None, ex, read_gap, dma_gap,
            close="s_waitcnt vmcnt(%d)" % (2 * nf if full else 0), mf=mf2)
    segment(dt, st, 0, None, [("read", reads("B", 0, "nxt", range(nf)) +
                                reads("A", 0, "nxt", range(nf)))], 1, dma_gap, mf=mf3)
    for op in "AB":
        if lay[op] == KC:
            st.emit("v_xor_b32 %%[r%s_cur], %s, %%[r%s_cur]" % (op, X, op))
            st.emit("v_xor_b32 %%[r%s_nxt], %s, %%[r%s_nxt]" % (op, X, op))
        else:
            for w in ("curlo", "curhi", "nxtlo", "nxthi"):
                st.emit("v_xor_b32 %%[r%s_%s], %s, %%[r%s_%s]" % (op, w, X, op, w))
        st.emit("s_xor_b32 %%[m%s], %%[m%s], %s" % (op, op, X))
        if full:
            st.emit("s_add_u32 %%[so%s], %%[so%s], %%[ks%s]" % (op, op, op))
    return st.lines, st.pending


def body_4bar(st, la, lb, dt, kind, read_gap, dma_gap):
    """One K-tile iteration.  kind: 'full' (stages t+2, reads t+1),
    'nodma' (reads t+1, stages nothing), 'last' (neither)."""
    lay = {"A": la, "B": lb}

    def reads(op, s, which, idxs):
        return ("read", [r for i in idxs for r in read_ops(lay[op], op, s, i, which)])

    full, last = kind == "full", kind == "last"
    nf, X = GEO["nf"], "0x%x" % GEO["buf"]
    h, q = nf // 2, nf // 4
    segment(dt, st, 0, range(0, h), [reads("B", 1, "cur", range(nf))], read_gap, dma_gap,
            close=None if last else "lgkm0")
    ex = [reads("A", 1, "cur", range(nf))]
    if full:
        ex.append(("dma", dma_ops("B")))
    segment(dt, st, 0, range(h, nf), ex, read_gap, dma_gap, close=None if last else "lgkm0")
    ex = [("dma", dma_ops("A"))] if full else []
    close = None if last else "s_waitcnt vmcnt(%d)" % (3 * nf if full else nf)
    segment(dt, st, 1, range(0, h), ex, read_gap, dma_gap, close=close)
    if last:
        segment(dt, st, 1, range(h, nf), [], read_gap, dma_gap)
        st.emit("s_nop 15")
        st.emit("s_nop 15")
        return st.lines, st.pending
    segment(dt, st, 1, range(h, h + q), [reads("B", 0, "nxt", range(nf))], 1, dma_gap,
            close="s_waitcnt vmcnt(%d)" % (2 * nf if full else 0))
    segment(dt, st, 1, range(h + q, nf), [reads("A", 0, "nxt", range(nf))], 1, dma_gap)
    for op in "AB":
        if lay[op] == KC:
            st.emit("v_xor_b32 %%[r%s_cur], %s, %%[r%s_cur]" % (op, X, op))
            st.emit("v_xor_b32 %%[r%s_nxt], %s, %%[r%s_nxt]" % (op, X, op))
        else:
            for w in ("curlo", "curhi", "nxtlo", "nxthi"):
                st.emit("v_xor_b32 %%[r%s_%s], %s, %%[r%s_%s]" % (op, w, X, op, w))
        st.emit("s_xor_b32 %%[m%s], %%[m%s], %s" % (op, op, X))
        if full:
            st.emit("s_add_u32 %%[so%s], %%[so%s], %%[ks%s]" % (op, op, op))
    return st.lines, st.pending


def split_pre_main(lines):
    """Split a generated stream for the persistent kernel: PRE = the prologue's
    LDS-DMA issue of K-tiles 0 and 1 (issued for the NEXT output tile before
    the current tile's epilogue, so its load latency hides under the epilogue),
    MAIN = the rest, whose first wait counts the epilogue's stores issued in
    between (``%[pw]``: 2 nf loads of K-tile 1 + the stores, capped at 63)."""
    nf = GEO["nf"]
    first_wait = "s_waitcnt vmcnt(%d)" % (2 * nf)
    idx = lines.index(first_wait)
    assert lines[0] == "s_mov_b32 %[keep], m0"
    pre = lines[:idx] + ["s_mov_b32 m0, %[keep]"]
    main = ["s_mov_b32 %[keep], m0", "s_waitcnt vmcnt(%[pw])"] + lines[idx + 1:]
    return pre, main


def c_string(lines):
    return "\n".join('  "%s\\n"' % l for l in lines)


ABL = set(a for a in os.environ.get("FX_GEN_ABL", "").split(",") if a)


def ablate(lines):
    """Lab-only ablations (FX_GEN_ABL=novm,nodma,nobar,nolds): timing builds
    with a class of instructions removed; their results are wrong.  (A
    VGPR-staged variant of this loop -- buffer_load -> VGPR -> ds_write, one
    barrier per K-tile -- measured 5-10 % slower on every shape:
    profiles/r4_gemm_vgpr/.)"""
    out = []
    for l in lines:
        if "novm" in ABL and l.startswith("s_waitcnt vmcnt"):
            continue
        if "nodma" in ABL and l.startswith("buffer_load"):
            continue
        if "nobar" in ABL and l == "s_barrier":
            continue
        if "nolds" in ABL and (l.startswith("ds_read") or l.startswith("s_waitcnt lgkmcnt")):
            continue
        out.append(l)
    return out


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    path = os.environ.get("FX_GEN_OUT") or os.path.join(here, "..", "csrc", "kernels",
                                                        "gemm_asm.inc")
    read_gap = int(os.environ.get("FX_GEN_READ_GAP", "1"))
    # T256: one DMA per 4 MFMAs, wave-staggered slots; T128 (8-MFMA segments):
    # one per 2 MFMAs, no stagger
    knobs = {"T256": (int(os.environ.get("FX_GEN_DMA_GAP", "4")),
                      int(os.environ.get("FX_GEN_STAGGER", "1"))),
             "T128": (int(os.environ.get("FX_GEN_DMA_GAP_T128", "2")), 0)}
    CFG["dma_start"] = int(os.environ.get("FX_GEN_DMA_START", "0"))
    # K-loop structure per geometry: "4bar" (default) or "2bar" (body_2bar)
    scheds = {"T256": os.environ.get("FX_GEN_SCHED_T256", os.environ.get("FX_GEN_SCHED", "4bar")),
              "T128": os.environ.get("FX_GEN_SCHED_T128", os.environ.get("FX_GEN_SCHED", "4bar"))}
    for key, env in (("p1", "FX_GEN_P1"), ("p3", "FX_GEN_P3")):
        if os.environ.get(env):
            CFG[key] = int(os.environ[env])
    parts = ["// GENERATED by tools/gen_gemm_asm.py -- do not edit.\n"
             "// K-loops of gemm5_kernel (csrc/kernels/gemm5.hip); read_gap=%d, "
             "(dma_gap, stagger) T256=%s T128=%s, sched %s\n" % (read_gap, knobs["T256"],
                                                                 knobs["T128"], scheds)]
    names = {KC: "KC", MC: "MC"}
    for tag in ("T256", "T128"):
        set_geometry(tag)
        dma_gap, CFG["stagger"] = knobs[tag]
        CFG["sched"] = scheds[tag]
        for la, lb in ((KC, KC), (KC, MC), (MC, MC)):
            for dt in ("bf16", "f16"):
                lines = ablate(generate(la, lb, dt, read_gap, dma_gap))
                parts.append("#define FX_G5_%s_%s_%s_%s \\\n%s\n" % (
                    tag, names[la], names[lb], dt.upper(),
                    " \\\n".join('  "%s\\n"' % l for l in lines)))
                if la == MC and lb == MC:
                    continue  # weight gradients (fp32 out) are not persistent
                pre, main = split_pre_main(lines)
                if dt == "bf16":  # the DMA prologue is the same for both dtypes
                    parts.append("#define FX_G5_%s_%s_%s_PRE \\\n%s\n" % (
                        tag, names[la], names[lb],
                        " \\\n".join('  "%s\\n"' % l for l in pre)))
                parts.append("#define FX_G5_%s_%s_%s_%s_MAIN \\\n%s\n" % (
                    tag, names[la], names[lb], dt.upper(),
                    " \\\n".join('  "%s\\n"' % l for l in main)))
    with open(path, "w") as f:
        f.write("\n".join(parts))
    print("wrote", os.path.normpath(path), file=sys.stderr)


if __name__ == "__main__":
    main()

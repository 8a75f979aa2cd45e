"""LDS bank-conflict simulator for the flash-attention tile images.

Models gfx950 banking (MI355X_MICROARCH.md §LDS): ``ds_read_b128`` is serviced
in four 16-lane groups, ``ds_read_b64_tr_b16`` in two 32-lane halves, bank =
(byte/4) mod 64.  For a candidate XOR swizzle of the 16-byte chunk index it
reports the worst LDS cycles per wave-instruction for the two access patterns
used by ``csrc/kernels/flash_attn.hip``:

* row reads of the 32x32x16 MFMA operand (lane l -> row l&31, chunk 2s+(l>>5)),
  ideal 4 cycles;
* transposed reads for V^T / K^T / Q^T / dO^T fragments, ideal 2 cycles.

Run ``python tools/lds_bank_sim.py`` to search the linear (GF(2)) swizzles
for D=64 and D=128; the kernel uses the first conflict-free one found
(D=128 coincides with the guide's "plain 256-byte rows" image).
"""
import itertools

G128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
        list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
G128 = G128 + [[l + 32 for l in g] for g in G128]


def cost_b128(addrs):
    tot = 0
    for g in G128:
        banks = {}
        for l in g:
            for w in range(4):
                banks.setdefault((addrs[l] // 4 + w) % 64, set()).add(addrs[l] // 4 + w)
        tot += max(len(v) for v in banks.values())
    return tot


def cost_tr(addrs):
    tot = 0
    for h in range(2):
        banks = {}
        for l in range(32 * h, 32 * h + 32):
            for w in range(2):
                banks.setdefault((addrs[l] // 4 + w) % 64, set()).add(addrs[l] // 4 + w)
        tot += max(len(v) for v in banks.values())
    return tot


def make_off(D, fbits):
    nch = D // 8
    rowb = D * 2

    def off(row, ch):
        f = 0
        for i, rb in enumerate(fbits):
            if bin(row & rb).count("1") % 2:
                f |= 1 << i
        return rowb * row + 16 * ((ch ^ f) % nch)
    return off


def test(D, off):
    worst_r = worst_t = 0
    for r0 in range(0, 64, 32):
        for s in range(D // 16):
            addrs = [off(r0 + (l & 31), 2 * s + (l >> 5)) for l in range(64)]
            worst_r = max(worst_r, cost_b128(addrs))
    for kb in range(0, 64, 16):
        for dbase in range(0, D, 32):
            for second in (0, 8):
                addrs = []
                for l in range(64):
                    hh, gi, i = l >> 5, (l >> 4) & 1, l & 15
                    q, p = i >> 2, i & 3
                    row = kb + second + 4 * hh + q
                    col = dbase + 16 * gi + 4 * p
                    addrs.append(off(row, col // 8) + 2 * (col % 8))
                worst_t = max(worst_t, cost_tr(addrs))
    return worst_r, worst_t


def search(D):
    nbits = (D // 8).bit_length() - 1
    for fb in itertools.product(range(64), repeat=nbits):
        r, t = test(D, make_off(D, fb))
        if r == 4 and t == 2:
            return fb, (r, t)
    return None


def loff_subtiled(D):
    """The kernels' LDS image (csrc/kernels/flash_attn.hip ``loff``): 8-row x
    32-column subtiles of 512 B with the chunk XORed inside its 4-chunk group."""
    def off(row, ch):
        return (16 * D) * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) + \
            16 * ((ch & 3) ^ ((row >> 2) & 3))
    return off


def check_frag():
    """``Frag`` (flash_attn.hip) reads every operand fragment as a per-lane base
    plus an immediate; check those closed forms against ``loff`` for every lane,
    32-row block, k-step and transposed-read block, for D = 64 / 96 / 128."""
    for D in (64, 96, 128):
        off = loff_subtiled(D)
        for lane in range(64):
            h, r = lane >> 5, lane & 31
            rbase = 16 * D * (r >> 3) + 64 * (r & 7)
            rb = [rbase + 16 * (h ^ ((r >> 2) & 3)), rbase + 16 * ((2 + h) ^ ((r >> 2) & 3))]
            gi, q, p = (lane >> 4) & 1, (lane >> 2) & 3, lane & 3
            tbase = 64 * (4 * h + q) + 8 * (p & 1)
            c = 2 * gi + (p >> 1)
            tb = [tbase + 16 * (c ^ h), tbase + 16 * (c ^ (2 + h)) + 16 * D]
            for t in range(4):
                for s in range(D // 16):
                    assert off(32 * t + r, 2 * s + h) == rb[s & 1] + 64 * D * t + 512 * (s >> 1)
                for ss in range(2):
                    for dt in range(D // 32):
                        kb = 32 * t + 16 * ss + 4 * h
                        ch = 4 * dt + 2 * gi + (p >> 1)
                        for e in (0, 1):
                            want = off(kb + 8 * e + q, ch) + 8 * (p & 1)
                            assert want == tb[e] + 64 * D * t + 32 * D * ss + 512 * dt
        print("D=%d: Frag closed forms match loff for all lanes; banks (row, tr) = %s"
              % (D, test(D, off)))


if __name__ == "__main__":
    import sys
    if "--check-frag" in sys.argv:
        check_frag()
        sys.exit(0)
    for D in (64, 128):
        print("D=%d naive" % D, test(D, make_off(D, (0,) * ((D // 8).bit_length() - 1))))
        print("D=%d found" % D, search(D))
    print("D=128 guide image (b)", test(128, make_off(128, (4, 8, 1, 2))))

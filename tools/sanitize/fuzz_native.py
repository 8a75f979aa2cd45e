"""Fuzz the native index builders inside the ASan/UBSan driver
(``csrc/native/sanitize/driver.cpp``; run by ``tools/sanitize/run_native.sh``).

Imports only numpy and the built-in ``_native`` module (no torch: the
process is sanitizer-instrumented and should stay small).  Each case checks
outputs against an inline Python oracle so a sanitizer-clean run is also a
correct one."""
import sys

import numpy as np

import _native

ITERS = int(sys.argv[1]) if len(sys.argv) > 1 else 40


def sample_idx_oracle(sizes, doc_idx, seq, epochs, tpe):
    n = (epochs * tpe - 1) // seq
    out = np.zeros((n + 1, 2), dtype=np.int32)
    d, off = 0, 0
    for s in range(1, n + 1):
        need = seq + 1
        while True:
            avail = sizes[doc_idx[d]] - off
            if avail >= need:
                off += need - 1
                break
            need -= avail
            d += 1
            off = 0
        out[s] = (d, off)
    return out


def check_sample_idx(rs):
    ndoc = rs.randint(1, 60)
    sizes = rs.randint(0 if rs.rand() < 0.3 else 1, rs.randint(2, 400), size=ndoc).astype(np.int32)
    if sizes.sum() < 2:
        sizes[0] = 2
    tpe = int(sizes.sum())
    epochs = rs.randint(1, 4)
    doc_idx = np.concatenate([rs.permutation(ndoc) for _ in range(epochs)]).astype(np.int32)
    seq = int(rs.randint(2, max(3, tpe)))
    got = _native.build_sample_idx(sizes, doc_idx, seq, epochs, tpe)
    ref = sample_idx_oracle(sizes, doc_idx, seq, epochs, tpe)
    assert got.dtype == np.int32 and np.array_equal(got, ref), (seq, epochs, tpe)
    # a too-short doc_idx must raise, not read past the end
    try:
        _native.build_sample_idx(sizes, doc_idx[:1], seq, epochs + 3, tpe)
        raise AssertionError("expected ValueError for an exhausted doc_idx")
    except ValueError:
        pass


def check_mapping(rs):
    nsent = rs.randint(0, 9, size=rs.randint(1, 80))
    docs = np.concatenate([[0], np.cumsum(nsent)]).astype(np.int64)
    ns = int(docs[-1])
    sizes = rs.randint(1, 700 if rs.rand() < 0.3 else 200, size=max(ns, 1)).astype(np.int32)[:ns]
    max_seq = int(rs.randint(2, 300))
    m = _native.build_mapping(docs, sizes, int(rs.randint(1, 4)), int(rs.randint(1, 10 ** 5)),
                              max_seq, float(rs.choice([0.0, 0.1, 0.5])), int(rs.randint(1, 99)),
                              False, int(rs.randint(1, 4)))
    assert m.ndim == 2 and m.shape[1] == 3
    if len(m):
        assert (m[:, 0] < m[:, 1]).all() and (m[:, 1] <= ns).all()
        assert ((m[:, 2] >= 2) & (m[:, 2] <= max_seq)).all()
    titles = rs.randint(0, 8, size=len(docs) - 1).astype(np.int32)
    b = _native.build_blocks_mapping(docs, sizes, titles, int(rs.randint(1, 3)),
                                     int(rs.randint(1, 10 ** 5)), int(rs.randint(16, 300)),
                                     int(rs.randint(1, 99)), False, bool(rs.rand() < 0.5))
    assert b.ndim == 2 and b.shape[1] == 4
    if len(b):
        assert (b[:, 2] < len(docs) - 1).all() and (b[:, 1] <= ns).all()


def check_blending(rs):
    k = int(rs.randint(1, 6))
    w = rs.rand(k)
    w /= w.sum()
    n = int(rs.randint(1, 5000))
    di = np.zeros(n, dtype=np.uint8)
    dsi = np.zeros(n, dtype=np.int64)
    _native.build_blending_indices(di, dsi, w, k, n, False)
    assert di.max() < k
    for d in range(k):
        assert dsi[di == d].tolist() == list(range(int((di == d).sum())))


def check_buckets(rs):
    numels = rs.randint(1, 1000, size=rs.randint(1, 200)).tolist()
    cap = int(rs.randint(1, 3000))
    b = _native.plan_buckets(numels, cap)
    assert len(b) == len(numels) and list(b) == sorted(b)


def main():
    rs = np.random.RandomState(1234)
    for _ in range(ITERS):
        check_sample_idx(rs)
        check_mapping(rs)
        check_blending(rs)
        check_buckets(rs)
    print("fuzz_native: %d iterations clean" % ITERS)


main()

"""Host-code sanitizers: the native index builders compiled with
ASan + UBSan into a standalone driver that embeds CPython, fuzzed against
Python oracles (``tools/sanitize/run_native.sh``)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which(os.environ.get("CXX", "g++")) is None, reason="no host C++ compiler")
def test_native_builders_asan_ubsan_clean():
    r = subprocess.run([os.path.join(ROOT, "tools", "sanitize", "run_native.sh"), "8"],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600)
    out = r.stdout
    assert r.returncode == 0, out[-4000:]
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert "iterations clean" in out


def test_sample_idx_rejects_short_doc_idx():
    """Hardening found by the sanitizer run: an exhausted doc_idx raises."""
    import numpy as np
    native = pytest.importorskip("fleetx_amd._C._native")
    sizes = np.array([5, 5], dtype=np.int32)
    with pytest.raises(ValueError):
        native.build_sample_idx(sizes, np.array([0], dtype=np.int32), 4, 3, 10)

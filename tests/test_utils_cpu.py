"""Local-cache cached_path (reference download.py rank-0 handshake) and the
environment checks (reference check.py / version.py)."""
import os
import threading
import time

import pytest


def test_cached_path_local_and_cache(tmp_path, monkeypatch):
    from fleetx_amd.utils import download as D
    f = tmp_path / "vocab.json"
    f.write_text("{}")
    assert D.cached_path(str(f)) == str(f)
    assert D.cached_path("file://" + str(f)) == str(f)
    with pytest.raises(FileNotFoundError):
        D.cached_path(str(tmp_path / "missing"))
    url = "https://example.com/models/gpt2/vocab.json"
    dst = D.map_path(url, str(tmp_path / "cache"))
    monkeypatch.setenv("LOCAL_RANK", "0")
    monkeypatch.delenv("FLEETX_ALLOW_DOWNLOAD", raising=False)
    with pytest.raises(FileNotFoundError, match="place the file at"):
        D.cached_path(url, cache_dir=str(tmp_path / "cache"))
    os.makedirs(os.path.dirname(dst))
    open(dst, "w").write("x")
    assert D.cached_path(url, cache_dir=str(tmp_path / "cache")) == dst


def test_cached_path_nonzero_rank_waits_for_rank0(tmp_path, monkeypatch):
    from fleetx_amd.utils import download as D
    url = "https://example.com/a/b.bin"
    cache = str(tmp_path / "c")
    dst = D.map_path(url, cache)
    monkeypatch.setenv("LOCAL_RANK", "1")
    monkeypatch.setenv("FLEETX_ALLOW_DOWNLOAD", "1")

    def rank0():
        time.sleep(0.3)
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        open(dst + ".tmp", "w").write("y")
        os.replace(dst + ".tmp", dst)
    t = threading.Thread(target=rank0)
    t.start()
    assert D.cached_path(url, cache_dir=cache, timeout_s=10, poll_s=0.05) == dst
    t.join()


def test_version_and_gpu_checks():
    import torch
    from fleetx_amd.utils import check as C
    assert C.version_check(exit=False) == torch.__version__
    assert C._ver("2.10.0+rocm7.0") == (2, 10)
    if not torch.cuda.is_available():
        with pytest.raises(RuntimeError):
            C.check_gpu(exit=False)

"""Local-cache ``cached_path`` (reference ``ppfleetx/utils/download.py:27-128``).

The reference resolves a URL to ``~/.cache/ppfleetx/<path>``: local rank 0
downloads into the cache while every other rank polls for the file, so a
node fetches each asset once.  This environment has no network, so the
MI355X build keeps the same contract over an offline cache:

* a local path (or ``file://`` URL) is returned as is (must exist);
* an ``http(s)://`` URL maps to ``<cache_dir>/<url path>``; if that file is
  already in the cache (put there by a previous run or copied in by hand)
  it is returned;
* otherwise local rank 0 tries to fetch it (``FLEETX_ALLOW_DOWNLOAD=1`` only,
  atomically: ``.part`` file + rename) while the other ranks of the node wait
  for the final file to appear -- exactly the reference's rank-0 handshake --
  and a clear error names the cache path to populate when downloading is off.
"""
import os
import time
import urllib.parse

DEFAULT_CACHE = os.path.expanduser(os.environ.get("FLEETX_CACHE_DIR", "~/.cache/fleetx_amd"))


def is_url(path):
    return str(path).startswith(("http://", "https://"))


def map_path(url, cache_dir=None):
    """Cache location of ``url``: ``<cache_dir>/<host>/<path>``."""
    u = urllib.parse.urlparse(url)
    return os.path.join(cache_dir or DEFAULT_CACHE, u.netloc, u.path.lstrip("/"))


def _local_rank():
    return int(os.environ.get("LOCAL_RANK", os.environ.get("PADDLE_RANK_IN_NODE", "0")))


def _local_world():
    return int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))


def _fetch(url, dst):
    import urllib.request
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    tmp = "%s.part.%d" % (dst, os.getpid())
    with urllib.request.urlopen(url, timeout=60) as r, open(tmp, "wb") as f:
        while True:
            chunk = r.read(1 << 20)
            if not chunk:
                break
            f.write(chunk)
    os.replace(tmp, dst)


def cached_path(url_or_path, cache_dir=None, timeout_s=3600, poll_s=1.0):
    """Resolve ``url_or_path`` to a local file (see module docstring)."""
    p = str(url_or_path)
    if p.startswith("file://"):
        p = urllib.parse.urlparse(p).path
    if not is_url(p):
        if not os.path.exists(p):
            raise FileNotFoundError(p)
        return p
    dst = map_path(p, cache_dir)
    if os.path.exists(dst):
        return dst
    allow = os.environ.get("FLEETX_ALLOW_DOWNLOAD", "0") == "1"
    if _local_rank() == 0:
        if not allow:
            raise FileNotFoundError(
                "{} is not in the local cache and downloading is disabled "
                "(FLEETX_ALLOW_DOWNLOAD=1 to fetch); place the file at {}".format(p, dst))
        _fetch(p, dst)
        return dst
    if not allow and _local_world() > 1:
        raise FileNotFoundError("{} not cached at {}".format(p, dst))
    t0 = time.time()
    while not os.path.exists(dst):      # other local ranks wait for rank 0's copy
        if time.time() - t0 > timeout_s:
            raise TimeoutError("waited {} s for local rank 0 to fetch {}".format(timeout_s, p))
        time.sleep(poll_s)
    return dst

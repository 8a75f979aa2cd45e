"""Counter-based RNG streams for dropout (replayable under recompute).

Capability parity: Paddle ``get_rng_state_tracker()`` with the reference's
``global_seed`` / ``local_seed`` streams (``ppfleetx/utils/env.py:27-46``,
used at ``hybrid_model.py:279-285,546-559,615-619``).

MI355X-first design: there is no global device generator in the hot path.
Every dropout site asks the tracker for a fresh 64-bit *key* derived from
``(stream seed, stream offset)``; the HIP kernels hash ``(key, element
coordinate)`` to a 16-bit uniform, so the same key regenerates the same mask
in the backward kernel and in an activation-recompute replay.  Saving and
restoring the tracker state (``get_states``/``set_states``) is therefore all
that recompute and checkpoint/resume need.

The hash is ``lowbias32`` (a 32-bit avalanche permutation); :func:`keep_mask`
is the exact PyTorch reproduction used by CPU execution and by the kernel
tests.
"""
import contextlib

import torch

MASK32 = 0xFFFFFFFF
_GOLDEN = 0x9E3779B97F4A7C15


def splitmix64(x):
    x = (x + _GOLDEN) & 0xFFFFFFFFFFFFFFFF
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def lowbias32_int(x):
    x &= MASK32
    x ^= x >> 16
    x = (x * 0x7FEB352D) & MASK32
    x ^= x >> 15
    x = (x * 0x846CA68B) & MASK32
    x ^= x >> 16
    return x


def lowbias32(x):
    """Tensor version on int64 tensors holding uint32 values."""
    x = x & MASK32
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & MASK32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & MASK32
    x = x ^ (x >> 16)
    return x


def threshold16(p):
    """Drop when rand16 < thr; keep probability is 1 - thr/65536."""
    return int(round(p * 65536.0))


def key_words(key):
    return key & MASK32, (key >> 32) & MASK32


def elementwise_rand16(numel, key, device="cpu"):
    """16-bit uniforms for a flat tensor of ``numel`` elements.

    Element ``i``: ``h = lowbias32(lo32(i>>1) ^ lowbias32(hi32(i>>1) ^ khi) ^ klo)``,
    low half for even ``i``, high half for odd ``i``.  Must match
    ``csrc/kernels/fx_rng.h``.
    """
    klo, khi = key_words(key)
    i = torch.arange(numel, dtype=torch.int64, device=device)
    pair = i >> 1
    lo = pair & MASK32
    hi = pair >> 32
    c = lowbias32(hi ^ khi) ^ klo
    h = lowbias32(lo ^ c)
    return torch.where((i & 1) == 1, h >> 16, h & 0xFFFF)


def keep_mask(shape, p, key, device="cpu"):
    numel = 1
    for s in shape:
        numel *= s
    r = elementwise_rand16(numel, key, device)
    return (r >= threshold16(p)).reshape(shape)


def attention_rand16(bh, sq, sk, key, device="cpu"):
    """16-bit uniforms for attention probabilities ``[bh, sq, sk]``.

    Element ``(b, q, k)``: ``h = lowbias32(((q << 16) | (k >> 1)) ^ C_b)`` with
    ``C_b = lowbias32(b ^ khi) ^ klo``; low half for even ``k``.
    """
    klo, khi = key_words(key)
    b = torch.arange(bh, dtype=torch.int64, device=device).view(bh, 1, 1)
    q = torch.arange(sq, dtype=torch.int64, device=device).view(1, sq, 1)
    k = torch.arange(sk, dtype=torch.int64, device=device).view(1, 1, sk)
    cb = lowbias32(b ^ khi) ^ klo
    h = lowbias32(((q << 16) | (k >> 1)) ^ cb)
    return torch.where((k & 1) == 1, h >> 16, h & 0xFFFF)


def attention_keep_mask(bh, sq, sk, p, key, device="cpu"):
    return attention_rand16(bh, sq, sk, key, device) >= threshold16(p)


class RNGStream:
    def __init__(self, seed):
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.offset = 0

    def next_key(self):
        # 63-bit keys: they travel as int64 scalars through autograd (and the
        # profiler's record_shapes), which rejects values >= 2^63
        k = splitmix64(self.seed ^ splitmix64(self.offset)) & 0x7FFFFFFFFFFFFFFF
        self.offset += 1
        return k


class RNGStatesTracker:
    """Named RNG streams; ``rng_state(name)`` selects the active stream."""

    def __init__(self):
        self.streams = {}
        self._active = []

    def reset(self):
        self.streams = {}
        self._active = []

    def add(self, name, seed):
        if name in self.streams:
            raise ValueError("rng state {} already exists".format(name))
        self.streams[name] = RNGStream(seed)

    def get_states(self):
        return {k: (s.seed, s.offset) for k, s in self.streams.items()}

    def set_states(self, states):
        for k, (seed, off) in states.items():
            if k not in self.streams:
                self.streams[k] = RNGStream(seed)
            self.streams[k].seed = seed
            self.streams[k].offset = off

    @contextlib.contextmanager
    def rng_state(self, name="global_seed"):
        if name not in self.streams:
            raise ValueError("rng state {} does not exist".format(name))
        self._active.append(name)
        try:
            yield
        finally:
            self._active.pop()

    def next_key(self, name=None):
        if name is None:
            name = self._active[-1] if self._active else "global_seed"
        if name not in self.streams:
            self.add(name, 1234)
        return self.streams[name].next_key()


_TRACKER = RNGStatesTracker()


def get_rng_state_tracker():
    return _TRACKER


def model_parallel_random_seed(seed, mp_rank=0, pp_rank=0, data_rank=0):
    """Reference seed rules (``env.py:27-46``): ``global_seed`` equal across mp
    ranks of a data replica, ``local_seed`` distinct per mp/pp rank."""
    tracker = get_rng_state_tracker()
    tracker.reset()
    global_seed = seed + data_rank
    local_seed = seed + 123 + mp_rank * 10 + pp_rank * 1000
    tracker.add("global_seed", global_seed)
    tracker.add("local_seed", local_seed)
    return global_seed, local_seed

"""Deterministic synthetic key/packet generators shared by the golden-vector generator and the tests.

Test infrastructure only.  numpy's PCG64 stream is stable across platforms and numpy versions, so a
(seed, n, lo, hi) tuple names the same key set here and on the GPU box.
"""
import numpy as np


def random_packets(seed, n, lo, hi):
    """n packets with lengths ~ U[lo, hi] and uniformly random bytes.

    Returns (blob: bytes, offsets: np.uint64[n+1]) -- the packed offset+byte layout the C-ABI takes.
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    lengths = rng.integers(lo, hi + 1, size=n, dtype=np.int64)
    offsets = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lengths, out=offsets[1:])
    blob = rng.bytes(int(offsets[-1]))
    return blob, offsets


def packet_list(seed, n, lo, hi):
    blob, offsets = random_packets(seed, n, lo, hi)
    return [blob[int(offsets[i]):int(offsets[i + 1])] for i in range(n)]


def named_packets(n, start=0, fmt=b"packet-%d"):
    return [fmt % i for i in range(start, start + n)]


def pack(keys):
    """list[bytes] -> (blob, offsets u64[n+1])."""
    offsets = np.zeros(len(keys) + 1, dtype=np.uint64)
    if keys:
        np.cumsum(np.fromiter((len(k) for k in keys), dtype=np.int64, count=len(keys)), out=offsets[1:])
    return b"".join(keys), offsets

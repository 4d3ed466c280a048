"""Bit positions by multiply-high (dsy_message.h bit_position): pos = chunk % m (bloomfilter.py:171) computed as
a - mulhi(a, ceil(2^32/m)) * m, with one wrap-around fix for 4-byte chunks.

CPU: the same integer formula in numpy against % -- every (chunk, m) pair of the 2-byte 'H' family (m a multiple of
eight below 2^15, chunk below 2^16) and, for the 4-byte 'L' family (2^15 <= m < 2^31), edge sizes and edge chunks
(0, 2^32-1, multiples of m and their neighbours) plus random ones.  GPU: the device positions (dsy_bloom_indices)
against the oracle's hashlib digests for sizes spread over both families and both ends of each."""
import numpy as np
import pytest

from oracle.bloom_ref import OracleBloom

M32 = np.uint64(0xFFFFFFFF)


def recip(m):
    """mod_recip (dsy_message.h): ceil(2^32 / m) for 2 <= m < 2^31."""
    return 0xFFFFFFFF // m + 1


def pos_h(a, m):
    q = (a * np.uint64(recip(m))) >> np.uint64(32)
    return a - q * np.uint64(m)


def pos_l(a, m):
    q = (a * np.uint64(recip(m))) >> np.uint64(32)
    r = (a - q * np.uint64(m)) & M32
    return np.minimum(r, (r + np.uint64(m)) & M32)


def test_h_family_every_pair():
    a = np.arange(1 << 16, dtype=np.uint64)
    for m in range(8, 1 << 15, 8):
        r = pos_h(a, m)
        if not np.array_equal(r, a % np.uint64(m)):
            bad = int(np.flatnonzero(r != a % np.uint64(m))[0])
            pytest.fail("m=%d chunk=%d: %d != %d" % (m, bad, int(r[bad]), bad % m))


def test_l_family_edges_and_random():
    rng = np.random.default_rng(7)
    sizes = [1 << 15, (1 << 15) + 8, 10160 * 8, 1 << 20, (1 << 20) + 8, (1 << 24) - 8, 1 << 30, (1 << 31) - 8,
             (1 << 31) - 16, 3 * (1 << 29)]
    sizes += [int(x) * 8 for x in rng.integers(1 << 12, 1 << 28, 200)]
    rand = rng.integers(0, 1 << 32, 20000, dtype=np.uint64)
    for m in sizes:
        mu = np.uint64(m)
        mult = (np.arange(0, (1 << 32) // m + 1, max(1, (1 << 32) // m // 4000), dtype=np.uint64) * mu)
        mult = mult[mult <= M32]
        edges = np.concatenate([np.array([0, 1, m - 1, m, m + 1, 0xFFFFFFFF, 0xFFFFFFFE], dtype=np.uint64),
                                mult, np.minimum(mult + np.uint64(1), M32), mult[1:] - np.uint64(1), rand])
        edges = edges[edges <= M32]
        assert np.array_equal(pos_l(edges, m), edges % mu), m


@pytest.mark.gpu
def test_device_positions_match_hashlib():
    from dispersy_amd import _native
    from dispersy_amd.bloomfilter import pack_keys
    ctx = _native.default_context()
    rng = np.random.default_rng(11)
    keys = [rng.bytes(int(n)) for n in rng.integers(0, 300, 400)]
    blob, off = pack_keys(keys)
    cases = [(8, 1), (16, 3), (24, 8), (4096, 10), (10160, 7), (32760, 8), (32752, 5),
             (1 << 15, 4), ((1 << 15) + 8, 5), (1 << 20, 7), ((1 << 24) - 8, 12), ((1 << 31) - 8, 3)]
    cases += [(int(x) * 8, int(kk)) for x, kk in zip(rng.integers(1, 1 << 12, 6), rng.integers(1, 9, 6))]
    cases += [(int(x) * 8, int(kk)) for x, kk in zip(rng.integers(1 << 12, 1 << 27, 6), rng.integers(1, 17, 6))]
    for m, k in cases:
        ref = OracleBloom(m, k, b"\x07")
        p = _native.bloom_params(m, k, _native.HASH_KINDS[ref.hash_name], ref.chunk, b"\x07")
        got = ctx.bloom_indices(p, blob, off).reshape(len(keys), k).tolist()
        assert got == [ref.indices(x) for x in keys], (m, k)

"""BloomFilter parity on the MI355X: the HIP kernels against the reference's golden vectors and the CPU oracle.

Bit-exact: filter bytes, bit positions, membership and not_filter output order.
"""
import hashlib

import numpy as np
import pytest

from dispersy_amd import BloomFilter
from dispersy_amd import _native
from dispersy_amd.bloomfilter import pack_keys
from golden_util import expected_bytes, keys_for, load
from keys import packet_list, random_packets
from oracle.bloom_ref import OracleBloom

pytestmark = pytest.mark.gpu

BLOOM = load("bloom_vectors.json")


def make(case):
    ctor, prefix = case["ctor"], bytes.fromhex(case["prefix"])
    if ctor[0] == "m_f":
        return BloomFilter(ctor[1], float(ctor[2]), prefix)
    return BloomFilter(float(ctor[1]), ctor[2], prefix)


@pytest.mark.parametrize("case", BLOOM["cases"], ids=[c["name"] for c in BLOOM["cases"]])
def test_golden_case(case):
    e = case["expect"]
    keys, probes = keys_for(case["keys"]), keys_for(case["probes"])
    bf = make(case)
    assert (bf.size, bf.functions, bf.hash_name, bf.chunk_bytes) == (e["m"], e["k"], e["hash"], e["chunk"])
    if keys:
        blob, off = pack_keys(keys[:64])
        idx = _native.default_context().bloom_indices(bf.params, blob, off)
        assert idx.tolist() == e["indices"]
    blob, off = pack_keys(probes[:16])
    assert _native.default_context().bloom_indices(bf.params, blob, off).tolist() == e["probe_indices"]
    bf.add_keys(keys)
    assert hashlib.sha256(bf.bytes).hexdigest() == e["bytes_sha256"]
    assert bf.bytes == expected_bytes(e)
    assert bf.bits_checked == e["bits_checked"]
    assert bf.contains_many(probes).astype(int).tolist() == e["present"]
    assert [i for _, i in bf.not_filter((p, i) for i, p in enumerate(probes))] == e["missing"]
    clone = BloomFilter(bf.bytes, bf.functions, bf.prefix)
    assert clone.bytes == bf.bytes
    assert [p in clone for p in probes[:20]] == [bool(x) for x in e["present"][:20]]


def test_chunk_q_indices():
    """m >= 2^31: 8-byte 'Q' chunks, 64-bit modulo (bloomfilter.py:135-136)."""
    ctx = _native.default_context()
    for row in BLOOM["chunk_q"]:
        p = _native.bloom_params(row["m"], row["k"], _native.HASH_KINDS[row["hash"]], row["chunk"],
                                 bytes.fromhex(row["prefix"]))
        blob, off = pack_keys(keys_for(row["keys"]))
        assert ctx.bloom_indices(p, blob, off).tolist() == row["indices"]


def test_single_add_and_contains():
    bf = BloomFilter(10160, 0.01, prefix=b"\x2a")
    ref = OracleBloom.from_m_f(10160, 0.01, b"\x2a")
    for i in range(50):
        key = b"packet-%d" % i
        bf.add(key)
        ref.add(key)
        assert bf.bytes == ref.to_bytes()
    assert all(b"packet-%d" % i in bf for i in range(50))
    assert bf._filter == ref.bits
    bf.clear()
    assert bf.bits_checked == 0 and not any(bf.bytes)


@pytest.mark.parametrize("m,f,prefix", [(10160, 0.01, b"\x00\x01\x02\x03"), (4096, 0.001, b"x"),
                                        (1 << 20, 0.01, b"\x07"), (1 << 16, 0.001, b"\x33" * 70),
                                        (1 << 16, 0.0001, b""), (8192, 0.00001, b"q" * 200)])
def test_heavy_tail_against_oracle(m, f, prefix):
    """Pareto-ish lengths up to the UDP cap (endpoint.py:263), all hash families, vs the oracle."""
    rng = np.random.Generator(np.random.PCG64(m + len(prefix)))
    lengths = np.minimum((rng.pareto(1.2, 3000) + 1) * 60, 65476).astype(np.int64)
    lengths[:5] = [0, 1, 55, 56, 64]
    keys = [rng.bytes(int(n)) for n in lengths]
    bf, ref = BloomFilter(m, f, prefix), OracleBloom.from_m_f(m, f, prefix)
    bf.add_keys(keys[:1500])
    ref.add_keys(keys[:1500])
    assert bf.bytes == ref.to_bytes()
    assert bf.contains_many(keys).tolist() == [k in ref for k in keys]


def test_large_batch_against_oracle():
    """100k adds + 200k tests at the MTU size (config 1 shape, scaled to finish in seconds on the oracle)."""
    blob, off = random_packets(1234, 100_000, 100, 1500)
    bf = BloomFilter(10160, 0.01, prefix=b"\x00\x01\x02\x03")
    bf.add_packed(blob, off)
    ref = OracleBloom.from_m_f(10160, 0.01, b"\x00\x01\x02\x03")
    ref.add_keys(blob[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1))
    assert bf.bytes == ref.to_bytes()
    # at capacity: 1059 keys, then 200k probes
    keys = packet_list(99, 1059, 100, 1500)
    probes_blob, probes_off = random_packets(4321, 200_000, 100, 1500)
    bf2, ref2 = BloomFilter(10160, 0.01, prefix=b"\x00\x01\x02\x03"), OracleBloom.from_m_f(10160, 0.01, b"\x00\x01\x02\x03")
    bf2.add_keys(keys)
    ref2.add_keys(keys)
    got = _native.default_context().bloom_test(bf2.params, probes_blob, probes_off, bf2.bytes)
    want = [probes_blob[int(probes_off[i]):int(probes_off[i + 1])] in ref2 for i in range(len(probes_off) - 1)]
    assert got.astype(bool).tolist() == want


# ---- tests/test_bloomfilter.py of the reference, re-expressed (keys as bytes)
def test_ref_fixed_size_constructor():
    for bloom in (BloomFilter(128 * 8, 0.25), BloomFilter(128 * 8, 0.25, b""), BloomFilter(128 * 8, 0.25, prefix=b"")):
        bloom.add_keys(str(i).encode() for i in range(100))
        assert (bloom.size, len(bloom.bytes), bloom.prefix) == (1024, 128, b"")
    for bloom in (BloomFilter(128 * 8, 0.25, b"p"), BloomFilter(128 * 8, 0.25, prefix=b"p")):
        bloom.add_keys(str(i).encode() for i in range(100))
        assert (bloom.size, len(bloom.bytes), bloom.prefix) == (1024, 128, b"p")


def test_ref_load_constructor():
    for prefix in (b"", b"p"):
        bloom = BloomFilter(128 * 8, 0.25, prefix)
        bloom.add_keys(str(i).encode() for i in range(100))
        raw, k = bloom.bytes, bloom.functions
        for clone in (BloomFilter(raw, k, prefix), BloomFilter(raw, k, prefix=prefix)):
            assert clone.size == 1024 and clone.bytes == raw and clone.prefix == prefix
            assert all(str(i).encode() in clone for i in range(100))


def test_ref_false_positives():
    for prefix in (b"", b"p"):
        for n in (128, 1024):
            for f in (0.1, 0.2, 0.3, 0.4):
                bloom = BloomFilter(f, n, prefix)
                bloom.add_keys(str(i).encode() for i in range(n))
                assert bloom.contains_many([str(i).encode() for i in range(n)]).all()
                fp = int(bloom.contains_many([str(i).encode() for i in range(n, n + 10000)]).sum())
                assert abs(fp / 10000.0 - f) <= 0.05


@pytest.mark.parametrize("m,f,prefix", [(10160, 0.01, b""), (10160, 0.01, b"\x05\x06\x07\x08"), (4096, 0.001, b"x"),
                                        (1 << 20, 0.01, b"\x07"), (1 << 16, 0.0001, b"abcde"),
                                        (1 << 15, 0.001, b"\x01\x02")])
def test_length_sorted_batches_against_oracle(m, f, prefix):
    """Batches above the sort threshold (dsy_capi kLenSortMin) hash in length-bucketed order, with LDS-DMA staging
    for MD5: adds and tests of 40 k heavy-tailed keys in every family against the oracle, outputs in key order."""
    rng = np.random.Generator(np.random.PCG64(m ^ len(prefix)))
    lengths = np.minimum((rng.pareto(1.2, 40_000) + 1) * 60, 20_000).astype(np.int64)
    lengths[:6] = [0, 1, 55, 56, 63, 64]
    keys = [rng.bytes(int(n)) for n in lengths]
    bf, ref = BloomFilter(m, f, prefix), OracleBloom.from_m_f(m, f, prefix)
    bf.add_keys(keys[:35_000])
    ref.add_keys(keys[:35_000])
    assert bf.bytes == ref.to_bytes()
    blob, off = pack_keys(keys)
    got = _native.default_context().bloom_test(bf.params, blob, off, bf.bytes)
    assert got.astype(bool).tolist() == [k in ref for k in keys]


def test_filter_or_reduce_is_the_union_of_shards():
    """Sharded large-filter build: per-shard filters OR-ed by dsy_filter_or_reduce == one filter over
    all keys (and == the oracle), for word counts with and without a 16-byte-vector tail."""
    import torch
    ctx = _native.default_context()
    dev = torch.device("cuda", 0)
    for m, f in ((1 << 20, 0.01), (10160, 0.01), (4104, 0.001)):
        blob, off = random_packets(m & 0xFFFF, 6000, 60, 700)
        keys = [blob[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]
        shards = [keys[i::3] for i in range(3)]
        parts = []
        for sh in shards:
            bf = BloomFilter(m, f, b"\x07")
            bf.add_keys(sh)
            raw = bf.bytes + b"\x00" * ((-len(bf.bytes)) % 4)
            parts.append(np.frombuffer(raw, dtype=np.int32))
        words = len(parts[0])
        d_parts = torch.from_numpy(np.concatenate(parts)).to(dev)
        d_out = torch.full((words,), -1, dtype=torch.int32, device=dev)
        _native.check(ctx.lib.dsy_filter_or_reduce(ctx.handle, d_parts.data_ptr(), 3, words, d_out.data_ptr()))
        ctx.synchronize()
        whole = BloomFilter(m, f, b"\x07")
        whole.add_keys(keys)
        ref = OracleBloom.from_m_f(m, f, b"\x07")
        ref.add_keys(keys)
        got = d_out.cpu().numpy().tobytes()[:m // 8]
        assert got == whole.bytes == ref.to_bytes()


def test_largest_filter_2_24_against_oracle():
    """cfg4's largest filter, BloomFilter(2**24, 0.01, b"\\x07") (SHA-256, 'L' chunks, k = 7): 200 k adds and 100 k
    probes against the oracle's bit positions (OracleBloom.indices, bloomfilter.py:150-160).  The positions are set
    in a numpy byte array in the filter's little-endian bit order (bloomfilter.py:288-298): the oracle's big-int OR
    costs O(m) per bit at 2 MB."""
    m = 1 << 24
    blob, off = random_packets(2424, 300_000, 100, 1500)
    n_add = 200_000
    bf = BloomFilter(m, 0.01, b"\x07")
    assert (bf.hash_name, bf.functions, bf.chunk_bytes) == ("sha256", 7, 4)
    bf.add_packed(blob[:int(off[n_add])], off[:n_add + 1])
    ref = OracleBloom.from_m_f(m, 0.01, b"\x07")
    pos = np.array([p for i in range(n_add) for p in ref.indices(blob[int(off[i]):int(off[i + 1])])], dtype=np.int64)
    want = np.zeros(m // 8, dtype=np.uint8)
    np.bitwise_or.at(want, pos >> 3, (1 << (pos & 7)).astype(np.uint8))
    assert bf.bytes == want.tobytes()
    assert bf.bits_checked == int(np.unpackbits(want).sum())
    probes = [blob[int(off[i]):int(off[i + 1])] for i in range(n_add - 1000, len(off) - 1)]
    got = bf.contains_many(probes)
    bits = np.unpackbits(want, bitorder="little")
    expect = [all(bits[p] for p in ref.indices(k)) for k in probes]
    assert got.astype(bool).tolist() == expect
    assert got[:1000].all() and sum(expect[1000:]) < 10


@pytest.mark.parametrize("or_mode", [0, 1, 2])
@pytest.mark.parametrize("m,f,prefix,n", [(10160, 0.01, b"\x00\x01\x02\x03", 40_000), (10160, 0.01, b"\x2a", 300),
                                          (4096, 0.001, b"x", 40_000), (1 << 20, 0.01, b"\x07", 5_000),
                                          (64, 0.5, b"", 3_000)])
def test_filter_build_or_modes(monkeypatch, or_mode, m, f, prefix, n):
    """Every filter-build mode (DSY_OR_MODE: per-lane atomics, skip-if-set, wave-aggregated leaders) gives the oracle's
    bytes: saturating MTU and SHA-1 filters (length-sorted, LDS-DMA), a sparse one, an HBM-resident 2^20 filter, and
    a 64-bit filter where most lanes of a wave hit the same word."""
    monkeypatch.setenv("DSY_OR_MODE", str(or_mode))
    ctx = _native.Context(0)
    try:
        blob, off = random_packets(m + n + or_mode, n, 60, 1500)
        bf = BloomFilter(m, f, prefix)
        got = ctx.bloom_add(bf.params, blob, off, b"\x00" * (len(bf.bytes) + (-len(bf.bytes)) % 4))
        ref = OracleBloom.from_m_f(m, f, prefix)
        ref.add_keys(blob[int(off[i]):int(off[i + 1])] for i in range(n))
        assert got[:len(bf.bytes)] == ref.to_bytes()
    finally:
        ctx.close()


@pytest.mark.parametrize("lines", [0, 3], ids=["windows", "lines"])
@pytest.mark.parametrize("m,f,prefix,n_add", [(10160, 0.01, b"\x00\x01\x02\x03", 1500), (4096, 0.001, b"x", 300),
                                              (10160, 0.01, b"", 1500), (10160, 0.01, b"\x05" * 5, 1500)],
                         ids=["md5-p4", "sha1-p1", "md5-p0", "md5-p5"])
def test_single_filter_staging_variants(monkeypatch, lines, m, f, prefix, n_add):
    """Single-filter membership over >= kLenSortMin keys (length-sorted, LDS-DMA staged k_bloom) under both staging
    variants (DSY_BLOOM_LINES: 0 = each key's own window, 3 = whole 128-byte lines for MD5 and SHA-1, with the 5-byte
    prefix falling back to windows) against the oracle: unaligned packed keys of 1..1500 bytes, a filter that is not
    saturated, so membership tells keys apart."""
    monkeypatch.setenv("DSY_BLOOM_LINES", str(lines))
    ctx = _native.Context(0)
    try:
        n = 40_000
        blob, off = random_packets(9000 + n_add + lines, n, 1, 1500)
        bf = BloomFilter(m, f, prefix)
        filt = ctx.bloom_add(bf.params, blob, off[:n_add + 1], b"\x00" * (len(bf.bytes) + (-len(bf.bytes)) % 4))
        ref = OracleBloom.from_m_f(m, f, prefix)
        keys = [blob[int(off[i]):int(off[i + 1])] for i in range(n)]
        ref.add_keys(keys[:n_add])
        assert filt[:len(bf.bytes)] == ref.to_bytes()
        got = ctx.bloom_test(bf.params, blob, off, filt)
        want = np.array([k in ref for k in keys], dtype=np.uint8)
        assert got[:n_add].all()
        assert 0 < int(want[n_add:].sum()) < n - n_add
        assert (got.astype(np.uint8) == want).all()
    finally:
        ctx.close()

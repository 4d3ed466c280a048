"""Host-side logic of the drop-in BloomFilter (CPU only, no device calls): sizing math, hash-family choice,
constructor overloads and errors, serialisation -- against the reference's golden vectors."""
import pytest

from dispersy_amd import BloomFilter
from dispersy_amd.bloomfilter import hash_family
from golden_util import load

BLOOM = load("bloom_vectors.json")


def test_ctor_vectors():
    for row in BLOOM["ctor"]:
        if row["ctor"] == "bad":
            continue
        args = (row["a"], row["b"])
        if "error" in row:
            with pytest.raises(Exception) as ei:
                BloomFilter(*args)
            assert type(ei.value).__name__ == row["error"], row
            continue
        bf = BloomFilter(*args)
        assert (bf.size, bf.functions, bf.hash_name, bf.chunk_bytes) == (row["m"], row["k"], row["hash"], row["chunk"])
        for f, cap in row.get("capacity", {}).items():
            assert bf.get_capacity(float(f)) == cap


def test_bad_overloads():
    # bloomfilter.py:114-115: any other argument-type combination is a RuntimeError
    for args in (("x", 3), (3, 3), (1.5, 0.5), (b"\x00", 1.0)):
        with pytest.raises(RuntimeError):
            BloomFilter(*args)
    with pytest.raises(AssertionError):
        BloomFilter(b"", 3)  # bloomfilter.py:85
    with pytest.raises(AssertionError):
        BloomFilter(12, 0.5)  # m % 8 (bloomfilter.py:95)
    with pytest.raises(AssertionError):
        BloomFilter(64, 0.5, "p")  # prefix must be bytes (bloomfilter.py:130)
    with pytest.raises(AssertionError):
        BloomFilter(64, 0.5, b"p" * 256)  # len(prefix) < 256 (bloomfilter.py:131)
    with pytest.raises(AssertionError):
        BloomFilter(1 << 16, 1e-9)  # > 512 digest bits (bloomfilter.py:144)


def test_serialisation_round_trip_host_only():
    raw = bytes(range(256)) * 5
    bf = BloomFilter(raw, 7, b"\x2a")
    assert bf.size == len(raw) * 8 and bf.bytes == raw and bf.prefix == b"\x2a"
    assert bf._filter == int.from_bytes(raw, "little")
    assert bf.bits_checked == bin(int.from_bytes(raw, "little")).count("1")
    bf.clear()
    assert bf.bytes == bytes(len(raw)) and bf.bits_checked == 0


def test_golden_bytes_load():
    for case in BLOOM["cases"]:
        e = case["expect"]
        if "bytes_hex" not in e:
            continue
        raw = bytes.fromhex(e["bytes_hex"])
        bf = BloomFilter(raw, e["k"], bytes.fromhex(e["prefix"]))
        assert bf.bits_checked == e["bits_checked"]
        assert (bf.hash_name, bf.chunk_bytes) == (e["hash"], e["chunk"])


def test_hash_family_table():
    assert hash_family(10160, 7) == ("md5", 2)
    assert hash_family(4096, 10) == ("sha1", 2)
    assert hash_family(1 << 20, 7) == ("sha256", 4)
    assert hash_family(1 << 31, 7) == ("sha512", 8)

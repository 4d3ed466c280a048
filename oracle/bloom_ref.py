"""ORACLE -- test infrastructure only.

A Python-3 CPU restatement of the reference Bloom filter (/root/reference/bloomfilter.py).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and only as the checker or
as the timed CPU baseline -- never as part of the product path (dispersy_amd/ never imports oracle/).

Parity pinning: tests/test_oracle_golden.py checks this restatement against tests/golden/bloom_vectors.json,
which gen_golden.py produced by running the reference's own bloomfilter.py (shimmed for Python 3).

The digest arithmetic is hashlib (OpenSSL), exactly what the reference calls (bloomfilter.py:25).  The bit
array is a Python int, as in the reference, so the CPU baseline keeps the reference's cost model
(O(m) per `1 << pos` at large m).
"""
import hashlib
import math
import struct

LN2 = math.log(2)


def capacity_for(m, f):
    """n = int(m * ln2^2 / |ln f|)  -- bloomfilter.py:73-75 (same float evaluation order)."""
    return int(m * (math.log(2) ** 2 / abs(math.log(f))))


def functions_for(m, n):
    """k = int(ceil(ln2 * m / n))  -- bloomfilter.py:69-71.  ZeroDivisionError when n == 0, as the reference."""
    return int(math.ceil(math.log(2) * m / n))


def bits_for(f, n):
    """m = int(ceil(|n ln f / ln2^2| / 8.0) * 8)  -- bloomfilter.py:110."""
    return int(math.ceil(abs((n * math.log(f)) / (math.log(2) ** 2)) / 8.0) * 8)


def hash_family(m, k):
    """(chunk_bytes, struct code, hashlib name) -- bloomfilter.py:134-156."""
    chunk, code = (8, "Q") if m >= 1 << 31 else (4, "L") if m >= 1 << 15 else (2, "H")
    need = chunk * k * 8
    if need > 512:
        raise AssertionError("cannot create a hash for %d bits" % need)
    for limit, name in ((128, "md5"), (160, "sha1"), (256, "sha256"), (384, "sha384"), (512, "sha512")):
        if need <= limit:
            return chunk, code, name
    raise AssertionError(need)


class OracleBloom(object):
    """Same observable behaviour as the reference BloomFilter for bytes keys."""

    def __init__(self, m, k, prefix=b"", bits=0):
        assert m > 0 and m % 8 == 0 and 0 < k <= m and 0 <= len(prefix) < 256
        self.m, self.k, self.prefix, self.bits = m, k, bytes(prefix), bits
        self.chunk, code, self.hash_name = hash_family(m, k)
        digest_size = hashlib.new(self.hash_name).digest_size
        # k big-endian unsigned chunks from the digest start, the rest skipped (bloomfilter.py:158-160)
        self._unpack = struct.Struct(">" + code * k + "x" * (digest_size - self.chunk * k)).unpack
        self._salt = hashlib.new(self.hash_name, self.prefix)

    # -- constructors mirroring the three overloads (bloomfilter.py:78-117)
    @classmethod
    def from_m_f(cls, m, f, prefix=b""):
        return cls(m, functions_for(m, capacity_for(m, f)), prefix)

    @classmethod
    def from_f_n(cls, f, n, prefix=b""):
        m = bits_for(f, n)
        return cls(m, functions_for(m, n), prefix)

    @classmethod
    def from_bytes(cls, raw, k, prefix=b""):
        assert len(raw) > 0
        return cls(len(raw) * 8, k, prefix, int.from_bytes(raw, "little"))

    # -- hashing
    def indices(self, key):
        h = self._salt.copy()
        h.update(key)
        return [c % self.m for c in self._unpack(h.digest())]

    def add(self, key):
        for pos in self.indices(key):
            self.bits |= 1 << pos

    def add_keys(self, keys):
        bits, m, unpack, salt_copy = self.bits, self.m, self._unpack, self._salt.copy
        for key in keys:
            h = salt_copy()
            h.update(key)
            for c in unpack(h.digest()):
                bits |= 1 << (c % m)
        self.bits = bits

    def __contains__(self, key):
        return all(self.bits >> pos & 1 for pos in self.indices(key))

    def not_filter(self, iterator):
        """Lazy: yields tuples whose first element has a zero probe bit (bloomfilter.py:214-237)."""
        bits, m, unpack, salt_copy = self.bits, self.m, self._unpack, self._salt.copy
        for tup in iterator:
            h = salt_copy()
            h.update(tup[0])
            for c in unpack(h.digest()):
                if not bits & (1 << (c % m)):
                    yield tup
                    break

    def to_bytes(self):
        """Little-endian bit order, m/8 bytes (bloomfilter.py:288-298)."""
        return self.bits.to_bytes(self.m // 8, "little")

    @property
    def bits_checked(self):
        return bin(self.bits).count("1")

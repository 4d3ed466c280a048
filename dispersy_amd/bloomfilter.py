"""Drop-in `BloomFilter` whose digest/probe work runs in hand-written HIP kernels on an MI355X.

Same constructor overloads, methods and properties as the reference (/root/reference/bloomfilter.py:34-298),
with Python-3 `bytes` where the reference had Python-2 `str`:

    BloomFilter(int m_size, float f_error_rate, prefix=b"")   bloomfilter.py:89-99
    BloomFilter(float f_error_rate, int n_capacity, prefix=b"") bloomfilter.py:101-112
    BloomFilter(bytes raw, int k_functions, prefix=b"")        bloomfilter.py:79-87

Host side (here): the sizing math, the hash-family choice and the serialisation.  Device side (libdsybloom.so):
every digest of `prefix || key`, its slicing into k big-endian chunks mod m, and the bit set/probe.  The filter
itself is kept as its serialised little-endian bytes (`.bytes`), which is the exact layout the kernels use.
There is no CPU path for the digests: without the HIP library, add/test raise `NativeUnavailable`.
"""
import ctypes
import struct
import logging
from math import ceil, log

import numpy as np

from . import _native

logger = logging.getLogger(__name__)

__all__ = ["BloomFilter", "hash_family"]

_DIGEST_BITS = ((128, "md5"), (160, "sha1"), (256, "sha256"), (384, "sha384"), (512, "sha512"))


def _n_capacity(m_size, f_error_rate):
    # bloomfilter.py:73-75 -- identical float expression, so identical rounding
    return int(m_size * (log(2) ** 2 / abs(log(f_error_rate))))


def _k_functions(m_size, n_capacity):
    # bloomfilter.py:69-71 (ZeroDivisionError when n_capacity == 0, as the reference)
    return int(ceil(log(2) * m_size / n_capacity))


def hash_family(m_size, k_functions):
    """(hash name, chunk bytes) chosen from (m, k) as bloomfilter.py:134-156 does."""
    chunk = 8 if m_size >= (1 << 31) else 4 if m_size >= (1 << 15) else 2
    bits_required = chunk * k_functions * 8
    assert bits_required <= 512, \
        "Combining multiple hashfunctions is not implemented, cannot create a hash for %d bits" % bits_required
    for limit, name in _DIGEST_BITS:
        if bits_required <= limit:
            return name, chunk
    raise AssertionError(bits_required)


def _overload(args, kargs):
    """The three constructor forms of bloomfilter.py:77-117."""
    if len(args) >= 2 and isinstance(args[0], (bytes, bytearray)) and isinstance(args[1], int):
        raw = bytes(args[0])
        prefix = kargs.get("prefix", args[2] if len(args) >= 3 else b"")
        assert 0 < len(raw), len(raw)
        return len(raw) * 8, args[1], prefix, raw
    if len(args) >= 2 and isinstance(args[0], int) and isinstance(args[1], float):
        m_size, f_error_rate = args[0], args[1]
        prefix = kargs.get("prefix", args[2] if len(args) >= 3 else b"")
        assert 0 < m_size, m_size
        assert m_size % 8 == 0, "size must be a multiple of eight (%d)" % m_size
        assert 0.0 < f_error_rate < 1.0, f_error_rate
        return m_size, _k_functions(m_size, _n_capacity(m_size, f_error_rate)), prefix, None
    if len(args) >= 2 and isinstance(args[0], float) and isinstance(args[1], int):
        f_error_rate, n_capacity = args[0], args[1]
        prefix = kargs.get("prefix", args[2] if len(args) >= 3 else b"")
        assert 0.0 < f_error_rate < 1.0, f_error_rate
        assert 0 < n_capacity, n_capacity
        m_size = int(ceil(abs((n_capacity * log(f_error_rate)) / (log(2) ** 2)) / 8.0) * 8)
        return m_size, _k_functions(m_size, n_capacity), prefix, None
    raise RuntimeError("Unknown combination of argument types %s" % str([type(arg) for arg in args]))


def pack_keys(keys):
    """list of bytes -> (blob, offsets u64[n+1]) -- the packed layout of the C-ABI."""
    n = len(keys)
    offsets = np.zeros(n + 1, dtype=np.uint64)
    if n:
        np.cumsum(np.fromiter(map(len, keys), dtype=np.int64, count=n), out=offsets[1:])
    return b"".join(keys), offsets


class BloomFilter(object):
    """Bloom filter with the reference's API; see module docstring."""

    # not_filter pulls the iterator in growing chunks (read-ahead is invisible to a read-only cursor)
    NOT_FILTER_FIRST_CHUNK = 256
    NOT_FILTER_MAX_CHUNK = 1 << 16

    def __init__(self, *args, **kargs):
        self._logger = logging.getLogger(self.__class__.__name__)
        m_size, k_functions, prefix, raw = _overload(args, kargs)
        assert isinstance(m_size, int), type(m_size)
        assert 0 < m_size, m_size
        assert m_size % 8 == 0, "size must be a multiple of eight (%d)" % m_size
        assert isinstance(k_functions, int), type(k_functions)
        assert 0 < k_functions <= m_size, [k_functions, m_size]
        assert isinstance(prefix, bytes), type(prefix)
        assert 0 <= len(prefix) < 256, len(prefix)
        self._m_size, self._k_functions, self._prefix = m_size, k_functions, prefix
        self._hash_name, self._chunk = hash_family(m_size, k_functions)
        self._raw = bytearray(raw) if raw is not None else bytearray(m_size // 8)
        # the filter bytes' address, for dsy_sync_respond_refs: the ctypes view exports the bytearray's buffer, so
        # it can never be reallocated under the address (every update is an equal-length slice assignment)
        self._view = (ctypes.c_char * len(self._raw)).from_buffer(self._raw)
        self._addr = ctypes.addressof(self._view)
        # this filter's part of a dsy_request (m, k, hash family, prefix; range and filter offset unused) and the two
        # addresses dsy_sync_respond_refs takes per claim, as 16 bytes: a batch's refs are one join
        q = self._req = _native.Request()
        q.m_bits, q.k, q.hash_kind, q.chunk_bytes = m_size, k_functions, _native.HASH_KINDS[self._hash_name], self._chunk
        q.prefix_len = len(prefix)
        ctypes.memmove(q.prefix, prefix, len(prefix))
        self._refs = struct.pack("<QQ", ctypes.addressof(q), self._addr)
        self._params = None
        self._record = None

    # ------------------------------------------------------------------------------------------ device
    @property
    def params(self):
        """The dsy_bloom_params of this filter (built lazily; needs the HIP library)."""
        if self._params is None:
            self._params = _native.bloom_params(self._m_size, self._k_functions, _native.HASH_KINDS[self._hash_name],
                                                self._chunk, self._prefix)
        return self._params

    @property
    def request_record(self):
        """This filter's part of a dsy_request record (m, k, hash family, prefix; the claim's range and the filter
        offset left zero), as bytes: built once -- the shape and prefix never change -- so a batch of claims is one
        join of records (SyncCommunity.request_records), not a field-by-field fill per claim."""
        if self._record is None:
            self._record = bytes(self._req)
        return self._record

    @staticmethod
    def _ctx():
        return _native.default_context()

    # ----------------------------------------------------------------------------------------- methods
    def add(self, key):
        """Add KEY to the BloomFilter (bloomfilter.py:163-172)."""
        self.add_keys((key,))

    def add_keys(self, keys):
        """Add a sequence of KEYS to the BloomFilter (bloomfilter.py:174-194); one kernel launch for all of them."""
        keys = keys if isinstance(keys, list) else list(keys)
        for key in keys:
            assert isinstance(key, bytes), type(key)
        if not keys:
            return
        blob, offsets = pack_keys(keys)
        self._raw[:] = self._ctx().bloom_add(self.params, blob, offsets, self._raw)

    def add_packed(self, blob, offsets):
        """Add keys already packed as (blob, offsets[n+1]) -- avoids building a list of bytes objects."""
        if len(offsets) > 1:
            self._raw[:] = self._ctx().bloom_add(self.params, blob, offsets, self._raw)

    def add_store_rows(self, store, rows):
        """Add the packets of `store` rows (a SyncStore already in HBM): the claim side's bloom.add_keys over
        selected rows (community.py:821, :924) without moving packets back to the host."""
        rows = np.ascontiguousarray(rows, dtype=np.uint64)
        if not len(rows):
            return
        ctx = store.ctx
        buf = ctypes.create_string_buffer(bytes(self._raw), len(self._raw))
        _native.check(ctx.lib.dsy_bloom_add_rows(ctx.handle, ctypes.byref(self.params), store.handle,
                                                 rows.ctypes.data, len(rows), buf))
        self._raw[:] = buf.raw

    def add_store_modulo(self, store, meta_ids, offset, modulo):
        """The claim side's modulo strategy on the device: select the live rows of `meta_ids` with
        (global_time + offset) % modulo == 0 (community.py:918, :922) and add their packets (:924) in one call
        (dsy_claim_modulo).  Returns the number of rows added."""
        ids = np.ascontiguousarray(meta_ids, dtype=np.uint32)
        ctx = store.ctx
        buf = ctypes.create_string_buffer(bytes(self._raw), len(self._raw))
        count = ctypes.c_uint64(0)
        _native.check(ctx.lib.dsy_claim_modulo(ctx.handle, ctypes.byref(self.params), store.handle, ids.ctypes.data,
                                               len(ids), int(offset), int(modulo), buf, ctypes.byref(count)))
        self._raw[:] = buf.raw
        return count.value

    def claim_largest(self, store, meta_ids, from_gbtime, capacity, nrsyncpackets, acceptable_global_time):
        """The largest claim strategy's selection and add_keys on the device (dsy_claim_largest, community.py:783-830
        after the random draws): returns (time_low, time_high, rows added, nrsyncpackets after); rows added 0 means
        the empty claim.  IndexError where the reference raises it (community.py:857)."""
        ids = np.ascontiguousarray(meta_ids, dtype=np.uint32)
        ctx = store.ctx
        buf = ctypes.create_string_buffer(bytes(self._raw), len(self._raw))
        out = (ctypes.c_uint64 * 4)()
        rc = ctx.lib.dsy_claim_largest(ctx.handle, ctypes.byref(self.params), store.handle, ids.ctypes.data, len(ids),
                                       int(from_gbtime), int(capacity), int(nrsyncpackets), int(acceptable_global_time),
                                       buf, out)
        if rc == _native.DSY_EEMPTY:
            raise IndexError("list index out of range")
        _native.check(rc)
        self._raw[:] = buf.raw
        return int(out[0]), int(out[1]), int(out[2]), int(out[3])

    def clear(self):
        """Set all bits in the filter to zero (bloomfilter.py:196-200)."""
        self._raw[:] = bytes(len(self._raw))

    def __contains__(self, key):
        """bloomfilter.py:202-212."""
        blob, offsets = pack_keys([key])
        return bool(self._ctx().bloom_test(self.params, blob, offsets, self._raw)[0])

    def contains_many(self, keys):
        """Vectorised __contains__: numpy bool array, one kernel launch."""
        keys = keys if isinstance(keys, list) else list(keys)
        if not keys:
            return np.zeros(0, dtype=bool)
        blob, offsets = pack_keys(keys)
        return self._ctx().bloom_test(self.params, blob, offsets, self._raw).astype(bool)

    def not_filter(self, iterator):
        """Yields all tuples in ITERATOR whose first element is NOT in the filter, lazily and in input order
        (bloomfilter.py:214-237).  Tuples are tested on the GPU in read-ahead chunks."""
        it = iter(iterator)
        chunk = self.NOT_FILTER_FIRST_CHUNK
        while True:
            batch = []
            for tup in it:
                assert isinstance(tup, tuple)
                assert len(tup) > 0
                assert isinstance(tup[0], bytes)
                batch.append(tup)
                if len(batch) >= chunk:
                    break
            if not batch:
                return
            present = self.contains_many([t[0] for t in batch])
            for tup, hit in zip(batch, present):
                if not hit:
                    yield tup
            if len(batch) < chunk:
                return
            chunk = min(chunk * 4, self.NOT_FILTER_MAX_CHUNK)

    def get_capacity(self, f_error_rate):
        """bloomfilter.py:239-246."""
        assert isinstance(f_error_rate, float)
        assert 0 < f_error_rate < 1
        return _n_capacity(self._m_size, f_error_rate)

    def get_bits_checked(self):
        """Deprecated accessor (bloomfilter.py:248-255)."""
        self._logger.warning("get_bits_checked function is deprecated, please use the bits_checked property")
        return self.bits_checked

    @property
    def bits_checked(self):
        """Number of set bits (bloomfilter.py:257-263)."""
        return int(np.unpackbits(np.frombuffer(bytes(self._raw), dtype=np.uint8)).sum())

    @property
    def size(self):
        return self._m_size

    @property
    def functions(self):
        return self._k_functions

    @property
    def prefix(self):
        return self._prefix

    @property
    def bytes(self):
        """Little-endian bit order, m/8 bytes (bloomfilter.py:288-298)."""
        return bytes(self._raw)

    @property
    def _filter(self):
        """The filter as an int, as the reference keeps it (read by community.py:729's debug log)."""
        return int.from_bytes(self._raw, "little")

    @property
    def hash_name(self):
        return self._hash_name

    @property
    def chunk_bytes(self):
        return self._chunk

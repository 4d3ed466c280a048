"""The introduction-request sync block on the wire (the reference's conversion.py:712-730 encode, :732-799 decode).

    struct '>QQHHBH'  time_low u64, time_high u64 (0: "up to your global time"), modulo u16, offset u16,
                      functions u8, size u16 (filter bits)                              conversion.py:193, :727
    prefix            1 byte                                                            :725, :769
    filter            size/8 bytes, BloomFilter.bytes, to the end of the payload        :787-791

Batches go through the C-ABI (dsy_sync_decode / dsy_sync_encode in include/dsybloom.h): a receive batch decodes
straight into the dsy_request records and aligned filter words the batched responder consumes, so no Python object
is built per claim.  The single-block helpers raise `DropPacket` with the reference's messages.
"""
import ctypes
import struct
from collections import namedtuple

import numpy as np

from . import _native
from .bloomfilter import BloomFilter

__all__ = ["DropPacket", "DROP_REASONS", "DECODE_ASSERT", "SyncBatch", "raise_for_status", "decode_sync_blocks", "encode_sync_blocks",
           "decode_sync_block", "encode_sync_block"]

SYNC_HEADER = _native.SYNC_HEADER


class DropPacket(Exception):
    """A sync block the reference's decoder drops (conversion.py:763-789)."""


# status code of dsy_sync_decode -> the reference's DropPacket message
DROP_REASONS = {
    1: "Insufficient packet size",
    2: "Invalid time_low value",
    3: "Invalid time_high value",
    4: "Invalid modulo value",
    5: "Invalid offset value",
    6: "Invalid functions value",
    7: "Invalid size value",
    8: "Invalid size value, must be a multiple of eight",
    9: "Invalid number of bytes available",
}
# status DSY_DECODE_ASSERT: the BloomFilter(bytes, k, prefix) constructor the decoder ends with (conversion.py:791)
# asserts 0 < k <= m and a <= 512-bit digest (bloomfilter.py:129, :144).  The reference raises that AssertionError out
# of the decoder -- no DropPacket -- and nothing on the receive path catches it (community.py:2086 catches DropPacket
# only), so the whole receive batch is abandoned.  Pinned by tests/golden/codec_vectors.json.
DECODE_ASSERT = 10

_U64 = (1 << 64) - 1

# a decoded receive batch: ctypes array of dsy_request (one per block; zeroed where status != 0), the packed
# filter words they point into, and the per-block status
SyncBatch = namedtuple("SyncBatch", "requests filters status")


def decode_sync_blocks(blocks, responder_global_time=0):
    """Decode a list of sync blocks (bytes from the block's first byte to the end of the payload).  With
    responder_global_time, time_high == 0 resolves to it and both bounds clamp to 2^63-1 (community.py:2545-2553)."""
    lib = _native.load_library()
    n = len(blocks)
    offsets = np.zeros(n + 1, dtype=np.uint64)
    if n:
        np.cumsum([len(b) for b in blocks], out=offsets[1:])
    blob = b"".join(bytes(b) for b in blocks)
    reqs = (_native.Request * max(n, 1))()
    status = np.zeros(max(n, 1), dtype=np.int32)
    cap = sum(((len(b) - SYNC_HEADER + 3) // 4) * 4 + 4 for b in blocks if len(b) >= SYNC_HEADER) + 64
    filters = ctypes.create_string_buffer(cap)
    used = ctypes.c_uint64()
    _native.check(lib.dsy_sync_decode(blob, offsets.ctypes.data, n, responder_global_time, reqs, filters, cap,
                                      ctypes.byref(used), status.ctypes.data))
    return SyncBatch(reqs, filters.raw[:used.value], status[:n])


def encode_sync_blocks(claims):
    """claims: iterable of (time_low, time_high, modulo, offset, BloomFilter) -> list of sync-block bytes."""
    lib = _native.load_library()
    claims = list(claims)
    n = len(claims)
    reqs = (_native.Request * max(n, 1))()
    parts, at = [], 0
    for i, (time_low, time_high, modulo, offset, bloom) in enumerate(claims):
        # conversion.py:723-726
        assert bloom.size % 8 == 0
        assert 0 < bloom.functions < 256
        assert len(bloom.prefix) == 1, "must have a one character prefix"
        # struct '>QQHHBH' (:727): a field that does not fit raises struct.error, as Struct.pack does
        if not (0 <= time_low <= _U64 and 0 <= time_high <= _U64 and 0 <= modulo <= 0xFFFF and
                0 <= offset <= 0xFFFF and bloom.size <= 0xFFFF):
            raise struct.error("sync block field out of range for '>QQHHBH'")
        q = reqs[i]
        q.time_low, q.time_high, q.modulo, q.offset = time_low, time_high, modulo, offset
        q.m_bits, q.k, q.prefix_len = bloom.size, bloom.functions, 1
        q.prefix[0] = bloom.prefix[0]
        q.filter_offset = at
        parts.append(bloom.bytes)
        at += len(bloom.bytes)
    filters = b"".join(parts)
    cap = at + SYNC_HEADER * n
    out = ctypes.create_string_buffer(max(cap, 1))
    offs = np.zeros(n + 1, dtype=np.uint64)
    _native.check(lib.dsy_sync_encode(reqs, n, filters, out, cap, offs.ctypes.data))
    raw = out.raw
    return [raw[int(offs[i]):int(offs[i + 1])] for i in range(n)]


def encode_sync_block(time_low, time_high, modulo, offset, bloom_filter):
    """The bytes _encode_introduction_request appends for payload.sync (conversion.py:721-728)."""
    return encode_sync_blocks([(time_low, time_high, modulo, offset, bloom_filter)])[0]


def raise_for_status(status, index=0):
    """The reference's verdict for a non-zero dsy_sync_decode status: DropPacket, or the AssertionError of the
    BloomFilter constructor (DECODE_ASSERT)."""
    if status == DECODE_ASSERT:
        raise AssertionError("BloomFilter(bytes, functions, prefix) of sync block %d asserts (bloomfilter.py:129, :144)"
                             % index)
    raise DropPacket(DROP_REASONS.get(status, "Invalid sync block (%d)" % status))


def decode_sync_block(data):
    """(time_low, time_high, modulo, offset, BloomFilter) of one sync block; DropPacket with the reference's message
    (conversion.py:762-789), or AssertionError where its BloomFilter constructor asserts (:791)."""
    batch = decode_sync_blocks([data])
    st = int(batch.status[0])
    if st:
        raise_for_status(st)
    q = batch.requests[0]
    raw = batch.filters[q.filter_offset:q.filter_offset + q.m_bits // 8]
    return q.time_low, q.time_high, q.modulo, q.offset, BloomFilter(raw, q.k, bytes([q.prefix[0]]))

"""ORACLE -- test infrastructure only (see oracle/bloom_ref.py for the rules).

Restatement of the introduction-request sync block codec of the reference: encode conversion.py:721-728, decode
conversion.py:762-794 (struct '>QQHHBH' of conversion.py:193, checks in the reference's order, the DropPacket
messages verbatim), plus the BloomFilter(bytes, functions, prefix) constructor asserts the decode ends with
(bloomfilter.py:79-87, :125-156).  Parity pinning: the reference's conversion.py needs Twisted/M2Crypto and cannot
be imported here, so this restatement is pinned by the format string and the checks it quotes.
"""
import struct
from math import ceil

from oracle.bloom_ref import hash_family

QQHHBH = struct.Struct(">QQHHBH")


class DropPacket(Exception):
    pass


def encode(time_low, time_high, modulo, offset, functions, size, prefix, filter_bytes):
    assert size % 8 == 0
    assert 0 < functions < 256
    assert len(prefix) == 1
    assert len(filter_bytes) == int(ceil(size / 8))
    return QQHHBH.pack(time_low, time_high, modulo, offset, functions, size) + prefix + filter_bytes


def decode(data, offset=0):
    """-> (time_low, time_high, modulo, offset, functions, size, prefix, filter_bytes) or DropPacket."""
    if len(data) < offset + 24:
        raise DropPacket("Insufficient packet size")
    time_low, time_high, modulo, modulo_offset, functions, size = QQHHBH.unpack_from(data, offset)
    offset += 23
    prefix = data[offset:offset + 1]
    offset += 1
    if not time_low > 0:
        raise DropPacket("Invalid time_low value")
    if not (time_high == 0 or time_low <= time_high):
        raise DropPacket("Invalid time_high value")
    if not 0 < modulo:
        raise DropPacket("Invalid modulo value")
    if not 0 <= modulo_offset < modulo:
        raise DropPacket("Invalid offset value")
    if not 0 < functions:
        raise DropPacket("Invalid functions value")
    if not 0 < size:
        raise DropPacket("Invalid size value")
    if not size % 8 == 0:
        raise DropPacket("Invalid size value, must be a multiple of eight")
    length = size // 8
    if not length == len(data) - offset:
        raise DropPacket("Invalid number of bytes available")
    # BloomFilter(data[offset:], functions, prefix=prefix): 0 < k <= m and a digest of <= 512 bits
    if functions > size:
        raise DropPacket("Invalid bloom filter parameters")
    try:
        hash_family(size, functions)
    except AssertionError:
        raise DropPacket("Invalid bloom filter parameters")
    return time_low, time_high, modulo, modulo_offset, functions, size, prefix, bytes(data[offset:offset + length])

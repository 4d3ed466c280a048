"""ORACLE -- test infrastructure only (see oracle/bloom_ref.py for the rules).

Restatement of the introduction-request sync block codec of the reference: encode conversion.py:721-728, decode
conversion.py:762-794 (struct '>QQHHBH' of conversion.py:193, checks in the reference's order, the DropPacket
messages verbatim), plus the BloomFilter(bytes, functions, prefix) constructor asserts the decode ends with
(bloomfilter.py:79-87, :125-156).  Parity pinning: tests/golden/codec_vectors.json holds the verdicts of the
reference's own _decode_introduction_request / _encode_introduction_request (lifted from conversion.py's AST by
tests/golden/gen_codec_golden.py) for 2400 fuzzed payloads and 171 claims; tests/test_oracle_golden.py checks this
restatement against them.
"""
import struct
from math import ceil

from oracle.bloom_ref import hash_family

QQHHBH = struct.Struct(">QQHHBH")


class DropPacket(Exception):
    pass


def encode(time_low, time_high, modulo, offset, functions, size, prefix, filter_bytes):
    """conversion.py:723-728: the asserts, then struct.pack (struct.error for a field that does not fit)."""
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
    # BloomFilter(data[offset:], functions, prefix=prefix) (conversion.py:791) asserts 0 < k <= m
    # (bloomfilter.py:129) and a digest of <= 512 bits (:144): AssertionError, not a DropPacket
    assert 0 < functions <= size, [functions, size]
    hash_family(size, functions)
    return time_low, time_high, modulo, modulo_offset, functions, size, prefix, bytes(data[offset:offset + length])

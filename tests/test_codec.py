"""The introduction-request sync block codec (conversion.py:712-799) of the C-ABI against the oracle restatement:
round trips, every DropPacket reason in the reference's order, truncation and a seeded fuzz.  Host code only (no
GPU): dsy_sync_decode / dsy_sync_encode parse bytes."""
import struct

import numpy as np
import pytest

from dispersy_amd import _native
from dispersy_amd.bloomfilter import BloomFilter
from dispersy_amd.conversion import (DECODE_ASSERT, DROP_REASONS, DropPacket, decode_sync_block, decode_sync_blocks,
                                     encode_sync_block, encode_sync_blocks)
from oracle import codec_ref

pytestmark = pytest.mark.skipif(not __import__("os").path.isfile(_native.LIB_PATH), reason="libdsybloom.so not built")

HDR = struct.Struct(">QQHHBH")


def block(time_low=1, time_high=0, modulo=1, offset=0, functions=7, size=10160, prefix=b"\x2a", body=None):
    body = bytes(range(256)) * (size // 8 // 256 + 1) if body is None else body
    return HDR.pack(time_low, time_high, modulo, offset, functions, size) + prefix + body[:size // 8]


def oracle_status(data):
    try:
        codec_ref.decode(data)
        return None
    except codec_ref.DropPacket as e:
        return str(e)
    except AssertionError:
        return "AssertionError"


def status_text(code):
    return None if code == 0 else "AssertionError" if code == DECODE_ASSERT else DROP_REASONS[code]


def test_round_trip_mtu_claim():
    ref = BloomFilter(10160, 0.01, prefix=b"\x11")
    bf = BloomFilter(np.random.Generator(np.random.PCG64(1)).bytes(10160 // 8), ref.functions, b"\x11")
    raw = encode_sync_block(5, 900, 3, 2, bf)
    assert raw == codec_ref.encode(5, 900, 3, 2, bf.functions, bf.size, bf.prefix, bf.bytes)
    lo, hi, mod, off, out = decode_sync_block(raw)
    assert (lo, hi, mod, off) == (5, 900, 3, 2)
    assert (out.size, out.functions, out.prefix, out.bytes) == (bf.size, bf.functions, bf.prefix, bf.bytes)


@pytest.mark.parametrize("kwargs,reason", [
    (dict(time_low=0), "Invalid time_low value"),
    (dict(time_low=10, time_high=9), "Invalid time_high value"),
    (dict(modulo=0), "Invalid modulo value"),
    (dict(modulo=4, offset=4), "Invalid offset value"),
    (dict(functions=0), "Invalid functions value"),
    (dict(size=0), "Invalid size value"),
    (dict(size=10161), "Invalid size value, must be a multiple of eight"),
])
def test_drop_reasons(kwargs, reason):
    data = block(**kwargs)
    assert oracle_status(data) == reason
    with pytest.raises(DropPacket, match="^" + reason.replace("(", r"\(") + "$"):
        decode_sync_block(data)


@pytest.mark.parametrize("kwargs", [dict(functions=200, size=40000), dict(functions=255, size=8),
                                    dict(functions=33, size=10160), dict(functions=17, size=32768)])
def test_bloom_constructor_asserts_are_not_drops(kwargs):
    """k > m or more than 512 digest bits: the reference's BloomFilter(bytes, k, prefix) asserts inside the decoder
    (bloomfilter.py:129, :144) -- an AssertionError, not a DropPacket (tests/golden/codec_vectors.json)."""
    data = block(**kwargs)
    assert oracle_status(data) == "AssertionError"
    assert int(decode_sync_blocks([data]).status[0]) == DECODE_ASSERT
    with pytest.raises(AssertionError):
        decode_sync_block(data)


def test_length_mismatch_and_truncation():
    good = block()
    for data in (good[:-1], good + b"\x00", good[:23], b""):
        want = oracle_status(data)
        assert want in ("Invalid number of bytes available", "Insufficient packet size")
        with pytest.raises(DropPacket) as e:
            decode_sync_block(data)
        assert str(e.value) == want


def test_batch_fuzz_against_oracle():
    rng = np.random.Generator(np.random.PCG64(2024))
    blocks = []
    for i in range(3000):
        size = int(rng.choice([8, 512 * 8, 10160, 65528, int(rng.integers(0, 70000))]))
        functions = int(rng.choice([1, 7, 10, int(rng.integers(0, 256))]))
        modulo = int(rng.integers(0, 5))
        data = block(time_low=int(rng.integers(0, 3)), time_high=int(rng.integers(0, 4)), modulo=modulo,
                     offset=int(rng.integers(0, 5)), functions=functions, size=size & 0xFFFF,
                     prefix=bytes([i & 255]), body=rng.bytes(size // 8 + 2))
        cut = int(rng.integers(0, 4))
        data = data[:len(data) - cut] if cut < 3 else data + b"\x00"
        blocks.append(data)
    batch = decode_sync_blocks(blocks, responder_global_time=77)
    for i, data in enumerate(blocks):
        want = oracle_status(data)
        got = int(batch.status[i])
        assert status_text(got) == want, i
        if not got:
            lo, hi, mod, off, k, m, prefix, body = codec_ref.decode(data)
            q = batch.requests[i]
            assert (q.time_low, q.time_high, q.modulo, q.offset, q.k, q.m_bits) == (lo, hi or 77, mod, off, k, m)
            assert bytes([q.prefix[0]]) == prefix and q.filter_offset % 4 == 0
            assert batch.filters[q.filter_offset:q.filter_offset + m // 8] == body
            assert (q.hash_kind, q.chunk_bytes) == (_native.HASH_KINDS[BloomFilter(body, k).hash_name], BloomFilter(body, k).chunk_bytes)


def test_encode_rejects_what_the_wire_cannot_carry():
    with pytest.raises(AssertionError):
        encode_sync_block(1, 0, 1, 0, BloomFilter(10160, 0.01, prefix=b"ab"))
    with pytest.raises(struct.error):
        encode_sync_block(1, 0, 65536, 0, BloomFilter(4096, 0.001, prefix=b"a"))
    # only the decoder validates time_low / modulo / offset: the encoder writes them as given (conversion.py:727)
    raw = encode_sync_block(0, 0, 0, 3, BloomFilter(4096, 0.001, prefix=b"a"))
    assert HDR.unpack_from(raw)[:4] == (0, 0, 0, 3)
    many = encode_sync_blocks([(i + 1, 0, 7, i % 7, BloomFilter(4096, 0.001, prefix=bytes([i]))) for i in range(50)])
    assert all(len(b) == 24 + 512 for b in many)
    assert [decode_sync_block(b)[:4] for b in many] == [(i + 1, 0, 7, i % 7) for i in range(50)]


# ------------------------------------------------------------------ pinned by the reference (codec_vectors.json)
def _golden_decode_cases():
    import hashlib
    import codec_cases
    from golden_util import load
    vec = load("codec_vectors.json")["decode"]
    payloads = codec_cases.decode_payloads()
    assert len(payloads) == len(vec)
    out = []
    for p, rec in zip(payloads, vec):
        assert hashlib.sha256(p).hexdigest()[:16] == rec["sha256"], "codec_cases drifted from the golden file"
        flags = p[18]
        if rec.get("drop") == "Invalid connection type flag" or not flags & 0x02:
            continue  # decided by the introduction-request header before the sync block (conversion.py:751-761)
        out.append((p[21:], rec))
    return out


def _expected(rec):
    if "drop" in rec:
        return rec["drop"]
    if "error" in rec:
        return rec["error"]
    return None


def test_decode_matches_reference_vectors():
    """dsy_sync_decode reproduces the reference decoder's verdict on every fuzzed sync block: the decoded claim
    (filter bytes by digest), the DropPacket message, or the BloomFilter constructor's AssertionError."""
    import hashlib
    cases = _golden_decode_cases()
    assert len(cases) > 2000
    blocks = [b for b, _ in cases]
    batch = decode_sync_blocks(blocks, responder_global_time=0)
    kinds = set()
    for i, (blk, rec) in enumerate(cases):
        want = _expected(rec)
        kinds.add(want)
        assert status_text(int(batch.status[i])) == want, (i, rec)
        assert oracle_status(blk) == want, (i, rec)
        if want is None:
            s, q = rec["sync"], batch.requests[i]
            assert (q.time_low, q.time_high, q.modulo, q.offset, q.k, q.m_bits) == (
                s["time_low"], s["time_high"], s["modulo"], s["offset"], s["functions"], s["size"])
            assert bytes([q.prefix[0]]).hex() == s["prefix"]
            body = batch.filters[q.filter_offset:q.filter_offset + q.m_bits // 8]
            assert hashlib.sha256(body).hexdigest()[:16] == s["filter_sha256"]
    assert "AssertionError" in kinds and None in kinds and "Invalid offset value" in kinds


def test_encode_matches_reference_vectors():
    import hashlib
    import codec_cases
    from golden_util import load
    for rec in load("codec_vectors.json")["encode"]:
        time_low, time_high, modulo, offset, m, k, prefix, seed = rec["claim"]
        body = codec_cases.filter_body(m, seed)
        try:
            bf = BloomFilter(body, k, bytes.fromhex(prefix))
        except AssertionError:
            assert rec.get("error") == "AssertionError" and rec.get("stage") == "BloomFilter", rec
            continue
        try:
            raw = encode_sync_block(time_low, time_high, modulo, offset, bf)
        except AssertionError:
            assert rec.get("error") == "AssertionError", rec
            continue
        except struct.error:
            assert rec.get("error") == "error", rec  # struct.error
            continue
        assert "error" not in rec, rec
        assert len(raw) == rec["length"] and hashlib.sha256(raw).hexdigest() == rec["sha256"]
        if "hex" in rec:
            assert raw.hex() == rec["hex"]

"""Deterministic inputs of the sync-block codec vectors (test infrastructure, shared by gen_codec_golden.py and
tests/test_codec.py): introduction-request payloads (conversion.py:732-799 decodes them) and claims to encode
(:712-730).  Everything derives from fixed numpy PCG64 seeds; the golden file stores only the reference's verdicts
plus a digest of each payload."""
import struct

import numpy as np

HEADER = struct.Struct(">4sH4sH4sHBH")  # destination, source lan, source wan (ip, port), flags, identifier: 21 B
SYNC = struct.Struct(">QQHHBH")          # conversion.py:193

SIZES = [0, 8, 10, 16, 64, 512 * 8, 9808, 10160, 10304, 32760, 32768, 65528, 65535]
FUNCTIONS = [0, 1, 2, 7, 8, 10, 16, 17, 20, 32, 33, 64, 255]


def filter_body(m, seed):
    return np.random.Generator(np.random.PCG64(seed)).bytes(m // 8)


def _pick(rng, values):
    return values[int(rng.integers(0, len(values)))]


def _u64(rng):
    return int(rng.integers(0, 1 << 62)) * 4 + int(rng.integers(0, 4))


def decode_payloads(n=2400, seed=8080):
    rng = np.random.Generator(np.random.PCG64(seed))
    out = []
    for i in range(n):
        flags = _pick(rng, [0x02, 0x03, 0x82, 0x83, 0xC2, 0xC3])
        if i % 97 == 5:
            flags = 0x42  # connection type 01: "Invalid connection type flag"
        elif i % 89 == 7:
            flags = _pick(rng, [0x00, 0x81, 0xC0])  # no sync block
        head = HEADER.pack(bytes(rng.integers(0, 256, 4, dtype=np.uint8)), int(rng.integers(0, 65536)),
                           bytes(rng.integers(0, 256, 4, dtype=np.uint8)), int(rng.integers(0, 65536)),
                           bytes(rng.integers(0, 256, 4, dtype=np.uint8)), int(rng.integers(0, 65536)),
                           flags, int(rng.integers(0, 65536)))
        r = rng.random
        time_low = _pick(rng, [0, 1, 2, 1000, 2 ** 63 - 1, 2 ** 63, 2 ** 64 - 1]) if r() < 0.5 else _u64(rng)
        t = r()
        time_high = (0 if t < 0.3 else time_low if t < 0.4 else max(time_low - 1, 0) if t < 0.5 else
                     min(time_low + int(rng.integers(0, 1 << 40)), 2 ** 64 - 1) if t < 0.9 else _u64(rng))
        modulo = _pick(rng, [0, 1, 1, 2, 7, 9443, 65535]) if r() < 0.7 else int(rng.integers(0, 65536))
        t = r()
        offset = 0 if t < 0.4 else max(modulo - 1, 0) if t < 0.6 else modulo if t < 0.7 else int(rng.integers(0, 65536))
        functions = _pick(rng, FUNCTIONS) if r() < 0.8 else int(rng.integers(0, 256))
        size = _pick(rng, SIZES) if r() < 0.85 else int(rng.integers(0, 65536))
        prefix = bytes([int(rng.integers(0, 256))])
        body = rng.bytes((size + 7) // 8)
        t = r()
        if t < 0.05:
            body = body[:-1]
        elif t < 0.08:
            body = body + b"\x00"
        elif t < 0.1:
            body = b""
        block = SYNC.pack(time_low, time_high, modulo, offset, functions, size) + prefix + body
        if i % 61 == 3:
            block = block[:int(rng.integers(0, 24))]  # header cut short: "Insufficient packet size"
        out.append(head + block)
    return out


def encode_claims():
    """(time_low, time_high, modulo, offset, m, k, prefix_hex, body_seed)."""
    rng = np.random.Generator(np.random.PCG64(9090))
    claims = []
    for i in range(160):
        m = _pick(rng, [8, 64, 512 * 8, 9808, 10160, 32768, 65528])
        k = _pick(rng, [1, 4, 7, 10, 16])
        modulo = _pick(rng, [1, 3, 9443, 65535])
        claims.append((int(rng.integers(1, 1 << 40)), _pick(rng, [0, 1 << 41]), modulo,
                       int(rng.integers(0, modulo)), m, k, bytes([i & 255]).hex(), 100 + i))
    # what the wire cannot carry: the asserts of conversion.py:723-726 and the '>QQHHBH' field widths
    claims += [(1, 0, 1, 0, 10160, 7, "", 1), (1, 0, 1, 0, 10160, 7, "4142", 2), (1, 0, 65536, 0, 4096, 10, "41", 3),
               (1, 0, 7, 65536, 4096, 10, "41", 4), (2 ** 64, 0, 1, 0, 4096, 10, "41", 5), (1, 0, 1, 0, 65536, 7, "41", 6),
               (1, 2 ** 64, 1, 0, 4096, 10, "41", 7), (0, 0, 1, 0, 4096, 10, "41", 8), (1, 0, 0, 0, 4096, 10, "41", 9),
               (1, 0, 1, 0, 8, 2, "41", 10), (1, 0, 1, 0, 8, 9, "41", 11)]
    return claims

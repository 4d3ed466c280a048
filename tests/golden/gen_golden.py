"""Generate golden vectors for the Bloom-filter sync hot path FROM THE REFERENCE ITSELF.

Test infrastructure.  Runs only in the survey/build container, where /root/reference exists; it refuses to
run anywhere else.  Nothing from the reference is copied into the repository: the reference module lives
only in this process's memory, and only the generated input/output vectors (JSON / gzip'd binaries under
tests/golden/) are committed.

How the Python-2 reference is run under Python 3:
  * /root/reference/bloomfilter.py is read as text and three py2-isms are rewritten in memory:
    integer `/` -> `//` (bloomfilter.py:160, :297) and the `""` default prefix -> `b""` (:84, :93, :105).
    The text is exec'd into a fresh namespace that pre-binds `long = int` and `str = bytes`, so its
    `isinstance(..., str)` asserts mean bytes.  Every other line runs as written.
  * community.py cannot be imported (Twisted/M2Crypto/libnacl are absent).  The five sync-path methods
    (`_get_packets_for_bloomfilters` community.py:2746-2811, `_select_and_fix` :881-903,
    `_select_bloomfilter_range` :839-879, `_dispersy_claim_sync_bloom_filter_largest` :763-837 and
    `_dispersy_claim_sync_bloom_filter_modulo` :908-933) are lifted out of the module's AST unchanged and
    bound to a stub object whose database is an sqlite3 connection built from the reference's own schema
    string (dispersydatabase.py:17-68).  Run with `python -O` so `if __debug__:` log blocks (which call
    py2-only `str.encode("HEX")`) are compiled out.

Usage:  PYTHONDONTWRITEBYTECODE=1 python -O tests/golden/gen_golden.py
"""
import ast
import gzip
import hashlib
import json
import math
import os
import random as _pyrandom
import sqlite3
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from keys import named_packets, packet_list  # noqa: E402

REF = "/root/reference"


def _require_reference():
    if not os.path.isfile(os.path.join(REF, "bloomfilter.py")):
        raise SystemExit("gen_golden.py: /root/reference is absent -- the golden vectors are generated only in the "
                         "build container; the committed fixtures under tests/golden/ are the artefact.")


def load_reference_bloomfilter():
    src = open(os.path.join(REF, "bloomfilter.py")).read()
    for old, new, count in (("bits_required / 8", "bits_required // 8", 1),
                            ("self._m_size / 4", "self._m_size // 4", 1),
                            ('else "")', 'else b"")', 3)):
        assert src.count(old) == count, (old, src.count(old))
        src = src.replace(old, new)
    mod = types.ModuleType("ref_bloomfilter")
    mod.__dict__.update({"long": int, "str": bytes, "__name__": "ref_bloomfilter"})
    exec(compile(src, "ref_bloomfilter.py", "exec"), mod.__dict__)
    return mod


# ----------------------------------------------------------------------------------------------- bloom vectors
def key_spec_keys(spec):
    kind = spec["kind"]
    if kind == "named":
        return named_packets(spec["n"], spec.get("start", 0), spec.get("fmt", "packet-%d").encode())
    if kind == "random":
        return packet_list(spec["seed"], spec["n"], spec["lo"], spec["hi"])
    if kind == "str_int":
        return [str(i).encode() for i in range(spec["start"], spec["stop"])]
    if kind == "ragged":
        import numpy as np
        rng = np.random.Generator(np.random.PCG64(spec["seed"]))
        return [rng.bytes(n) for n in spec["lengths"]]
    raise ValueError(kind)


def hash_name(bf):
    return bf._salt.name


def chunk_of(bf):
    return {"H": 2, "L": 4, "Q": 8}[[c for c in "HLQ" if c in bf._fmt_unpack.__self__.format][0]]


def make_filter(B, case):
    ctor = case["ctor"]
    prefix = bytes.fromhex(case["prefix"])
    if ctor[0] == "m_f":
        return B.BloomFilter(ctor[1], float(ctor[2]), prefix)
    if ctor[0] == "f_n":
        return B.BloomFilter(float(ctor[1]), ctor[2], prefix)
    raise ValueError(ctor)


RAGGED = list(range(0, 131)) + [183, 184, 191, 192, 247, 248, 255, 256, 1000, 1500, 4096, 9000]

BLOOM_CASES = [
    # SURVEY §8c KAT anchors
    dict(name="mtu_md5_kat", ctor=("m_f", 10160, 0.01), prefix="2a", keys=dict(kind="named", n=1000),
         probes=dict(kind="named", n=2000, start=500)),
    dict(name="node_sha1_kat", ctor=("m_f", 4096, 0.001), prefix="78", keys=dict(kind="named", n=300),
         probes=dict(kind="named", n=2000, start=150)),
    dict(name="large_sha256_kat", ctor=("m_f", 1 << 20, 0.01), prefix="07", keys=dict(kind="named", n=10000),
         probes=dict(kind="named", n=4000, start=8000)),
    # BASELINE config 1 at capacity: 4-byte prefix, random 100-1500 B packets
    dict(name="cfg1_capacity_md5", ctor=("m_f", 10160, 0.01), prefix="00010203",
         keys=dict(kind="random", seed=1234, n=1059, lo=100, hi=1500),
         probes=dict(kind="random", seed=4321, n=3000, lo=100, hi=1500)),
    # every production MTU size
    dict(name="mtu_10304", ctor=("m_f", 10304, 0.01), prefix="ff", keys=dict(kind="random", seed=11, n=1075, lo=60, hi=1500),
         probes=dict(kind="random", seed=12, n=1000, lo=60, hi=1500)),
    dict(name="mtu_9808", ctor=("m_f", 9808, 0.01), prefix="00", keys=dict(kind="random", seed=13, n=1023, lo=60, hi=1500),
         probes=dict(kind="random", seed=14, n=1000, lo=60, hi=1500)),
    dict(name="mtu_sha1_f001", ctor=("m_f", 10160, 0.001), prefix="41", keys=dict(kind="random", seed=15, n=706, lo=60, hi=1500),
         probes=dict(kind="random", seed=16, n=1000, lo=60, hi=1500)),
    # hash families / chunk widths
    dict(name="l_sha256_32768", ctor=("m_f", 32768, 0.01), prefix="10", keys=dict(kind="random", seed=17, n=3418, lo=60, hi=700),
         probes=dict(kind="random", seed=18, n=2000, lo=60, hi=700)),
    dict(name="l_sha384", ctor=("m_f", 32768, 0.001), prefix="20", keys=dict(kind="random", seed=19, n=2000, lo=1, hi=600),
         probes=dict(kind="random", seed=20, n=2000, lo=1, hi=600)),
    dict(name="l_sha512", ctor=("m_f", 65536, 0.0001), prefix="30", keys=dict(kind="random", seed=21, n=2000, lo=1, hi=600),
         probes=dict(kind="random", seed=22, n=2000, lo=1, hi=600)),
    dict(name="h_sha512", ctor=("m_f", 16384, 1e-8), prefix="31", keys=dict(kind="random", seed=23, n=300, lo=1, hi=300),
         probes=dict(kind="random", seed=24, n=1000, lo=1, hi=300)),
    dict(name="l_md5_nopad", ctor=("m_f", 32768, 0.1), prefix="40", keys=dict(kind="random", seed=25, n=6000, lo=1, hi=300),
         probes=dict(kind="random", seed=26, n=2000, lo=1, hi=300)),
    dict(name="h_sha256_k", ctor=("m_f", 8192, 0.00001), prefix="50", keys=dict(kind="random", seed=27, n=300, lo=1, hi=300),
         probes=dict(kind="random", seed=28, n=1000, lo=1, hi=300)),
    # empty "no-sync" filter (community.py:837)
    dict(name="nosync_8", ctor=("m_f", 8, 0.1), prefix="00", keys=dict(kind="named", n=0),
         probes=dict(kind="named", n=50)),
    # test_bloomfilter.py shapes (FP-rate configs, keys str(i))
    *[dict(name="fp_%s_%g_%d" % (p or "none", f, n), ctor=("f_n", f, n), prefix=p.encode().hex(),
           keys=dict(kind="str_int", start=0, stop=n), probes=dict(kind="str_int", start=n, stop=n + 10000))
      for p in ("", "p") for n in (128, 1024) for f in (0.1, 0.2, 0.3, 0.4)],
    dict(name="fixed_128x8_p", ctor=("m_f", 1024, 0.25), prefix="70", keys=dict(kind="str_int", start=0, stop=100),
         probes=dict(kind="str_int", start=0, stop=300)),
    # ragged key lengths across every MD padding boundary, for each hash family
    *[dict(name="ragged_%s" % tag, ctor=ctor, prefix="5a", keys=dict(kind="ragged", seed=31 + i, lengths=RAGGED),
           probes=dict(kind="ragged", seed=31 + i, lengths=RAGGED))
      for i, (tag, ctor) in enumerate((("md5", ("m_f", 10160, 0.01)), ("sha1", ("m_f", 4096, 0.001)),
                                       ("sha256", ("m_f", 1 << 16, 0.01)), ("sha384", ("m_f", 1 << 16, 0.001)),
                                       ("sha512", ("m_f", 1 << 16, 0.0001))))],
    # prefix lengths across block boundaries (the salt carries a partially/fully absorbed prefix)
    *[dict(name="prefix%d_%s" % (plen, tag), ctor=ctor, prefix=bytes((j * 37 + 11) & 0xFF for j in range(plen)).hex(),
           keys=dict(kind="ragged", seed=77 + plen, lengths=list(range(0, 70)) + [127, 128, 129, 300]),
           probes=dict(kind="ragged", seed=77 + plen, lengths=list(range(0, 70)) + [127, 128, 129, 300]))
      for plen in (0, 55, 56, 63, 64, 65, 111, 112, 127, 128, 129, 200, 255)
      for tag, ctor in (("md5", ("m_f", 10160, 0.01)), ("sha512", ("m_f", 1 << 16, 0.0001)))],
]


def run_bloom_case(B, case):
    keys = key_spec_keys(case["keys"])
    probes = key_spec_keys(case["probes"])
    bf = make_filter(B, case)
    bf.add_keys(iter(keys))
    m = bf.size
    fmt = bf._fmt_unpack

    def indices(key):
        h = bf._salt.copy()
        h.update(key)
        return [pos % m for pos in fmt(h.digest())]

    present = [1 if p in bf else 0 for p in probes]
    tuples = [(p, i) for i, p in enumerate(probes)]
    missing = [i for _, i in bf.not_filter(iter(tuples))]
    raw = bf.bytes
    out = dict(case)
    out["expect"] = dict(
        m=m, k=bf.functions, hash=hash_name(bf), chunk=chunk_of(bf), prefix=bf.prefix.hex(),
        bits_checked=bin(bf._filter).count("1"), bytes_sha256=hashlib.sha256(raw).hexdigest(),
        indices=[indices(key) for key in keys[:64]],
        probe_indices=[indices(p) for p in probes[:16]],
        present=present, missing=missing)
    if m <= 1 << 16:
        out["expect"]["bytes_hex"] = raw.hex()
    else:
        fn = "bloom_%s.bin.gz" % case["name"]
        with gzip.open(os.path.join(HERE, fn), "wb", compresslevel=9) as f:
            f.write(raw)
        out["expect"]["bytes_file"] = fn
    # round trip through the (bytes, k, prefix) constructor (bloomfilter.py:79-87)
    clone = B.BloomFilter(raw, bf.functions, bf.prefix)
    assert clone.bytes == raw and clone.size == m
    return out


def chunk_q_vectors(B):
    """m >= 2^31 selects 8-byte 'Q' chunks (bloomfilter.py:135-136).  Building such a filter in the reference
    allocates a 256 MB int per probe, so only the digest->index slicing is recorded."""
    res = []
    for m, f, prefix in (((1 << 31), 0.01, b"\x01"), ((1 << 31) + 8, 0.1, b"qq"), ((1 << 33), 0.05, b"")):
        bf = B.BloomFilter(m, f, prefix)
        keys = packet_list(901, 64, 0, 400)
        rows = []
        for key in keys:
            h = bf._salt.copy()
            h.update(key)
            rows.append([pos % m for pos in bf._fmt_unpack(h.digest())])
        res.append(dict(m=m, f=f, prefix=prefix.hex(), keys=dict(kind="random", seed=901, n=64, lo=0, hi=400),
                        k=bf.functions, hash=hash_name(bf), chunk=chunk_of(bf), indices=rows))
    return res


def ctor_vectors(B):
    """Sizing math of the three constructor overloads (bloomfilter.py:69-117) incl. the error cases."""
    rows = []
    for m in (8, 16, 64, 128, 1024, 4096, 9488, 9808, 10128, 10160, 10304, 32760, 32768, 65536, 1 << 20, 1 << 24):
        for f in (0.5, 0.25, 0.1, 0.01, 0.001, 0.0001, 1e-6, 1e-8):
            try:
                bf = B.BloomFilter(m, f)
                rows.append(dict(ctor="m_f", a=m, b=f, m=bf.size, k=bf.functions, hash=hash_name(bf), chunk=chunk_of(bf),
                                 capacity={str(g): bf.get_capacity(g) for g in (0.1, 0.01, 0.001)}))
            except Exception as e:  # noqa: BLE001 - the exception type is the vector
                rows.append(dict(ctor="m_f", a=m, b=f, error=type(e).__name__))
    for f in (0.4, 0.3, 0.2, 0.1, 0.01, 0.001):
        for n in (1, 2, 10, 128, 142, 1024, 1059, 100000):
            try:
                bf = B.BloomFilter(f, n)
                rows.append(dict(ctor="f_n", a=f, b=n, m=bf.size, k=bf.functions, hash=hash_name(bf), chunk=chunk_of(bf)))
            except Exception as e:  # noqa: BLE001
                rows.append(dict(ctor="f_n", a=f, b=n, error=type(e).__name__))
    for bad in ((b"", 3), ("x", 3), (3, 3), (1.5, 0.5), (12, 0.5)):
        try:
            B.BloomFilter(*bad)
            rows.append(dict(ctor="bad", a=repr(bad), error=None))
        except Exception as e:  # noqa: BLE001
            rows.append(dict(ctor="bad", a=repr(bad), error=type(e).__name__))
    return rows


def main():
    _require_reference()
    B = load_reference_bloomfilter()
    bloom = [run_bloom_case(B, c) for c in BLOOM_CASES]
    with open(os.path.join(HERE, "bloom_vectors.json"), "w") as f:
        json.dump(dict(generator="tests/golden/gen_golden.py", source="/root/reference/bloomfilter.py (shimmed)",
                       cases=bloom, chunk_q=chunk_q_vectors(B), ctor=ctor_vectors(B)), f, separators=(",", ":"))
    print("bloom cases:", len(bloom))
    import gen_sync_golden
    gen_sync_golden.main(B)


if __name__ == "__main__":
    main()

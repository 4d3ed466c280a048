"""tests/oracle_pool.py (the full-size tests' fanned-out oracle) against oracle/sync_ref.respond_arrays run in this
process, on a small store: the same answers for every claim.  CPU only."""
import hashlib

import numpy as np

from oracle import sync_ref
from oracle.bloom_ref import OracleBloom
from oracle_pool import _Identity, check_claims


def test_pool_matches_in_process_oracle():
    rng = np.random.default_rng(3)
    n = 4000
    lens = rng.integers(20, 400, n)
    off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    blob = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    gts = np.sort(rng.integers(1, 1500, n)).astype(np.uint64)
    claims = []
    for i in range(24):
        bloom = OracleBloom.from_m_f(1024, 0.01, bytes([i]))
        lo, hi = (int(rng.integers(1, 700)), int(rng.integers(700, 1500))) if i % 2 else (1, 1499)
        modulo = 1 if i % 3 else 7
        offset = int(rng.integers(0, modulo))
        for r in rng.choice(n, 300, replace=False):
            bloom.add(blob[off[r]:off[r + 1]].tobytes())
        raw = bloom.to_bytes()
        claims.append((lo, hi, offset, modulo, raw, bloom.k, bytes([i])))
    rows = np.arange(n, dtype=np.int64)
    got = check_claims(claims, blob, off, rows, gts, 2000, 3000)
    metas = [dict(name="m", id=1, direction="ASC", priority=128, pruning=None)]
    for c, g in zip(claims, got):
        want = sync_ref.respond_arrays(lambda r: blob[off[r]:off[r + 1]].tobytes(), {1: (_Identity(), gts)}, metas,
                                       c[:4], OracleBloom.from_bytes(c[4], c[5], c[6]), 2000, 3000)
        assert g == want
    assert sum(map(len, got)) > 24
    assert hashlib.md5(b"").hexdigest()  # (hashlib is what both sides hash with)

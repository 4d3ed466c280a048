"""Claim side, largest strategy on the device: dsy_claim_largest runs the range selection of
`_dispersy_claim_sync_bloom_filter_largest` -- `_select_bloomfilter_range` / `_select_and_fix` (community.py:839-903)
-- over the store's HBM index and ORs the selected packets into the claim filter (:821).

The 80 reference-generated claim calls of tests/golden/sync_vectors.json go through it in test_sync_golden.py; here
the oracle (oracle/sync_ref.claim_largest: the reference's SELECT ... ORDER BY global_time LIMIT ? text in sqlite3)
checks it at larger sizes: many metas (the rank-across-metas path, in LDS and -- past 8192 candidates -- in global
scratch), thousands of rows sharing a global time (the trailing-group drop), appended rows, and the
`from_gbtime <= 1 / _nrsyncpackets < capacity` branch.  Every random draw of the community is replayed into the
oracle, so claims are compared exactly: range, filter bytes and _nrsyncpackets."""
import random

import numpy as np
import pytest

from dispersy_amd import BloomFilter
from dispersy_amd.community import SyncCommunity
from dispersy_amd.distribution import MetaMessage, SyncDistribution
from dispersy_amd.store import SyncStore
from golden_util import SYNC_SCHEMA, Replay
from oracle import sync_ref
from oracle.bloom_ref import OracleBloom

pytestmark = pytest.mark.gpu


class Recorder(object):
    """A seeded Random whose draws are logged, for Replay in the oracle."""

    def __init__(self, seed):
        self.rng, self.log = random.Random(seed), []

    def random(self):
        v = self.rng.random()
        self.log.append(("random", v))
        return v

    def expovariate(self, lambd):
        v = self.rng.expovariate(lambd)
        self.log.append(("expovariate", v))
        return v

    def randint(self, a, b):
        v = self.rng.randint(a, b)
        self.log.append(("randint", v))
        return v


def build(seed, n, n_metas, gt_max, ties):
    import sqlite3
    rng = np.random.Generator(np.random.PCG64(seed))
    rows = []
    for i in range(n):
        meta = int(rng.integers(1, n_metas + 1))
        gt = int(rng.integers(1, gt_max)) if not ties or rng.random() < 0.7 else int(rng.integers(1, 6)) * (gt_max // 6)
        rows.append((i + 1, gt, meta, int(rng.random() < 0.02), i.to_bytes(4, "big") + rng.bytes(int(rng.integers(20, 200)))))
    conn = sqlite3.connect(":memory:")
    conn.executescript(SYNC_SCHEMA)
    conn.executemany("INSERT INTO sync(id, community, member, global_time, meta_message, undone, packet, sequence) "
                     "VALUES (?, 1, ?, ?, ?, ?, ?, 0)", [(r[0], r[0], r[1], r[2], r[3], r[4]) for r in rows])
    return rows, conn


@pytest.mark.parametrize("n,n_metas,bits,ties", [
    (30_000, 1, 10160, False),   # one meta: the cut is an index
    (30_000, 6, 10160, True),    # six metas, ~5 k rows per shared global time: LDS ranking, group drops
    (40_000, 12, 10160, False),  # 12 x 1060 candidates > 8192: ranking in global scratch
    (8_000, 3, 1024, True),      # capacity 106: many pivot windows fit, more-rows-on-the-other-side path
])
def test_claim_largest_matches_oracle(n, n_metas, bits, ties):
    rows, conn = build(n + n_metas, n, n_metas, 50_000, ties)
    metas = [MetaMessage("m%d" % i, i, SyncDistribution("ASC", 128)) for i in range(1, n_metas + 1)]
    om = [dict(name="m%d" % i, id=i, direction="ASC", priority=128, pruning=None) for i in range(1, n_metas + 1)]
    store = SyncStore.from_rows(rows)
    gt_now = 50_000
    calls = 0
    for trial in range(24):
        rec = Recorder(1000 * n + trial)
        com = SyncCommunity(store, metas, global_time=gt_now, signature_length=1500 - 60 - 8 - 51 - 21 - 30 - bits // 8,
                            rng=rec, random_source=rec)
        assert com.dispersy_sync_bloom_filter_bits == bits
        nrsync = [0, 10 ** 9, store.count_live(range(1, n_metas + 1))][trial % 3]
        com._nrsyncpackets = nrsync
        acceptable = com.acceptable_global_time
        try:
            got = com._dispersy_claim_sync_bloom_filter_largest(None)
        except IndexError:
            got = IndexError
        replay = Replay(rec.log)
        try:
            want, nr_after = sync_ref.claim_largest(conn, om, bits, 0.01, gt_now, acceptable, nrsync, replay,
                                                    OracleBloom)
        except IndexError:
            want = IndexError
        if want is IndexError or got is IndexError:
            assert got is want
            continue
        lo, hi, modulo, offset, bf = got
        assert (lo, hi, modulo, offset) == want[:4], trial
        assert bf.bytes == want[4].to_bytes() and bf.prefix == want[4].prefix
        assert com._nrsyncpackets == nr_after
        calls += 1
    assert calls >= 12

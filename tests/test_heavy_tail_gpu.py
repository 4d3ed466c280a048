"""BASELINE config 5 through the drop-in responder: heavy-tailed packet sizes (discretised Pareto(1.2) clipped to
[60, 65476] B, the UDP cap of endpoint.py:263) and skewed global times (Zipf(1.1) over 1..10^6), answered by
SyncCommunity.respond (dsy_sync_respond -> k_pair_test's multi-window path) and checked against the sqlite3 +
hashlib oracle (oracle/sync_ref.respond_lists = community.py:2746-2811 + the byte-limited loop :2555-2567).

The claims are shaped like bench.py's heavy_tail leg: largest-style (modulo 1, a global-time range holding about one
filter capacity of rows), modulo-style (modulo = ceil(N / capacity), every global time, random offset) and a few
claims over the whole store.  Their filters are MD5 (m=10160, f=0.01 -- the MTU claim) or SHA-1 (m=4096, f=0.001 --
the test-harness filter of node.py:617), built from the claim's rows with 1 % withheld.  Capped windows and a 1 MiB
budget make claims walk many windows of packets up to 64 KB (about a millisecond of serial digest per lane)."""
import math
import sqlite3

import numpy as np
import pytest

from dispersy_amd import BloomFilter
from dispersy_amd.community import ClaimRequest, SyncCommunity
from dispersy_amd.distribution import MetaMessage, SyncDistribution
from dispersy_amd.store import SyncStore
from golden_util import SYNC_SCHEMA
from oracle import sync_ref
from oracle.bloom_ref import OracleBloom

pytestmark = pytest.mark.gpu

N_ROWS = 80_000
GT_MAX = 1_000_000
METAS = [("ht", 1, "ASC", 128, None), ("hd", 2, "DESC", 100, None)]


def pareto_lengths(rng, n):
    u = rng.random(n)
    return np.minimum(np.floor(60.0 * u ** (-1.0 / 1.2)), 65476).astype(np.int64)


def zipf_gts(rng, n):
    w = np.arange(1, GT_MAX + 1, dtype=np.float64) ** -1.1
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    return np.minimum(np.searchsorted(cdf, rng.random(n)) + 1, GT_MAX)


@pytest.fixture(scope="module")
def world():
    rng = np.random.Generator(np.random.PCG64(5))
    lengths = pareto_lengths(rng, N_ROWS)
    lengths[:4] = 65476  # a few packets at the cap, whatever the draw
    gts = zipf_gts(rng, N_ROWS)
    meta = np.where(rng.random(N_ROWS) < 0.8, 1, 2)
    rows = []
    for i in range(N_ROWS):
        packet = i.to_bytes(4, "big") + rng.bytes(int(lengths[i]) - 4)
        rows.append((i + 1, int(gts[i]), int(meta[i]), 0, packet))
    conn = sqlite3.connect(":memory:")
    conn.executescript(SYNC_SCHEMA)
    conn.executemany("INSERT INTO sync(id, community, member, global_time, meta_message, undone, packet, sequence) "
                     "VALUES (?, 1, ?, ?, ?, ?, ?, 0)", [(r[0], r[0], r[1], r[2], r[3], r[4]) for r in rows])
    store = SyncStore.from_rows(rows)
    metas = [MetaMessage(n, i, SyncDistribution(d, p, None)) for n, i, d, p, _ in METAS]
    com = SyncCommunity(store, metas, global_time=GT_MAX + 10)
    return rows, conn, store, com


def make_claims(store, rng, n_claims):
    """(ClaimRequest, OracleBloom) pairs shaped like bench.py heavy_tail."""
    gt = store.global_time
    order = np.argsort(gt, kind="stable")
    sgt = gt[order]
    reqs, oracle = [], []
    shapes = [(10160, 0.01), (4096, 0.001)]
    for q in range(n_claims):
        m, f = shapes[q % 2]
        cap = BloomFilter(m, f).get_capacity(f)
        kind = q % 6
        if kind in (0, 1, 2):  # largest-style: ~capacity rows' worth of global times
            a = int(rng.integers(0, len(sgt)))
            lo, hi = int(sgt[a]), int(sgt[min(a + cap - 1, len(sgt) - 1)])
            modulo, offset = 1, 0
        elif kind in (3, 4):  # modulo-style over every global time
            lo, hi = 1, GT_MAX
            modulo = int(math.ceil(store.n / float(cap)))
            offset = int(rng.integers(0, modulo))
            if q % 12 == 3:
                offset = modulo - 1  # the residue class of global time 1, which ~9 % of the rows share
        else:  # the whole store
            lo, hi, modulo, offset = 1, GT_MAX, 1, 0
        sel = np.flatnonzero((gt >= lo) & (gt <= hi) & ((gt + np.uint64(offset)) % np.uint64(modulo) == 0))
        known = sel[rng.random(len(sel)) >= 0.01]
        prefix = bytes([int(rng.integers(0, 256))])
        bf = BloomFilter(m, f, prefix)
        bf.add_store_rows(store, known)
        reqs.append(ClaimRequest(lo, hi, modulo, offset, bf))
        oracle.append(OracleBloom.from_bytes(bf.bytes, bf.functions, prefix))
    return reqs, oracle


def oracle_metas():
    return [dict(name=n, id=i, direction=d, priority=p, pruning=pr) for n, i, d, p, pr in METAS]


def test_heavy_tail_lengths_cover_the_udp_range(world):
    rows, _, store, _ = world
    lengths = np.diff(store.offsets.astype(np.int64))
    assert lengths.min() == 60 and lengths.max() == 65476
    assert (lengths > 16_384).sum() >= 20  # enough multi-hundred-block keys to make lanes uneven
    assert (store.global_time == 1).mean() > 0.05  # the Zipf head: one global time shared by thousands of rows


def test_heavy_tail_filters_match_oracle_build(world):
    """A few claim filters rebuilt by the oracle (hashlib add_keys over the same rows) are byte-identical."""
    rows, _, store, _ = world
    rng = np.random.Generator(np.random.PCG64(17))
    for m, f in ((10160, 0.01), (4096, 0.001)):
        pick = rng.choice(len(rows), size=3000, replace=False)
        prefix = bytes([int(rng.integers(0, 256))])
        bf, ob = BloomFilter(m, f, prefix), OracleBloom.from_m_f(m, f, prefix)
        bf.add_store_rows(store, pick)
        ob.add_keys(store.packet(int(r)) for r in pick)
        assert bf.bytes == ob.to_bytes()


@pytest.mark.parametrize("window", [0, 1024, 4096])
def test_heavy_tail_respond_vs_oracle(world, window):
    rows, conn, store, com = world
    rng = np.random.Generator(np.random.PCG64(55))
    if "claims" not in _CACHE:
        _CACHE["claims"] = make_claims(store, rng, 96)
    reqs, oracle = _CACHE["claims"]
    store.ctx.set_window(window)
    try:
        results = [(limit, com.respond(reqs, include_inactive=False, byte_limit=limit))
                   for limit in (5120, 1 << 20, 1 << 40)]
    finally:
        store.ctx.set_window(0)
    for limit, got in results:
        for i, (q, ob, g) in enumerate(zip(reqs, oracle, got)):
            key = (limit, i)
            if key not in _CACHE:
                _CACHE[key] = sync_ref.respond_lists(conn, oracle_metas(), (q.time_low, q.time_high, q.offset,
                                                                            q.modulo), ob, com.global_time, limit)
            assert store.rowid[g].tolist() == _CACHE[key], (i, q.time_low, q.time_high, q.modulo, q.offset, limit)


_CACHE = {}

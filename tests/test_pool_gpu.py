"""The responder with pooled families (DSY_POOL, off by default; DESIGN.md "Pooled families"): k_fill adds each
claim's block-count histogram into its family's, k_pool_scatter orders every active claim's window pairs into one
longest-first pool, and k_pair_test<POOL> reads the claim (filter, prefix, m, k) per lane.  A context created with
DSY_POOL=7 pools the MD5, SHA-1 and SHA-256 families; its answers must equal the sqlite + hashlib oracle's
(oracle/sync_ref.respond_lists = community.py:2746-2811 + :2555-2567) for mixed families, prefixes of 0-5 bytes,
capped windows (the pool is rebuilt every window), a never-pooled SHA-512 family beside the pooled ones, the
resident-grid deal (DSY_POOL_DEAL), and both placements: the scatter's atomics (the default) and the per-(claim, bin)
scan (k_pool_scan, DSY_POOL_SCAN=1).  16384-pair windows give the modulo-1 claims split windows (k_fill_sort's order,
no per-claim rows), for which the scan falls back to the atomics."""
import numpy as np
import pytest

from dispersy_amd import BloomFilter, _native
from dispersy_amd.community import ClaimRequest, SyncCommunity
from dispersy_amd.distribution import MetaMessage, SyncDistribution
from dispersy_amd.store import SyncStore
from oracle import sync_ref
from oracle.bloom_ref import OracleBloom
from test_respond_scale_gpu import METAS, build

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[("0", "0"), ("1", "0"), ("0", "1")], ids=["stride", "deal", "scan"])
def pooled_ctx(request, monkeypatch):
    monkeypatch.setenv("DSY_POOL", "7")
    monkeypatch.setenv("DSY_POOL_DEAL", request.param[0])
    monkeypatch.setenv("DSY_POOL_SCAN", request.param[1])
    ctx = _native.Context(0)  # the knobs are read when a ctx is created
    yield ctx
    ctx.close()


_WORLD = {}  # (skew, one_byte) -> the rows, the sqlite oracle and the claims: the same for every mode and window


def _world(skew, one_byte):
    """The store's rows and its sqlite copy, 72 claims (filters built on the device and by the oracle) and the
    oracle's answers -- none depends on the pooling mode or the window, so every (mode, window) case of one
    (skew, one_byte) shares them (the Python oracle's filter builds and sqlite walks are most of the test's time)."""
    key = (skew, one_byte)
    if key in _WORLD:
        return _WORLD[key]
    seed = 3 if skew is False else 4
    rows, conn = build(seed, 30_000, 120_000 if skew is False else 5_000, skew)
    gt_now = 120_100 if skew is False else 30_100
    chosen = [m for m in METAS if m[0] in ("a", "d")]
    served_oracle = [dict(name=n, id=i, direction=d, priority=p, pruning=None) for n, i, d, p, _ in chosen]
    rng = np.random.Generator(np.random.PCG64(91 + seed))
    packets = {r[0]: r[4] for r in rows}
    # SHA-1 / MD5 / SHA-256 (pooled) and SHA-512 (never pooled) claims in one call
    shapes = [(4096, 0.001), (10160, 0.01), (1 << 15, 0.01), (1 << 16, 0.0001)]
    reqs, want = [], {}
    for q in range(72):
        modulo = int(rng.choice([1, 1, 7, 331]))
        offset = int(rng.integers(0, modulo))
        lo = int(rng.integers(1, gt_now // 2))
        hi = int(rng.integers(lo, gt_now + 10))
        m, f = shapes[q % len(shapes)]
        prefix = bytes(rng.integers(0, 256, size=1 if one_byte else int(q % 6), dtype=np.uint8))
        bf, ob = BloomFilter(m, f, prefix), OracleBloom.from_m_f(m, f, prefix)
        known = [packets[r[0]] for r in rows if rng.random() < 0.9]
        bf.add_keys(known)
        ob.add_keys(known)
        reqs.append(ClaimRequest(lo, hi, modulo, offset, bf))
        for limit in (5120, 1 << 40):
            want[q, limit] = sync_ref.respond_lists(conn, served_oracle, (lo, hi, offset, modulo), ob, gt_now, limit,
                                                    False)
    assert {bf.hash_name for bf in (r.bloom_filter for r in reqs)} == {"md5", "sha1", "sha256", "sha512"}
    conn.close()
    _WORLD[key] = (rows, chosen, gt_now, reqs, want)
    return _WORLD[key]


@pytest.mark.parametrize("one_byte", [False, True], ids=["prefixes0-5", "prefix1"])
@pytest.mark.parametrize("window", [0, 256, 16384])
@pytest.mark.parametrize("skew", [False, "dense"])
def test_pooled_families_vs_oracle(pooled_ctx, skew, window, one_byte):
    """one_byte: every claim's prefix is 1 byte (every reference claim), so the pooled MD5 / SHA-1 families hash the
    line copy's padded messages (k_pair_test<..., POOL, PADDED>)."""
    rows, chosen, gt_now, reqs, want = _world(skew, one_byte)
    store = SyncStore.from_rows(rows, ctx=pooled_ctx)
    served = [MetaMessage(n, i, SyncDistribution(d, p, None)) for n, i, d, p, _ in chosen]
    com = SyncCommunity(store, served, global_time=gt_now)
    store.ctx.set_window(window)
    try:
        results = [(limit, com.respond(reqs, byte_limit=limit)) for limit in (5120, 1 << 40)]
    finally:
        store.ctx.set_window(0)
    for limit, got in results:
        for i, (q, g) in enumerate(zip(reqs, got)):
            assert store.rowid[g].tolist() == want[i, limit], (q.time_low, q.time_high, q.modulo, q.offset, limit)

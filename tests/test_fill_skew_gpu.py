"""Regression test for the late-wave race round 6 found in k_fill (Multi-GPU, "Whole-bench rehearsal"):
the window's start cursor was read by every wave when it reached fill_claim while thread 0 advanced it, so a wave
scheduled late selected nothing.  DSY_FILL_SKEW holds waves 1-3 of every one-workgroup fill back on purpose; claims
walked in capped windows end in a remainder window that such a fill selects (the arithmetic path of a largest-style
claim, no barrier before the cursor is written).  Every answer must equal the sqlite + hashlib oracle's
(oracle/sync_ref.respond_lists = community.py:2746-2811 + :2555-2567), and no bounds check may trip."""
import sqlite3

import numpy as np
import pytest

from dispersy_amd import BloomFilter, _native
from dispersy_amd.community import ClaimRequest, SyncCommunity
from dispersy_amd.distribution import MetaMessage, SyncDistribution
from dispersy_amd.store import SyncStore
from golden_util import SYNC_SCHEMA
from oracle import sync_ref
from oracle.bloom_ref import OracleBloom

pytestmark = pytest.mark.gpu

N = 40_000
GT_NOW = N + 100


@pytest.fixture
def skewed_ctx(monkeypatch):
    monkeypatch.setenv("DSY_FILL_SKEW", "64")  # ~0.25 ms: long past the remainder window's selection
    ctx = _native.Context(0)
    yield ctx
    ctx.close()
    monkeypatch.delenv("DSY_FILL_SKEW")
    _native.Context(0).close()  # a ctx created without the variable sets the process-wide skew back to 0


def test_late_waves_of_a_fill_vs_oracle(skewed_ctx):
    rng = np.random.Generator(np.random.PCG64(64))
    lengths = rng.integers(20, 700, size=N)
    rows = [(i + 1, i + 1, 1, 0, i.to_bytes(4, "big") + rng.bytes(int(lengths[i]) - 4)) for i in range(N)]
    conn = sqlite3.connect(":memory:")
    conn.executescript(SYNC_SCHEMA)
    conn.executemany("INSERT INTO sync(id, community, member, global_time, meta_message, undone, packet, sequence) "
                     "VALUES (?, 1, ?, ?, ?, ?, ?, 0)", [(r[0], r[0], r[1], r[2], r[3], r[4]) for r in rows])
    store = SyncStore.from_rows(rows, ctx=skewed_ctx)
    served = [MetaMessage("a", 1, SyncDistribution("ASC", 128, None))]
    served_oracle = [dict(name="a", id=1, direction="ASC", priority=128, pruning=None)]
    com = SyncCommunity(store, served, global_time=GT_NOW)
    packets = [r[4] for r in rows]
    reqs, blooms = [], []
    for q in range(12):
        lo = int(rng.integers(1, 4000))
        hi = int(rng.integers(N // 2, N + 1))  # 20 k - 40 k rows: capped windows of 8192, then a remainder
        prefix = bytes([q + 1])
        bf, ob = BloomFilter(10160, 0.01, prefix), OracleBloom.from_m_f(10160, 0.01, prefix)
        known = [packets[i] for i in range(lo - 1, hi) if rng.random() < 0.97]
        bf.add_keys(known)
        ob.add_keys(known)
        reqs.append(ClaimRequest(lo, hi, 1, 0, bf))
        blooms.append(ob)
    store.ctx.set_window(8192)
    try:
        got = com.respond(reqs, byte_limit=1 << 40)
    finally:
        store.ctx.set_window(0)
    for q, ob, g in zip(reqs, blooms, got):
        want = sync_ref.respond_lists(conn, served_oracle, (q.time_low, q.time_high, q.offset, q.modulo), ob, GT_NOW,
                                      1 << 40, False)
        assert store.rowid[g].tolist() == want, (q.time_low, q.time_high)

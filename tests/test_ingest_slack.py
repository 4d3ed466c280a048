"""The responder index's slack (dsy_store_append / store_flush): appended rows join the live index at the next read,
merged in place into the slack each meta's region keeps when they fit (their meta's tail from the first new entry on
is merged back), or by one whole-index merge that lays the regions out again.  Every read is checked against the
reference's SQL over one sqlite table that received the same INSERTs, DELETEs and UPDATEs (oracle/sync_ref): an empty
claim filter with no budget returns every row of the range, so the answer is the whole index order of the range.

The sequence mixes what moves the slack: appends at the top of a meta's global times (in place, no tail), appends of
older global times (in place, with tails), several appends before one read, global times from the whole history
(tails longer than a whole merge), a meta new to the index and a slack that
runs out (whole merges), DELETEs and undo (a dense index again), GlobalTimePruning's DELETE, and redo."""
import sqlite3

import numpy as np
import pytest

from dispersy_amd import BloomFilter, _native
from dispersy_amd.community import ClaimRequest, SyncCommunity
from dispersy_amd.distribution import GlobalTimePruning, MetaMessage, SyncDistribution
from dispersy_amd.store import SyncStore
from golden_util import SYNC_SCHEMA
from oracle import sync_ref
from oracle.bloom_ref import OracleBloom

pytestmark = pytest.mark.gpu

METAS = [("a", 1, "ASC", 128, None), ("d", 2, "DESC", 200, None), ("p", 3, "ASC", 150, (400, 800)),
         ("n", 4, "DESC", 100, None), ("q", 6, "ASC", 60, None)]


def metas():
    return [MetaMessage(n, i, SyncDistribution(d, p, GlobalTimePruning(*pr) if pr else None)) for n, i, d, p, pr in METAS]


def oracle_metas():
    return [dict(name=n, id=i, direction=d, priority=p, pruning=pr) for n, i, d, p, pr in METAS]


def stats(store):
    out = np.zeros(6, dtype=np.uint64)
    _native.check(store.ctx.lib.dsy_store_index_stats(store.handle, out.ctypes.data))
    return dict(zip(("live", "phys", "fast", "full", "bytes", "pending"), out.tolist()))


def test_slack_merges_match_the_reference():
    rng = np.random.Generator(np.random.PCG64(2024))
    next_id = [1]

    def make(n, metas_p, gt_lo, gt_hi):
        out = []
        for _ in range(n):
            i = next_id[0]
            next_id[0] += 1
            meta = int(rng.choice([m for m, _ in metas_p], p=[p for _, p in metas_p]))
            packet = i.to_bytes(4, "big") + rng.bytes(int(rng.integers(20, 300)))
            out.append((i, int(rng.integers(gt_lo, gt_hi)), meta, 0, packet))
        return out

    base = make(20_000, [(1, 0.6), (2, 0.3), (3, 0.1)], 1, 4_000)
    conn = sqlite3.connect(":memory:")
    conn.executescript(SYNC_SCHEMA)

    def insert(rows):
        conn.executemany("INSERT INTO sync(id, community, member, global_time, meta_message, undone, packet, sequence) "
                         "VALUES (?, 1, ?, ?, ?, ?, ?, 0)", [(r[0], r[0], r[1], r[2], r[3], r[4]) for r in rows])

    insert(base)
    store = SyncStore.from_rows(base)
    store.handle  # noqa: B018 -- on the device before the appends
    gt_now = [4_100]
    com = SyncCommunity(store, metas(), global_time=gt_now[0])

    def append(rows):
        got = store.append([r[4] for r in rows], [r[1] for r in rows], [r[2] for r in rows], [r[0] for r in rows])
        insert(rows)
        return got

    def set_time(t):
        gt_now[0] = t
        com.update_global_time(t)  # meta 3 (GlobalTimePruning, prune at 800): its rows up to t - 800 go
        conn.execute("DELETE FROM sync WHERE meta_message = 3 AND global_time <= ?", (t - 800,))

    def check(tag):
        empty_bf, empty_ob = BloomFilter(10160, 0.01, b"\x05"), OracleBloom.from_m_f(10160, 0.01, b"\x05")
        hi = gt_now[0] + 5
        claims = [(1, hi, 0, 1), (int(rng.integers(1, 3_000)), hi, 0, 1), (1, hi, 1, 3)]
        reqs = [ClaimRequest(lo, h, mod, off, empty_bf) for lo, h, off, mod in claims]
        got = com.respond(reqs, include_inactive=True, byte_limit=1 << 40)
        for (lo, h, off, mod), g in zip(claims, got):
            want = sync_ref.respond_lists(conn, oracle_metas(), (lo, h, off, mod), empty_ob, gt_now[0], 1 << 40, True)
            assert store.rowid[g].tolist() == want, (tag, lo, h, off, mod)
        st = stats(store)
        assert st["pending"] == 0 and st["live"] == sum(store.live_count(m) for m in (1, 2, 3, 4, 6)), (tag, st)
        return st

    s0 = check("upload")
    # 1. new global times at the top: the first append has no slack (a fresh upload is dense) -> one whole merge that
    # lays out the regions; the next ones fit the slack and need no tail
    top = 4_000
    for k in range(3):
        append(make(700, [(1, 0.6), (2, 0.4)], top, top + 60))
        top += 60
        set_time(top + 100)
        st = check("top %d" % k)
    assert st["full"] == s0["full"] + 1 and st["fast"] == s0["fast"] + 2, st
    # 2. older global times (tails merged in place) and two appends before one read; then global times from the whole
    # history: long tails, merged in place or -- when they would move more than the whole index (64 B per tail entry
    # against 32 B per entry of the index arrays) -- by one whole merge
    append(make(500, [(1, 0.5), (2, 0.5)], top - 700, top))
    append(make(300, [(2, 1.0)], top - 400, top))
    st2 = check("older")
    assert st2["fast"] == st["fast"] + 1 and st2["full"] == st["full"], st2
    append(make(500, [(1, 0.5), (2, 0.5)], 1, top))
    st2b = check("old")
    assert st2b["full"] + st2b["fast"] == st2["full"] + st2["fast"] + 1, st2b
    st2 = st2b
    # 3. a meta new to the index (whole merge), then in place again
    append(make(400, [(4, 0.5), (1, 0.5)], 100, top))
    st3 = check("new meta")
    assert st3["full"] == st2["full"] + 1, st3
    append(make(200, [(4, 1.0)], top, top + 10))
    st4 = check("new meta, in place")
    assert st4["fast"] == st3["fast"] + 1, st4
    # 4. DELETE and undo compact the index (no slack left): the next append merges the whole index again
    victims = rng.choice(store.n, 900, replace=False)
    store.delete_rows(victims)
    ids = store.rowid[np.unique(victims)].tolist()
    conn.executemany("DELETE FROM sync WHERE id = ?", [(i,) for i in ids])
    check("delete")
    live = np.flatnonzero((store.undone == 0) & ~store.deleted)
    undo = rng.choice(live, 400, replace=False)
    store.set_undone(undo, 1)
    conn.executemany("UPDATE sync SET undone = 1 WHERE id = ?", [(int(store.rowid[r]),) for r in undo])
    check("undo")
    append(make(600, [(1, 0.4), (2, 0.3), (3, 0.3)], top - 200, top + 40))
    st5 = check("after compaction")
    assert st5["full"] == st4["full"] + 1, st5
    # 5. redo half of the undone rows (the host-ordered whole merge), then GlobalTimePruning's DELETE of meta 3
    redo = undo[: len(undo) // 2]
    store.set_undone(redo, 0)
    conn.executemany("UPDATE sync SET undone = 0 WHERE id = ?", [(int(store.rowid[r]),) for r in redo])
    check("redo")
    append(make(300, [(3, 1.0)], top, top + 40))
    top += 40
    set_time(top + 500)
    check("prune")
    # 6. a slack that runs out: appends to one meta until its region is full -> a whole merge, then in place again
    before = stats(store)
    for k in range(8):
        append(make(6_000, [(2, 1.0)], top, top + 20))
        top += 20
        set_time(top + 10)
        check("fill %d" % k)
    after = stats(store)
    assert after["full"] > before["full"] and after["fast"] > before["fast"], (before, after)
    assert after["phys"] >= after["live"]


def test_index_stats_arguments():
    store = SyncStore.from_rows([(1, 5, 1, 0, b"abc")])
    assert store.ctx.lib.dsy_store_index_stats(store.handle, None) == _native.DSY_EINVAL
    out = np.zeros(6, dtype=np.uint64)
    _native.check(store.ctx.lib.dsy_store_index_stats(store.handle, out.ctypes.data))
    assert out.tolist()[:2] == [1, 1] and out[5] == 0


def test_gather_and_joined_appends_agree():
    """SyncStore.append hands bytes packets to dsy_store_append_gather (their own buffers, no joined copy) and other
    bytes-like packets to dsy_store_append (one joined blob): both reach the line copy the responder and the claim side
    hash from.  Checked through a claim filter built on the device from the appended rows against the oracle, the
    responder's answer for an empty filter against the reference's SQL, and the host copies of the packets."""
    from dispersy_amd.store import _BYTES_DATA
    assert _BYTES_DATA is not None  # CPython 3 on this image: the gather path is the one that runs
    rng = np.random.Generator(np.random.PCG64(77))

    def rows_of(first, n, gt0):
        return [(i, gt0 + k, 1, 0, i.to_bytes(4, "big") + rng.bytes(int(rng.integers(0, 600))))
                for k, i in enumerate(range(first, first + n))]

    base, a, b = rows_of(1, 3000, 1), rows_of(3001, 700, 3001), rows_of(3701, 500, 3701)
    a.append((4201, 4000, 1, 0, b""))  # an empty packet in the gather list
    b = [(r[0] + 501, r[1] + 1, r[2], r[3], r[4]) for r in b]
    store = SyncStore.from_rows(base)
    store.handle  # noqa: B018
    store.append([r[4] for r in a], [r[1] for r in a], [r[2] for r in a], [r[0] for r in a])
    store.append([bytearray(r[4]) for r in b], [r[1] for r in b], [r[2] for r in b], [r[0] for r in b])
    allr = base + a + b
    assert [store.packet(i) for i in range(store.n)] == [r[4] for r in allr]
    new = np.arange(len(base), store.n)
    bf, ob = BloomFilter(1 << 20, 0.01, b"\x09"), OracleBloom.from_m_f(1 << 20, 0.01, b"\x09")
    bf.add_store_rows(store, new)
    ob.add_keys([r[4] for r in a + b])
    assert bf.bytes == ob.to_bytes()
    conn = sqlite3.connect(":memory:")
    conn.executescript(SYNC_SCHEMA)
    conn.executemany("INSERT INTO sync(id, community, member, global_time, meta_message, undone, packet, sequence) "
                     "VALUES (?, 1, ?, ?, ?, ?, ?, 0)", [(r[0], r[0], r[1], r[2], r[3], r[4]) for r in allr])
    com = SyncCommunity(store, [MetaMessage("a", 1, SyncDistribution("ASC", 128))], global_time=5_000)
    empty_bf, empty_ob = BloomFilter(10160, 0.01, b"\x05"), OracleBloom.from_m_f(10160, 0.01, b"\x05")
    (got,) = com.respond([ClaimRequest(2_500, 5_000, 1, 0, empty_bf)], byte_limit=1 << 40)
    want = sync_ref.respond_lists(conn, [dict(name="a", id=1, direction="ASC", priority=128, pruning=None)],
                                  (2_500, 5_000, 0, 1), empty_ob, 5_000, 1 << 40, False)
    assert store.rowid[got].tolist() == want and len(want) > 1000

"""DELETEs of arbitrary store rows (SyncStore.delete_rows -> dsy_store_delete): the sequence-number conflict DELETE
(dispersy.py:1006-1007) and LastSyncDistribution's history pruning (:1581-1591) remove rows from the responder's live
index (a stable compaction on the device) and from the (member, global_time) duplicate table (tombstones), as the
same DELETEs do to the reference's sqlite `sync` table.  The oracle is that table with the DELETEs run verbatim
(oracle/sync_ref.respond_lists for the responder, is_duplicate_sync_message for the lookups)."""
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

METAS = [("a", 1, "ASC", 128, None), ("d", 2, "DESC", 200, None), ("p", 3, "ASC", 150, (400, 800))]
GT_NOW = 3_100


def make_rows(seed, n):
    """(rowid, gt, meta, undone, packet, member): unique (member, gt), ~3 % undone."""
    rng = np.random.Generator(np.random.PCG64(seed))
    rows, seen = [], set()
    while len(rows) < n:
        member, gt = int(rng.integers(1, 40)), int(rng.integers(1, 3_000))
        if (member, gt) in seen:
            continue
        seen.add((member, gt))
        i = len(rows)
        meta = int(rng.choice([1, 2, 3], p=[0.5, 0.3, 0.2]))
        packet = i.to_bytes(4, "big") + rng.bytes(int(rng.integers(20, 300)) - 4)
        rows.append((i + 1, gt, meta, int(rng.random() < 0.03) * (i + 1), packet, member))
    return rows


def sqlite_of(rows):
    conn = sqlite3.connect(":memory:")
    conn.executescript(SYNC_SCHEMA)
    conn.executemany("INSERT INTO sync(id, community, member, global_time, meta_message, undone, packet, sequence) "
                     "VALUES (?, 1, ?, ?, ?, ?, ?, 0)", [(r[0], r[5], r[1], r[2], r[3], r[4]) for r in rows])
    return conn


def metas():
    return [MetaMessage(n, i, SyncDistribution(d, p, GlobalTimePruning(*pr) if pr else None)) for n, i, d, p, pr in METAS]


def oracle_metas():
    return [dict(name=n, id=i, direction=d, priority=p, pruning=pr) for n, i, d, p, pr in METAS]


def live_ids(conn, m):
    return [i for (i,) in conn.execute("SELECT id FROM sync WHERE meta_message = ? AND undone = 0 ORDER BY global_time, id",
                                       (m,))]


def test_delete_rows_host_index():
    """CPU: the host columns after DELETEs (repeated rows, undone rows, rows deleted twice) match the table."""
    rows = make_rows(3, 3000)
    store = SyncStore.from_rows(rows, ctx=object())
    conn = sqlite_of(rows)
    rng = np.random.Generator(np.random.PCG64(4))
    for _ in range(3):
        pick = rng.integers(0, store.n, size=200)
        n_new = len(set(int(x) for x in pick) - set(np.flatnonzero(store.deleted).tolist()))
        assert store.delete_rows(np.concatenate([pick, pick[:20]])) == n_new
        conn.executemany("DELETE FROM sync WHERE id = ?", [(int(store.rowid[r]),) for r in pick])
    for m in (1, 2, 3):
        assert store.rowid[store.live_rows(m)].tolist() == live_ids(conn, m)
        assert store.count_live([m, m]) == len(live_ids(conn, m))
    gone = int(store.rowid[np.flatnonzero(store.deleted)[0]])
    with pytest.raises(KeyError):
        store.row_of_id(gone)
    kept = int(store.rowid[np.flatnonzero(~store.deleted)[0]])
    assert store.rowid[store.row_of_id(kept)] == kept


@pytest.mark.gpu
@pytest.mark.parametrize("lazy", [False, True])
def test_delete_rows_responder_and_dup_table(lazy):
    """DELETEs interleaved with appends and a GlobalTimePruning prune; the responder serves what the table holds
    after the same statements, and the duplicate check no longer finds a deleted (member, global_time) -- a new row
    with that key is found instead (the prune used to leave the keys behind)."""
    rows = make_rows(11, 16_000)
    n0 = 10_000
    store = SyncStore.from_rows(rows[:n0])
    conn = sqlite_of(rows[:n0])
    if not lazy:
        store.handle  # noqa: B018
    com = SyncCommunity(store, metas(), global_time=GT_NOW)
    rng = np.random.Generator(np.random.PCG64(12))
    deleted_keys = []

    def delete(k):
        pick = rng.integers(0, store.n, size=k)
        for r in pick.tolist():
            if not store.deleted[r]:
                deleted_keys.append((int(store.member[r]), int(store.global_time[r]), int(store.rowid[r])))
        store.delete_rows(pick)
        conn.executemany("DELETE FROM sync WHERE id = ?", [(int(store.rowid[r]),) for r in pick])

    delete(700)
    part = rows[n0:13_000]
    store.append([r[4] for r in part], [r[1] for r in part], [r[2] for r in part], [r[0] for r in part],
                 member=[r[5] for r in part])
    conn.executemany("INSERT INTO sync(id, community, member, global_time, meta_message, undone, packet, sequence) "
                     "VALUES (?, 1, ?, ?, ?, 0, ?, 0)", [(r[0], r[5], r[1], r[2], r[4]) for r in part])
    delete(900)
    com.update_global_time(GT_NOW + 1_200)  # meta 3 prunes rows up to global time 3500 - 800
    conn.execute("DELETE FROM sync WHERE meta_message = 3 AND global_time <= ?", (GT_NOW + 1_200 - 800,))
    delete(300)
    gt_now = GT_NOW + 1_200
    for m in (1, 2, 3):
        assert store.rowid[store.live_rows(m)].tolist() == live_ids(conn, m), m
    reqs, blooms = [], []
    packets = {r[0]: r[4] for r in rows}
    for q in range(32):
        lo, prefix = int(rng.integers(1, 3_000)), bytes([q])
        modulo = int(rng.choice([1, 1, 7]))
        bf, ob = BloomFilter(10160, 0.01, prefix), OracleBloom.from_m_f(10160, 0.01, prefix)
        known = [packets[r[0]] for r in rows[:13_000] if rng.random() < 0.9]
        bf.add_keys(known)
        ob.add_keys(known)
        reqs.append(ClaimRequest(lo, gt_now, modulo, int(rng.integers(0, modulo)), bf))
        blooms.append(ob)
    for include_inactive, limit in ((True, 1 << 40), (False, 5120)):
        got = com.respond(reqs, include_inactive=include_inactive, byte_limit=limit)
        for q, ob, g in zip(reqs, blooms, got):
            want = sync_ref.respond_lists(conn, oracle_metas(), (q.time_low, q.time_high, q.offset, q.modulo), ob,
                                          gt_now, limit, include_inactive)
            assert store.rowid[g].tolist() == want
    # duplicate lookups: deleted keys are gone (sqlite finds no row), stored keys are found
    pruned = [(int(store.member[r]), int(store.global_time[r])) for r in np.flatnonzero(store.deleted)[:50]]
    keys = [k[:2] for k in deleted_keys[:200]] + pruned
    alive = np.flatnonzero(~store.deleted)[:100]
    keys += [(int(store.member[r]), int(store.global_time[r])) for r in alive]
    pk = [b"probe-%d" % i for i in range(len(keys))]
    verdict, row = store.dup_check([k[0] for k in keys], [k[1] for k in keys], pk, [60] * len(keys))
    for (mem, gt), v in zip(keys, verdict.tolist()):
        found = conn.execute("SELECT id FROM sync WHERE member = ? AND global_time = ?", (mem, gt)).fetchone()
        assert (v != _native.DSY_DUP_NEW) == (found is not None), (mem, gt, v)
    # a deleted key INSERTed again: the lookup finds the new row
    mem, gt, _ = deleted_keys[0]
    [new_row] = store.append([b"again"], [gt], [1], member=[mem]).tolist()
    verdict, row = store.dup_check([mem], [gt], [b"again"], [60])
    assert verdict.tolist() == [_native.DSY_DUP_EXACT] and row.tolist() == [new_row]


@pytest.mark.gpu
def test_claim_modulo_counts_repeated_meta_ids_once():
    """`meta_message IN (1, 1, 2)` selects each row once (repeated ids were scanned twice)."""
    rows = make_rows(21, 6000)
    store = SyncStore.from_rows(rows)
    a, b = BloomFilter(10160, 0.01, b"\x05"), BloomFilter(10160, 0.01, b"\x05")
    n1 = a.add_store_modulo(store, [1, 2], 3, 7)
    n2 = b.add_store_modulo(store, [1, 1, 2, 2, 2], 3, 7)
    assert n1 == n2 > 0 and a.bytes == b.bytes

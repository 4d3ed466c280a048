"""Requester-side ingest: packets received after the store went to HBM are INSERTed
(`Dispersy._store`, dispersy.py:1475-1612) by SyncStore.append / dsy_store_append, and the responder serves them from
then on in the index order of the reference's `sync` table, (meta_message, global_time, rowid).

The oracle is the reference's own SQL over one sqlite table holding every row, inserted in rowid order
(oracle/sync_ref.respond_lists); the GPU store is built from the first rows and grows by appended batches -- with
global times equal to stored ones (ties go after the stored rows), metas below, between and above the stored ones,
and batches given out of global-time order."""
import sqlite3

import numpy as np
import pytest

from dispersy_amd import BloomFilter
from dispersy_amd.community import ClaimRequest, SyncCommunity
from dispersy_amd.distribution import GlobalTimePruning, MetaMessage, SyncDistribution
from dispersy_amd.store import SyncStore
from golden_util import SYNC_SCHEMA
from oracle import sync_ref
from oracle.bloom_ref import OracleBloom

METAS = [("z", 0, "DESC", 90, None), ("a", 1, "ASC", 128, None), ("d", 2, "DESC", 200, None),
         ("p", 3, "ASC", 150, (400, 800)), ("q", 5, "ASC", 60, None), ("r", 7, "ASC", 10, None)]  # r: not synced (priority <= 32)
GT_NOW = 3_100


def make_rows(seed, n, n0):
    """n rows with rowids 1..n; rows past n0 are the appended ones (undone = 0, as INSERTed) and are the only rows
    of metas 0 and 5 (new to the store, below and between the stored metas)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    rows = []
    for i in range(n):
        if i < n0:
            meta = int(rng.choice([1, 2, 3, 7], p=[0.5, 0.25, 0.15, 0.1]))
            undone = int(rng.random() < 0.03)
        else:
            meta = int(rng.choice([0, 1, 2, 3, 5, 7], p=[0.1, 0.4, 0.2, 0.1, 0.1, 0.1]))
            undone = 0
        gt = int(rng.integers(1, 3_000))  # ~7 rows per global time: ties between stored and appended rows
        packet = i.to_bytes(4, "big") + rng.bytes(int(rng.integers(20, 400)) - 4)
        rows.append((i + 1, gt, meta, undone, packet))
    return rows


def sqlite_of(rows):
    conn = sqlite3.connect(":memory:")
    conn.executescript(SYNC_SCHEMA)
    conn.executemany("INSERT INTO sync(id, community, member, global_time, meta_message, undone, packet, sequence) "
                     "VALUES (?, 1, ?, ?, ?, ?, ?, 0)", [(r[0], r[0], r[1], r[2], r[3], r[4]) for r in rows])
    return conn


def grow(store, rows, batches):
    """Append rows in rowid order, in the given number of batches (global times unsorted within a batch)."""
    for part in np.array_split(np.arange(len(rows)), batches):
        sel = [rows[i] for i in part]
        got = store.append([r[4] for r in sel], [r[1] for r in sel], [r[2] for r in sel], [r[0] for r in sel])
        assert store.rowid[got].tolist() == [r[0] for r in sel]


def test_append_host_index_matches_a_fresh_export():
    rows = make_rows(3, 3000, 1800)
    store = SyncStore.from_rows(rows[:1800], ctx=object())  # host only: no device handle is created
    grow(store, rows[1800:], 4)
    fresh = SyncStore.from_rows(rows, ctx=object())
    for m in (0, 1, 2, 3, 5, 7):
        assert store.rowid[store.live_rows(m)].tolist() == fresh.rowid[fresh.live_rows(m)].tolist(), m
    for i in range(store.n):
        assert store.packet(i) == rows[int(store.rowid[i]) - 1][4]
    with pytest.raises(ValueError):
        store.append([b"x"], [5], [1], [2])  # a rowid below the stored ones


def metas():
    return [MetaMessage(n, i, SyncDistribution(d, p, GlobalTimePruning(*pr) if pr else None)) for n, i, d, p, pr in METAS]


def oracle_metas():
    return [dict(name=n, id=i, direction=d, priority=p, pruning=pr) for n, i, d, p, pr in METAS]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["live", "lazy", "empty"])
def test_responder_serves_appended_rows_like_the_reference(mode):
    """live: the store is on the device before the appends (dsy_store_append merges the index in HBM, three
    batches); lazy: rows appended before the first device use (upload + one append); empty: a store that starts
    with no rows at all."""
    n, n0 = 24_000, {"live": 14_000, "lazy": 14_000, "empty": 0}[mode]
    rows = make_rows(17, n, n0)
    conn = sqlite_of(rows)
    store = SyncStore.from_rows(rows[:n0])
    if mode != "lazy":
        store.handle  # noqa: B018 -- upload now, so the appends below go through the device merge
    grow(store, rows[n0:], 3)
    com = SyncCommunity(store, metas(), global_time=GT_NOW)
    rng = np.random.Generator(np.random.PCG64(23))
    packets = {r[0]: r[4] for r in rows}
    reqs, blooms = [], []
    for q in range(48):
        modulo = int(rng.choice([1, 1, 3, 17]))
        offset = int(rng.integers(0, modulo))
        lo = int(rng.integers(1, GT_NOW // 2))
        hi = int(rng.integers(lo, GT_NOW + 10))
        prefix = bytes([int(rng.integers(0, 256))])
        bf, ob = BloomFilter(10160, 0.01, prefix), OracleBloom.from_m_f(10160, 0.01, prefix)
        known = [packets[r[0]] for r in rows if rng.random() < 0.9]
        bf.add_keys(known)
        ob.add_keys(known)
        reqs.append(ClaimRequest(lo, hi, modulo, offset, bf))
        blooms.append(ob)
    for include_inactive, limit in ((False, 5120), (True, 1 << 40)):
        got = com.respond(reqs, include_inactive=include_inactive, byte_limit=limit)
        for q, ob, g in zip(reqs, blooms, got):
            want = sync_ref.respond_lists(conn, oracle_metas(), (q.time_low, q.time_high, q.offset, q.modulo), ob,
                                          GT_NOW, limit, include_inactive)
            assert store.rowid[g].tolist() == want, (q, include_inactive, limit)


@pytest.mark.gpu
def test_claim_filter_over_appended_rows():
    """The claim side builds its filter from store rows on the device (dsy_bloom_add_rows): rows that arrived by
    append hash from the grown blob exactly as the reference hashes the packets it selected."""
    rows = make_rows(29, 6000, 4000)
    store = SyncStore.from_rows(rows[:4000])
    store.handle  # noqa: B018
    grow(store, rows[4000:], 2)
    pick = np.arange(store.n)[::3]
    for m, f, prefix in ((10160, 0.01, b"\x07"), (4096, 0.001, b"x"), (1 << 20, 0.01, b"\x01\x02")):
        bf, ob = BloomFilter(m, f, prefix), OracleBloom.from_m_f(m, f, prefix)
        bf.add_store_rows(store, pick)
        ob.add_keys([store.packet(int(i)) for i in pick])
        assert bf.bytes == ob.to_bytes()


@pytest.mark.gpu
def test_sync_round_trip_through_store_messages():
    """One requester/responder exchange on the Community surface: B claims, A answers, B stores the answer
    (store_messages = Dispersy._store + dispersy_store), so B's cached claim filter now holds the received packets
    (community.py:680-707) and A's answer to the reused claim skips them -- both checked against the oracle."""
    rows = make_rows(31, 8000, 8000)
    rows = [(r[0], r[1], 1, 0, r[4]) for r in rows]  # one synced meta, all live
    conn_a = sqlite_of(rows)
    meta = [MetaMessage("a", 1, SyncDistribution("ASC", 128))]
    rng = np.random.Generator(np.random.PCG64(37))
    have = [r for r in rows if rng.random() < 0.7]
    store_a, store_b = SyncStore.from_rows(rows), SyncStore.from_rows(have)
    draws = np.random.Generator(np.random.PCG64(41))

    class Rand(object):
        def random(self):
            return float(draws.random())

        def randint(self, a, b):
            return int(draws.integers(a, b + 1))

        def expovariate(self, lambd):
            return float(draws.exponential(1.0 / lambd))

    com_a = SyncCommunity(store_a, meta, global_time=GT_NOW)
    com_b = SyncCommunity(store_b, meta, global_time=GT_NOW, rng=Rand(), random_source=Rand())

    class RC(object):
        helper_candidate = None

    class Dist(object):
        def __init__(self, gt):
            self.priority, self.global_time = 128, gt

    class Msg(object):
        def __init__(self, gt, packet):
            self.distribution, self.packet, self.candidate, self.database_id = Dist(gt), packet, None, 1

    lo, hi, modulo, offset, bf = com_b.dispersy_claim_sync_bloom_filter(RC())
    claim_rows = [r for r in have if lo <= r[1] <= hi and (r[1] + offset) % modulo == 0]
    ob = OracleBloom.from_m_f(bf.size, 0.01, bf.prefix) if bf.size != 8 else None
    (got,) = com_a.respond([ClaimRequest(lo, hi, modulo, offset, bf)], byte_limit=5120)
    ob.add_keys([r[4] for r in claim_rows])
    want = sync_ref.respond_lists(conn_a, [dict(name="a", id=1, direction="ASC", priority=128, pruning=None)],
                                  (lo, hi, offset, modulo), ob, GT_NOW, 5120, False)
    assert store_a.rowid[got].tolist() == want and want
    sent = [rows[r - 1] for r in want]
    n_before = store_b.n
    new_rows = com_b.store_messages([Msg(r[1], r[4]) for r in sent])
    assert new_rows.tolist() == list(range(n_before, n_before + len(sent)))
    ob.add_keys([r[4] for r in sent if lo <= r[1] <= hi and (r[1] + offset) % modulo == 0])
    assert com_b._sync_cache.bloom_filter.bytes == ob.to_bytes()
    # B's store serves what it received, in index order
    fresh = SyncStore.from_rows(have + sent, ctx=object())
    assert store_b.rowid[store_b.live_rows(1)].tolist() != []
    assert sorted(store_b.packet(int(i)) for i in store_b.live_rows(1)) == sorted(fresh.packet(int(i)) for i in fresh.live_rows(1))
    # the reused claim: A no longer sends what B stored
    com_b._sync_cache.responses_received += 1
    again = com_b.dispersy_claim_sync_bloom_filter(RC())
    assert again[4] is bf
    (got2,) = com_a.respond([ClaimRequest(*again)], byte_limit=5120)
    want2 = sync_ref.respond_lists(conn_a, [dict(name="a", id=1, direction="ASC", priority=128, pruning=None)],
                                   (lo, hi, offset, modulo), ob, GT_NOW, 5120, False)
    assert store_a.rowid[got2].tolist() == want2
    assert not set(want2) & set(want)


@pytest.mark.gpu
@pytest.mark.parametrize("lazy", [False, True])
def test_global_time_pruning_deletes_from_the_responder(lazy):
    """update_global_time with GlobalTimePruning metas DELETEs their rows up to global_time - prune_threshold
    (community.py:1082-1096, run on sqlite verbatim as the oracle); the responder no longer serves them even with
    include_inactive=True, and appends after the DELETE still merge (dsy_store_prune + dsy_store_append)."""
    rows = make_rows(41, 12_000, 8_000)
    store = SyncStore.from_rows(rows[:8_000])
    if not lazy:
        store.handle  # noqa: B018
    com = SyncCommunity(store, metas(), global_time=GT_NOW)
    conn = sqlite_of(rows[:8_000])
    com.update_global_time(GT_NOW + 1_500)  # meta 3 (prune at 800): rows up to 3800 go
    for m in METAS:
        if m[4]:
            conn.execute("DELETE FROM sync WHERE meta_message = ? AND global_time <= ?", (m[1], GT_NOW + 1_500 - m[4][1]))
    grow(store, rows[8_000:], 2)
    conn.executemany("INSERT INTO sync(id, community, member, global_time, meta_message, undone, packet, sequence) "
                     "VALUES (?, 1, ?, ?, ?, ?, ?, 0)", [(r[0], r[0], r[1], r[2], r[3], r[4]) for r in rows[8_000:]])
    gt_now = GT_NOW + 1_500
    for m in (0, 1, 2, 3, 5, 7):
        want = [i for (i,) in conn.execute("SELECT id FROM sync WHERE meta_message = ? AND undone = 0 "
                                           "ORDER BY global_time, id", (m,))]
        assert store.rowid[store.live_rows(m)].tolist() == want, m
    rng = np.random.Generator(np.random.PCG64(43))
    reqs, blooms = [], []
    for q in range(24):
        lo, prefix = int(rng.integers(1, 3_000)), bytes([q])
        bf, ob = BloomFilter(10160, 0.01, prefix), OracleBloom.from_m_f(10160, 0.01, prefix)
        known = [r[4] for r in rows if rng.random() < 0.95]
        bf.add_keys(known)
        ob.add_keys(known)
        reqs.append(ClaimRequest(lo, gt_now, 1, 0, bf))
        blooms.append(ob)
    got = com.respond(reqs, include_inactive=True, byte_limit=1 << 40)
    for q, ob, g in zip(reqs, blooms, got):
        want = sync_ref.respond_lists(conn, oracle_metas(), (q.time_low, q.time_high, q.offset, q.modulo), ob,
                                      gt_now, 1 << 40, True)
        assert store.rowid[g].tolist() == want


def test_prune_host_index():
    """SyncStore.prune on the host columns: the meta's rows up to the threshold -- live and undone, as the SQL DELETE
    (community.py:1094-1096) -- leave, others stay (CPU)."""
    rows = make_rows(5, 2000, 2000)
    store = SyncStore.from_rows(rows, ctx=object())
    before = {m: store.rowid[store.live_rows(m)].tolist() for m in (1, 2, 3, 7)}
    undone_cut = [r[0] for r in rows if r[2] == 3 and r[3] != 0 and r[1] <= 1500]
    assert undone_cut
    k = store.prune(3, 1500)
    after = store.rowid[store.live_rows(3)].tolist()
    gt_of = {r[0]: r[1] for r in rows}
    assert k == len(before[3]) - len(after) + len(undone_cut) > len(undone_cut)
    assert all(bool(store.deleted[int(np.flatnonzero(store.rowid == i)[0])]) for i in undone_cut)
    assert after == [r for r in before[3] if gt_of[r] > 1500]
    assert all(store.rowid[store.live_rows(m)].tolist() == before[m] for m in (1, 2, 7))
    assert store.prune(3, 1500) == 0 and store.prune(99, 10 ** 6) == 0

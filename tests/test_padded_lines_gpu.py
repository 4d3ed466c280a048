"""The store's line copy holds every packet's padded message (dsy_message.h line_bytes_for: 0x80 and zeros after the
packet up to the end of its final 64-byte block), and the responder hashes 1-byte-prefixed claims straight from it
(k_pair_test<..., PADDED>) while 2- to 4-byte prefixes shift and mask (PADDED=false), in separate launches of one
call.  Packet lengths here walk every residue around the padding boundaries -- (1 + len) mod 64 in 55..64, where the
bit length spills into one more block, and (1 + len) mod 128 in 119..128, where the padded message needs one more
128-byte line -- for rows uploaded with the store and rows appended later (the append path lays out its own lines),
MD5 and SHA-1 filters, against the sqlite + hashlib oracle (oracle/sync_ref.respond_lists = community.py:2746-2811
+ :2555-2567)."""
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

GT_NOW = 3_000


def _lengths(rng, n):
    """Every length 1..400 (all residues mod 64 and mod 128 several times over), then boundary lengths of longer
    packets (127 + 128 j .. 136 + 128 j) and a few long ones."""
    base = list(range(1, 401))
    edges = [128 * j + d for j in range(3, 40) for d in range(-9, 2)]
    longs = [int(x) for x in rng.integers(2000, 9000, size=40)]
    out = base + edges + longs
    rng.shuffle(out)
    return (out * (n // len(out) + 1))[:n]


def _rows(seed, n):
    rng = np.random.Generator(np.random.PCG64(seed))
    lengths = _lengths(rng, n)
    gt = rng.integers(1, GT_NOW + 1, size=n)
    rows = [(i + 1, int(gt[i]), 1, 0, rng.bytes(lengths[i])) for i in range(n)]
    return rows


def _sqlite(rows):
    conn = sqlite3.connect(":memory:")
    conn.executescript(SYNC_SCHEMA)
    conn.executemany("INSERT INTO sync(id, community, member, global_time, meta_message, undone, packet, sequence) "
                     "VALUES (?, 1, ?, ?, ?, ?, ?, 0)", [(r[0], r[0], r[1], r[2], r[3], r[4]) for r in rows])
    return conn


@pytest.mark.parametrize("appended", [False, True], ids=["uploaded", "appended"])
def test_padding_boundaries_vs_oracle(appended):
    rows = _rows(61 if appended else 60, 6000)
    conn = _sqlite(rows)
    if appended:  # half the rows go through dsy_store_append's line layout, in two batches
        store = SyncStore.from_rows(rows[:3000])
        store.handle  # noqa: B018 -- on the device before the appends
        for part in (rows[3000:4500], rows[4500:]):
            store.append([r[4] for r in part], [r[1] for r in part], [r[2] for r in part], [r[0] for r in part])
    else:
        store = SyncStore.from_rows(rows)
    served = [MetaMessage("a", 1, SyncDistribution("ASC", 128, None))]
    served_oracle = [dict(name="a", id=1, direction="ASC", priority=128, pruning=None)]
    com = SyncCommunity(store, served, global_time=GT_NOW)
    rng = np.random.Generator(np.random.PCG64(7))
    packets = [r[4] for r in rows]
    reqs, blooms = [], []
    for q in range(48):
        plen = [1, 1, 1, 2, 3, 4][q % 6]  # 1 byte: the padded launch; 2-4 bytes: the masking launch
        m, f = [(10160, 0.01), (4096, 0.001)][q % 2]  # MD5 k = 7, SHA-1 k = 10
        prefix = bytes(rng.integers(0, 256, size=plen, dtype=np.uint8))
        bf, ob = BloomFilter(m, f, prefix), OracleBloom.from_m_f(m, f, prefix)
        known = [p for p in packets if rng.random() < 0.9]
        bf.add_keys(known)
        ob.add_keys(known)
        modulo = [1, 1, 5][q % 3]
        lo = int(rng.integers(1, GT_NOW // 2))
        reqs.append(ClaimRequest(lo, GT_NOW, modulo, int(rng.integers(0, modulo)), bf))
        blooms.append(ob)
    for limit in (5120, 1 << 40):
        got = com.respond(reqs, byte_limit=limit)
        for i, (q, ob, g) in enumerate(zip(reqs, blooms, got)):
            want = sync_ref.respond_lists(conn, served_oracle, (q.time_low, q.time_high, q.offset, q.modulo), ob,
                                          GT_NOW, limit, False)
            assert store.rowid[g].tolist() == want, (i, len(q.bloom_filter.prefix), limit)


@pytest.mark.parametrize("plens", [[2, 1, 3, 1], [4, 4, 1, 2, 1, 1, 3]], ids=["2131", "4412113"])
def test_one_family_mixed_prefixes_first_window(plens):
    """one hash family (MD5 m=10160) whose claims mix 1-byte and 2-4-byte prefixes, one meta (the
    fused first window, k_fill_first).  The 1-byte claims are moved to the front of the family's run, so the first
    active list is not the identity and k_fill_first must map its slots through it -- each claim's rows hashed against
    its own filter and prefix, and answered in its own slot."""
    rows = _rows(62, 3000)
    conn = _sqlite(rows)
    store = SyncStore.from_rows(rows)
    served = [MetaMessage("a", 1, SyncDistribution("ASC", 128, None))]
    served_oracle = [dict(name="a", id=1, direction="ASC", priority=128, pruning=None)]
    com = SyncCommunity(store, served, global_time=GT_NOW)
    rng = np.random.Generator(np.random.PCG64(11))
    packets = [r[4] for r in rows]
    reqs, blooms = [], []
    for q, plen in enumerate(plens):
        prefix = bytes(rng.integers(0, 256, size=plen, dtype=np.uint8))
        bf, ob = BloomFilter(10160, 0.01, prefix), OracleBloom.from_m_f(10160, 0.01, prefix)
        # claims differ in what they hold, so answering one with another's filter shows
        known = [p for p in packets if rng.random() < (0.5 if q % 2 else 0.95)]
        bf.add_keys(known)
        ob.add_keys(known)
        lo = int(rng.integers(1, GT_NOW // 4))
        reqs.append(ClaimRequest(lo, GT_NOW, 1 + q % 2, 0, bf))
        blooms.append(ob)
    for limit in (5120, 1 << 40):
        got = com.respond(reqs, byte_limit=limit)
        for i, (q, ob, g) in enumerate(zip(reqs, blooms, got)):
            want = sync_ref.respond_lists(conn, served_oracle, (q.time_low, q.time_high, q.offset, q.modulo), ob,
                                          GT_NOW, limit, False)
            assert store.rowid[g].tolist() == want, (i, plens, limit)


def test_packets_past_the_piece_limit_take_direct_loads():
    """the line-staged pieces keep 16-bit live-byte limits, which a padded message of a >= 65527-byte
    packet exceeds.  A store holding such packets (longer than the reference's UDP cap, e.g. built from another
    source) hashes through the direct loads (StoreView.max_len > kLinePathMaxLen) and still answers as the oracle."""
    rng = np.random.Generator(np.random.PCG64(63))
    lengths = [65525, 65526, 65527, 65528, 65534, 65535, 65536, 70001] + [int(x) for x in rng.integers(1, 3000, 200)]
    rng.shuffle(lengths)
    rows = [(i + 1, int(rng.integers(1, GT_NOW + 1)), 1, 0, rng.bytes(n)) for i, n in enumerate(lengths)]
    rows.sort(key=lambda r: r[1])
    rows = [(i + 1,) + r[1:] for i, r in enumerate(rows)]
    conn = _sqlite(rows)
    store = SyncStore.from_rows(rows)
    served = [MetaMessage("a", 1, SyncDistribution("ASC", 128, None))]
    served_oracle = [dict(name="a", id=1, direction="ASC", priority=128, pruning=None)]
    com = SyncCommunity(store, served, global_time=GT_NOW)
    packets = [r[4] for r in rows]
    reqs, blooms = [], []
    for q in range(8):
        m, f = [(10160, 0.01), (4096, 0.001)][q % 2]
        prefix = bytes(rng.integers(0, 256, size=[1, 2][q // 4], dtype=np.uint8))
        bf, ob = BloomFilter(m, f, prefix), OracleBloom.from_m_f(m, f, prefix)
        known = [p for p in packets if rng.random() < 0.7]
        bf.add_keys(known)
        ob.add_keys(known)
        reqs.append(ClaimRequest(1, GT_NOW, 1, 0, bf))
        blooms.append(ob)
    got = com.respond(reqs, byte_limit=1 << 40)
    for i, (q, ob, g) in enumerate(zip(reqs, blooms, got)):
        want = sync_ref.respond_lists(conn, served_oracle, (q.time_low, q.time_high, q.offset, q.modulo), ob,
                                      GT_NOW, 1 << 40, False)
        assert store.rowid[g].tolist() == want, i

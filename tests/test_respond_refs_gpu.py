"""dsy_sync_respond_refs (the drop-in SyncCommunity.respond path: per claim its four range fields and its BloomFilter's
(record, filter bytes) addresses; the library lays the filters out and gathers them into pinned staging while the GPU
selects) against dsy_sync_respond over a caller-packed blob and against the sqlite + hashlib oracle
(oracle/sync_ref.respond_lists = community.py:2746-2811 + :2555-2567): filter sizes that are not a multiple of 4 bytes
(10160 bits = 1270 bytes), mixed shapes in one batch, an empty batch, and the argument checks."""
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


def _claims(rows, gt_now, rng, shapes, n):
    packets = {r[0]: r[4] for r in rows}
    reqs, blooms = [], []
    for q in range(n):
        modulo = int(rng.choice([1, 3, 17]))
        lo = int(rng.integers(1, gt_now // 2))
        hi = int(rng.integers(lo, gt_now + 10))
        m, f = shapes[q % len(shapes)]
        prefix = bytes(rng.integers(0, 256, size=int(q % 4), dtype=np.uint8))
        bf, ob = BloomFilter(m, f, prefix), OracleBloom.from_m_f(m, f, prefix)
        known = [packets[r[0]] for r in rows if rng.random() < 0.85]
        bf.add_keys(known)
        ob.add_keys(known)
        reqs.append(ClaimRequest(lo, hi, modulo, int(rng.integers(0, modulo)), bf))
        blooms.append(ob)
    return reqs, blooms


@pytest.mark.parametrize("shapes", [[(10160, 0.01)], [(10160, 0.01), (4096, 0.001), (1 << 15, 0.01), (8, 0.5)]],
                         ids=["mtu", "mixed"])
def test_gather_equals_blob_and_oracle(shapes):
    rows, conn = build(11, 8_000, 40_000, False)
    store = SyncStore.from_rows(rows)
    gt_now = 40_100
    chosen = [m for m in METAS if m[0] in ("a", "d")]
    com = SyncCommunity(store, [MetaMessage(n, i, SyncDistribution(d, p, None)) for n, i, d, p, _ in chosen],
                        global_time=gt_now)
    served_oracle = [dict(name=n, id=i, direction=d, priority=p, pruning=None) for n, i, d, p, _ in chosen]
    reqs, blooms = _claims(rows, gt_now, np.random.Generator(np.random.PCG64(5)), shapes, 40)
    for limit in (2048, 1 << 40):
        got = com.respond(reqs, byte_limit=limit, random_seed=7)  # the refs path
        packed, R, blob = com.request_records(reqs)
        want_blob = com._respond_requests(packed, R, blob, False, limit, 7)  # a caller-packed blob
        for q, ob, g, b in zip(reqs, blooms, got, want_blob):
            assert g.tolist() == b.tolist()
            want = sync_ref.respond_lists(conn, served_oracle, (q.time_low, q.time_high, q.offset, q.modulo), ob,
                                          gt_now, limit, False)
            assert store.rowid[g].tolist() == want, (q.time_low, q.time_high, q.modulo, q.offset, limit)


def test_gather_of_many_claims_in_chunks():
    """>= 256 claims: the library gathers the filters in four chunks, each uploaded while the next is copied -- the
    answers equal the caller-packed blob path's for every claim (no gather there) and the oracle's for a sample."""
    rows, conn = build(12, 6_000, 30_000, False)
    store = SyncStore.from_rows(rows)
    gt_now = 30_100
    chosen = [m for m in METAS if m[0] in ("a", "d")]
    com = SyncCommunity(store, [MetaMessage(n, i, SyncDistribution(d, p, None)) for n, i, d, p, _ in chosen],
                        global_time=gt_now)
    served_oracle = [dict(name=n, id=i, direction=d, priority=p, pruning=None) for n, i, d, p, _ in chosen]
    shapes = [(10160, 0.01), (4096, 0.001), (1 << 15, 0.01), (8, 0.5), (10168, 0.01)]
    reqs, blooms = _claims(rows, gt_now, np.random.Generator(np.random.PCG64(9)), shapes, 300)
    for rep in range(3):  # the ctx's staging and filters workspace are reused call after call
        got = com.respond(reqs, byte_limit=4096, random_seed=11 + rep)
        packed, R, blob = com.request_records(reqs)
        want_blob = com._respond_requests(packed, R, blob, False, 4096, 11 + rep)
        assert [g.tolist() for g in got] == [b.tolist() for b in want_blob]
    for i in range(0, 300, 15):
        q = reqs[i]
        want = sync_ref.respond_lists(conn, served_oracle, (q.time_low, q.time_high, q.offset, q.modulo), blooms[i],
                                      gt_now, 4096, False)
        assert store.rowid[got[i]].tolist() == want, i


def test_refs_layout_and_argument_checks():
    rows, _ = build(12, 2_000, 9_000, False)
    store = SyncStore.from_rows(rows)
    com = SyncCommunity(store, [MetaMessage("a", 1, SyncDistribution("ASC", 128, None))], global_time=9_100)
    assert len(com.respond([])) == 0
    bfs = [BloomFilter(m, 0.01, b"") for m in (10160, 4096, 10160)]
    R = len(bfs)
    ranges = np.array([[1, 9_000, 1, 0]] * R, dtype=np.uint64)
    refs = np.frombuffer(b"".join(bf._refs for bf in bfs), dtype=np.uint64).copy()
    ctx, lib = store.ctx, store.ctx.lib
    mt, nm = com.meta_records()
    out, off = np.empty(1 << 16, dtype=np.uint64), np.zeros(R + 1, dtype=np.uint64)

    def call(rg, rf):
        return lib.dsy_sync_respond_refs(ctx.handle, store.handle, rg.ctypes.data, rf.ctypes.data, R, mt, nm, 9_100, 0,
                                         1 << 40, 1, out.ctypes.data, len(out), off.ctypes.data)

    _native.check(call(ranges, refs))
    # every row of gt 1..9000 is missing from the empty filters: the whole meta comes back, three times
    n_rows = int(sum(1 for r in rows if r[2] == 1 and r[1] <= 9_000 and not r[3]))
    assert np.diff(off).tolist() == [n_rows] * 3
    # a bound past 2^63-1 is clamped, as the record form requires of its caller (community.py:2545-2548)
    big = ranges.copy()
    big[:, 1] = np.uint64(0xFFFFFFFFFFFFFFFF)
    _native.check(call(big, refs))
    assert np.diff(off).tolist() == [n_rows] * 3
    bad = refs.copy()
    bad[3] = 0  # claim 1's filter address
    assert call(ranges, bad) == _native.DSY_EINVAL
    odd = ranges.copy()
    odd[2, 3] = 5  # offset >= modulo
    assert call(odd, refs) == _native.DSY_EINVAL

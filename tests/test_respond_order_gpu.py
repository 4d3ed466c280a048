"""The responder across a sequence of calls whose claim counts differ, in ONE process, every answer against the sqlite +
hashlib oracle (oracle/sync_ref.respond_lists = community.py:2746-2811 + the byte-limited loop :2555-2567).

Round 3 recorded an illegal memory access in the first synchronous call of the pipelined test when the drop-in
gather tests had run before it in the same process (gpurun_out/dbg_b.log).  tools/order_repro.py reproduced it on the
round-3 library with plain dsy_sync_respond calls (profiles/fault_r4.md).  The cause: the split windows' sort state
(bulk_hist / bulk_cur, R x 1024 words each) lives in a grow-only workspace whose layout depends on the call's R
(bulk_cur starts R x 1024 words in).  It was zeroed only when the workspace grew, and only the requested bytes of the
1.25x allocation, so a later call with a larger R that still fit read never-written memory as its sort cursors, and
k_fill_sort wrote task records past the claim's window.  Memory HIP hands back after other tests freed theirs is not
zero, so the fault depended on what ran before.  Now every call zeroes its own rows in its first kernel (k_setup /
k_fill_first), and device-side bounds checks turn any such index into DSY_EINTERNAL instead of a fault.

The sequence below is that order: the gather tests' workloads (mixed filter sizes including a saturated m = 8 filter,
prefixes of 0-3 bytes, two metas, a 2 KiB and an unbounded budget), an empty batch, three empty filters with an
unbounded budget, then memory poisoned with 0xFF and handed back to HIP, then batches of 64, 96, 128 and 160 claims --
each inside the slack of the workspace the one before grew -- synchronously and three in flight."""
import numpy as np
import pytest
import torch

from dispersy_amd import BloomFilter
from dispersy_amd.community import ClaimRequest, SyncCommunity
from dispersy_amd.distribution import MetaMessage, SyncDistribution
from dispersy_amd.store import SyncStore
from oracle import sync_ref
from oracle.bloom_ref import OracleBloom
from test_pipeline_gpu import _Batch, _submit, _wait
from test_respond_scale_gpu import METAS, build

pytestmark = pytest.mark.gpu

CHOSEN = [m for m in METAS if m[0] in ("a", "d")]


def _community(store, gt_now, chosen=CHOSEN):
    com = SyncCommunity(store, [MetaMessage(n, i, SyncDistribution(d, p, None)) for n, i, d, p, _ in chosen],
                        global_time=gt_now)
    served = [dict(name=n, id=i, direction=d, priority=p, pruning=None) for n, i, d, p, _ in chosen]
    return com, served


def _claims(rows, rng, n, shapes, gt_lo, gt_hi, span=None, keep=0.85, prefix_len=None):
    packets = {r[0]: r[4] for r in rows}
    reqs, blooms = [], []
    for q in range(n):
        modulo = int(rng.choice([1, 1, 3, 17]))
        lo = int(rng.integers(gt_lo, gt_hi))
        hi = lo + int(rng.integers(50, span)) if span else int(rng.integers(lo, gt_hi + 10))
        m, f = shapes[q % len(shapes)]
        plen = q % 4 if prefix_len is None else prefix_len
        prefix = bytes(rng.integers(0, 256, size=plen, dtype=np.uint8))
        bf, ob = BloomFilter(m, f, prefix), OracleBloom.from_m_f(m, f, prefix)
        known = [packets[r[0]] for r in rows if lo <= r[1] <= hi and rng.random() < keep]
        bf.add_keys(known)
        ob.add_keys(known)
        reqs.append(ClaimRequest(lo, hi, modulo, int(rng.integers(0, modulo)), bf))
        blooms.append(ob)
    return reqs, blooms


def _want(conn, served, reqs, blooms, gt_now, limit):
    return [sync_ref.respond_lists(conn, served, (q.time_low, q.time_high, q.offset, q.modulo), ob, gt_now, limit,
                                   False) for q, ob in zip(reqs, blooms)]


def _check(store, got, want, what):
    assert len(got) == len(want), what
    for i, (g, w) in enumerate(zip(got, want)):
        assert store.rowid[np.asarray(g, dtype=np.int64)].tolist() == w, (what, i)


def _poison(dev, mib=1024):
    """Fill device memory with 0xFF and hand it back to HIP (torch's cache emptied), so the next workspace the
    library grows is likely to start on non-zero bytes, as it did after the gather tests in round 3."""
    torch.cuda.synchronize()
    chunks = [torch.full((64 << 20,), 0xFF, dtype=torch.uint8, device=dev) for _ in range(mib // 64)]
    torch.cuda.synchronize()
    del chunks
    torch.cuda.empty_cache()


def test_calls_of_changing_claim_counts_vs_oracle():
    dev = torch.device("cuda", 0)
    rng = np.random.Generator(np.random.PCG64(5))
    # 1: the gather tests' workloads (two metas, so every call plans in k_setup and big claims take split windows)
    rows, conn = build(11, 8_000, 40_000, False)
    store = SyncStore.from_rows(rows)
    com, served = _community(store, 40_100)
    for shapes in ([(10160, 0.01)], [(10160, 0.01), (4096, 0.001), (1 << 15, 0.01), (8, 0.5)]):
        reqs, blooms = _claims(rows, rng, 40, shapes, 1, 20_000)
        for limit in (2048, 1 << 40):
            got = com.respond(reqs, byte_limit=limit, random_seed=7)
            _check(store, got, _want(conn, served, reqs, blooms, 40_100, limit), ("gather workload", shapes, limit))
    # 2: an empty batch, then three empty filters with an unbounded budget (every row of the meta comes back)
    rows2, conn2 = build(12, 2_000, 9_000, False)
    store2 = SyncStore.from_rows(rows2)
    com2, served2 = _community(store2, 9_100, [m for m in METAS if m[0] == "a"])
    assert len(com2.respond([], byte_limit=1 << 40)) == 0
    reqs2 = [ClaimRequest(1, 9_000, 1, 0, BloomFilter(m, 0.01, b"")) for m in (10160, 4096, 10160)]
    blooms2 = [OracleBloom.from_m_f(m, 0.01, b"") for m in (10160, 4096, 10160)]
    got = com2.respond(reqs2, byte_limit=1 << 40, random_seed=1)
    _check(store2, got, _want(conn2, served2, reqs2, blooms2, 9_100, 1 << 40), "empty filters")
    del store, store2
    # 3: recycled, non-zero device memory; then growing batches on a new store, synchronously and in flight
    _poison(dev)
    rows3, conn3 = build(3, 30_000, 12_000, False)
    store3 = SyncStore.from_rows(rows3)
    com3, served3 = _community(store3, 12_000)
    batches = []
    for b in range(4):
        reqs, blooms = _claims(rows3, rng, 64 + 32 * b, [(10160, 0.01), (10160, 0.01), (4096, 0.001)], 1, 11_000,
                               span=4000, keep=0.9, prefix_len=1)
        batches.append((reqs, blooms, _want(conn3, served3, reqs, blooms, 12_000, 5120)))
    for b, (reqs, blooms, want) in enumerate(batches):
        _check(store3, com3.respond(reqs, byte_limit=5120, random_seed=7), want, ("synchronous batch", b))
    ctx = store3.ctx
    bs = [_Batch(com3, reqs) for reqs, _, _ in batches]
    tickets = [(i, _submit(ctx, store3, com3, bs[i], 5120)) for i in range(3)]
    assert all(rc == 0 for _, (rc, _) in tickets)
    for i, (_, t) in tickets:
        got, _ = _wait(ctx, t, bs[i].R)
        _check(store3, got, batches[i][2], ("batch in flight", i))
    rc, t = _submit(ctx, store3, com3, bs[3], 5120)
    assert rc == 0
    got, _ = _wait(ctx, t, bs[3].R)
    _check(store3, got, batches[3][2], ("batch in flight", 3))

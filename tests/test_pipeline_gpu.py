"""The pipelined responder (dsy_sync_respond_submit / dsy_sync_respond_wait): up to three batches in flight on
their own workspaces and streams must answer exactly what the synchronous call answers, batch by batch, and the ctx
must refuse what would race with them (a fourth batch, a store change, a synchronous call)."""
import ctypes

import numpy as np
import pytest
import torch

from dispersy_amd import BloomFilter, _native
from dispersy_amd.community import ClaimRequest, SyncCommunity
from dispersy_amd.distribution import MetaMessage, SyncDistribution
from dispersy_amd.store import SyncStore

pytestmark = pytest.mark.gpu

_hip = None


def _d2h(ptr, n, dtype=np.uint64):
    """n elements at device pointer ptr -> numpy (hipMemcpy, device to host)."""
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so")
    out = np.zeros(max(n, 1), dtype=dtype)
    if n:
        assert _hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(ptr), ctypes.c_size_t(n * out.itemsize),
                              2) == 0
    return out[:n]


def _setup(n=30_000, seed=3):
    rng = np.random.Generator(np.random.PCG64(seed))
    gts = rng.integers(1, 12_000, size=n)
    rows = [(i + 1, int(gts[i]), 1 + int(i % 4 == 0), 0, i.to_bytes(4, "big") + rng.bytes(int(rng.integers(20, 900))))
            for i in range(n)]
    store = SyncStore.from_rows(rows)
    metas = [MetaMessage("a", 1, SyncDistribution("ASC", 128)), MetaMessage("d", 2, SyncDistribution("DESC", 200))]
    com = SyncCommunity(store, metas, global_time=12_000)
    batches = []
    for b in range(4):
        claims = []
        for i in range(64 + 32 * b):
            lo = int(rng.integers(1, 11_000))
            hi = lo + int(rng.integers(50, 4000))
            modulo = int(rng.integers(1, 6))
            bf = BloomFilter(10160 if i % 3 else 4096, 0.01 if i % 3 else 0.001, bytes([int(rng.integers(0, 256))]))
            bf.add_keys([r[4] for r in rows if lo <= r[1] <= hi and rng.random() < 0.9])
            claims.append(ClaimRequest(lo, hi, modulo, int(rng.integers(0, modulo)), bf))
        batches.append(claims)
    return store, com, batches


class _Batch(object):
    """One batch's C-ABI arguments: its dsy_request records and its filters in device memory."""

    def __init__(self, com, claims):
        self.reqs, self.R, blob = com.request_records(claims)
        self.d_filters = torch.frombuffer(bytearray(blob + bytes(64)), dtype=torch.uint8).to("cuda:0")
        torch.cuda.synchronize()
        self.mt, self.nm = com.meta_records()


def _submit(ctx, store, com, b, byte_limit):
    t = ctypes.c_uint64()
    rc = ctx.lib.dsy_sync_respond_submit(ctx.handle, store.handle, b.reqs.ctypes.data_as(ctypes.POINTER(_native.Request)),
                                         b.R, b.d_filters.data_ptr(), b.mt, b.nm, com.global_time, 0, byte_limit, 7,
                                         ctypes.byref(t))
    return rc, t.value


def _wait(ctx, ticket, R):
    p_out, p_off, pairs = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
    _native.check(ctx.lib.dsy_sync_respond_wait(ctx.handle, ticket, ctypes.byref(p_out), ctypes.byref(p_off),
                                                ctypes.byref(pairs)))
    off = _d2h(p_off.value, R + 1)
    rows = _d2h(p_out.value, int(off[R]))
    return [rows[int(off[i]):int(off[i + 1])].astype(np.int64).tolist() for i in range(R)], pairs.value


@pytest.mark.parametrize("byte_limit", [5120, 60_000])
def test_in_flight_batches_equal_synchronous(byte_limit):
    store, com, claim_batches = _setup()
    ctx = store.ctx
    want = [[r.tolist() for r in com.respond(c, byte_limit=byte_limit, random_seed=7)] for c in claim_batches]
    bs = [_Batch(com, c) for c in claim_batches]
    tickets = []
    for b in bs[:3]:
        rc, t = _submit(ctx, store, com, b, byte_limit)
        assert rc == 0
        tickets.append(t)
    assert len(set(tickets)) == 3
    # a fourth batch, a store change and a synchronous call would race with the three in flight
    rc3, _ = _submit(ctx, store, com, bs[3], byte_limit)
    assert rc3 == _native.DSY_EINVAL
    with pytest.raises(_native.DsyError):
        com.respond(claim_batches[3], byte_limit=byte_limit, random_seed=7)
    one = np.asarray([10], dtype=np.uint64)
    assert ctx.lib.dsy_store_delete(ctx.handle, store.handle, one.ctypes.data, 1, None) == _native.DSY_EINVAL
    got1, _ = _wait(ctx, tickets[1], bs[1].R)  # out of submission order
    assert got1 == want[1]
    rc3, t3 = _submit(ctx, store, com, bs[3], byte_limit)  # a slot is free again
    assert rc3 == 0
    got0, pairs0 = _wait(ctx, tickets[0], bs[0].R)
    got3, _ = _wait(ctx, t3, bs[3].R)
    got2, _ = _wait(ctx, tickets[2], bs[2].R)
    assert got0 == want[0]
    assert got2 == want[2]
    assert got3 == want[3]
    assert pairs0 > 0
    with pytest.raises(_native.DsyError):
        _wait(ctx, t3, bs[3].R)  # already waited for
    # nothing in flight: the synchronous call runs again
    assert [r.tolist() for r in com.respond(claim_batches[0], byte_limit=byte_limit, random_seed=7)] == want[0]


@pytest.mark.parametrize("depth", [2, 3])
def test_pipelined_stream_of_batches(depth):
    """Ten batches served `depth` deep, as bench.py does: every answer equals the synchronous one."""
    store, com, claim_batches = _setup(seed=4)
    ctx = store.ctx
    want = [[r.tolist() for r in com.respond(c, byte_limit=5120, random_seed=7)] for c in claim_batches]
    bs = [_Batch(com, c) for c in claim_batches]
    pending = []
    for k in range(10):
        i = k % len(bs)
        rc, t = _submit(ctx, store, com, bs[i], 5120)
        assert rc == 0
        pending.append((i, t))
        if len(pending) == depth:
            j, tj = pending.pop(0)
            got, _ = _wait(ctx, tj, bs[j].R)
            assert got == want[j], k
    for j, tj in pending:
        got, _ = _wait(ctx, tj, bs[j].R)
        assert got == want[j]

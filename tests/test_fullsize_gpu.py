"""BASELINE configs[1] at its full size: one responder with 10 M stored packets (100-1500 B, global_time 1..N) answers
1024 claims (half largest-style, half modulo-style, as bench.py's headline) through dsy_sync_respond, and EVERY
claim's answer is checked against the CPU oracle.

The oracle is oracle/sync_ref.respond_arrays -- the reference's responder (community.py:2746-2811 + the byte-limited
loop :2555-2567) over in-memory columns: the claim's candidates in send order, each hashed with hashlib through
oracle/bloom_ref's lazy not_filter (bloomfilter.py:214-237), the walk stopping at the packet that spends the budget.
It runs for every claim, fanned out over 16 spawned worker processes (tests/oracle_pool.py), on the packets of the
claims' candidate rows gathered from HBM.  MD5 MTU filters (m = 10160, f = 0.01) and the SHA-1 test-harness filters of
node.py:617 (m = 4096, f = 0.001); config 5 (heavy tail) checks 256 of its 1024 claims the same way."""
import ctypes
import math

import numpy as np
import pytest

from dispersy_amd import _native
from dispersy_amd.bloomfilter import BloomFilter
from oracle_pool import check_claims

pytestmark = pytest.mark.gpu

N = 10_000_000
R = 1024
LIMIT = 5120


@pytest.fixture(scope="module")
def world():
    import torch
    ctx = _native.Context(0)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    lengths = torch.randint(100, 1501, (N,), device=dev, generator=g, dtype=torch.int64)
    offsets = torch.zeros(N + 1, device=dev, dtype=torch.int64)
    torch.cumsum(lengths, 0, out=offsets[1:])
    total = int(offsets[-1].item())
    G = _native.BLOB_GUARD
    blob_full = torch.randint(0, 256, (total + 2 * G,), device=dev, generator=g, dtype=torch.uint8)
    blob = blob_full[G:]
    gt = torch.arange(1, N + 1, device=dev, dtype=torch.int64)
    meta = torch.ones(N, device=dev, dtype=torch.int32)
    torch.cuda.synchronize()
    store = ctypes.c_void_p()
    _native.check(ctx.lib.dsy_store_attach(ctx.handle, blob.data_ptr(), total, offsets.data_ptr(), N, gt.data_ptr(),
                                           meta.data_ptr(), None, ctypes.byref(store)))
    yield torch, ctx, dev, store, blob, offsets, lengths.cpu().numpy()
    ctx.lib.dsy_store_free(store)
    del blob_full, offsets, gt, meta
    torch.cuda.empty_cache()


def claims_of(ctx, store, rng, bits, f):
    """bench.py's headline claims: even ones largest-style (~capacity consecutive global times), odd ones
    modulo-style (the whole store, one residue class); each filter holds its range but a random 1 %."""
    capacity = BloomFilter(bits, f).get_capacity(f)
    modulo_m = int(math.ceil(N / float(capacity)))
    reqs = (_native.Request * R)()
    out, raws, off = [], [], 0
    for i in range(R):
        if i % 2 == 0:
            lo = int(rng.integers(1, N - capacity + 1))
            hi, modulo, offset = lo + capacity - 1, 1, 0
            rows = np.arange(lo - 1, hi, dtype=np.int64)
        else:
            lo, hi, modulo = 1, N, modulo_m
            offset = int(rng.integers(0, modulo))
            first = (modulo - offset) % modulo or modulo
            rows = np.arange(first, N + 1, modulo, dtype=np.int64) - 1
        pre = bytes([int(rng.integers(0, 256))])
        bf = BloomFilter(bits, f, pre)
        known = np.ascontiguousarray(rows[rng.random(len(rows)) >= 0.01].astype(np.uint64))
        buf = ctypes.create_string_buffer(bf.bytes, len(bf.bytes))
        _native.check(ctx.lib.dsy_bloom_add_rows(ctx.handle, ctypes.byref(bf.params), store, known.ctypes.data,
                                                 len(known), buf))
        raw = buf.raw + b"\x00" * ((-len(buf.raw)) % 4)
        q = reqs[i]
        q.time_low, q.time_high, q.modulo, q.offset = lo, hi, modulo, offset
        q.filter_offset, q.m_bits, q.k = off, bf.size, bf.functions
        q.hash_kind, q.chunk_bytes = _native.HASH_KINDS[bf.hash_name], bf.chunk_bytes
        q.prefix_len = 1
        q.prefix[0] = pre[0]
        out.append((rows, bf, pre, buf.raw, off))
        raws.append(raw)
        off += len(raw)
    return reqs, out, b"".join(raws)


@pytest.mark.parametrize("bits,f", [(10160, 0.01), (4096, 0.001)])
def test_full_size_every_claim(world, bits, f):
    torch, ctx, dev, store, blob, offsets, lens = world
    lib = ctx.lib
    rng = np.random.Generator(np.random.PCG64(7 if bits == 10160 else 8))
    reqs, claims, fblob = claims_of(ctx, store, rng, bits, f)
    metas = (_native.Meta * 1)()
    metas[0].meta_id, metas[0].direction = 1, _native.DSY_ASC
    h_off = np.zeros(R + 1, dtype=np.uint64)
    h_idx = np.zeros(1 << 22, dtype=np.uint64)
    torch.cuda.synchronize()
    # the host-buffer entry point: the filters go up the bus, the answers come back
    _native.check(lib.dsy_sync_respond(ctx.handle, store, reqs, R, fblob, len(fblob), metas, 1, N, 0, LIMIT, 99,
                                       h_idx.ctypes.data, len(h_idx), h_off.ctypes.data))
    # the oracle over every claim: the packets of all candidate rows, gathered from HBM, in worker processes
    rows = np.unique(np.concatenate([c[0] for c in claims]))
    packets, poff = gather_rows(torch, dev, blob, offsets, rows)
    want = check_claims([oracle_claim(reqs[i], c) for i, c in enumerate(claims)], packets, poff, rows,
                        np.arange(1, N + 1, dtype=np.uint64), N, LIMIT, work=[len(c[0]) for c in claims])
    sent = 0
    for i in range(R):
        got = h_idx[h_off[i]:h_off[i + 1]].astype(np.int64).tolist()
        assert got == want[i], (i, len(got), len(want[i]))
        sent += len(got)
    assert sent > R  # most claims send several packets


def gather_rows(torch, dev, blob, offsets, rows, chunk=1 << 18):
    """The packets of store rows `rows` (sorted), back to back, copied from the device blob in chunks: (bytes as
    a uint8 array, offsets)."""
    d_off = offsets
    lens = (d_off[torch.from_numpy(rows + 1).to(dev)] - d_off[torch.from_numpy(rows).to(dev)]).cpu().numpy()
    poff = np.zeros(len(rows) + 1, dtype=np.int64)
    np.cumsum(lens, out=poff[1:])
    out = np.empty(int(poff[-1]), dtype=np.uint8)
    for a in range(0, len(rows), chunk):
        b = min(len(rows), a + chunk)
        d_rows = torch.from_numpy(rows[a:b]).to(dev)
        beg, ln = d_off[d_rows], d_off[d_rows + 1] - d_off[d_rows]
        koff = torch.zeros(b - a + 1, device=dev, dtype=torch.int64)
        torch.cumsum(ln, 0, out=koff[1:])
        n = int(koff[-1].item())
        seg = torch.repeat_interleave(torch.arange(b - a, device=dev), ln)
        pos = torch.arange(n, device=dev, dtype=torch.int64)
        out[int(poff[a]):int(poff[b])] = blob[beg[seg] + (pos - koff[seg])].cpu().numpy()
        del d_rows, beg, ln, koff, seg, pos
    return out, poff


def oracle_claim(q, c):
    """(time_low, time_high, offset, modulo, filter bytes, k, prefix) of claim q (its claims_of tuple c)."""
    return (int(q.time_low), int(q.time_high), int(q.offset), int(q.modulo), c[3], c[1].functions, c[2])


def heavy_tail_world(torch, ctx, dev):
    """bench.py's config 5 store: discretised Pareto(1.2) lengths clipped to [60, 65476] (the UDP cap,
    endpoint.py:263) and Zipf(1.1) global times over 1..10^6 (gt 1 holds ~9 % of the rows)."""
    G = _native.BLOB_GUARD
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    u = torch.rand(N, device=dev, generator=g, dtype=torch.float64)
    lengths = torch.clamp(torch.floor(60.0 * u.pow(-1.0 / 1.2)), max=65476).to(torch.int64)
    del u
    offsets = torch.zeros(N + 1, device=dev, dtype=torch.int64)
    torch.cumsum(lengths, 0, out=offsets[1:])
    total = int(offsets[-1].item())
    blob_full = torch.randint(0, 256, (total + 2 * G,), device=dev, generator=g, dtype=torch.uint8)
    w = torch.arange(1, 1_000_001, device=dev, dtype=torch.float64).pow(-1.1)
    cdf = torch.cumsum(w, 0)
    cdf /= cdf[-1].clone()
    gt = torch.searchsorted(cdf, torch.rand(N, device=dev, generator=g, dtype=torch.float64)) + 1
    gt = torch.clamp(gt, max=1_000_000).sort().values.contiguous()
    meta = torch.ones(N, device=dev, dtype=torch.int32)
    torch.cuda.synchronize()
    store = ctypes.c_void_p()
    _native.check(ctx.lib.dsy_store_attach(ctx.handle, blob_full.data_ptr() + G, total, offsets.data_ptr(), N,
                                           gt.data_ptr(), meta.data_ptr(), None, ctypes.byref(store)))
    return store, blob_full, offsets, lengths.cpu().numpy(), gt.cpu().numpy()


def test_heavy_tail_full_size_sample(world):
    """Config 5 at its full size: the 1024 claims of bench.py's heavy_tail leg in one call (claims whose filters
    saturate walk 10^5-10^6 rows over many windows), 256 of them checked completely against the oracle, as above."""
    torch, ctx, dev = world[0], world[1], world[2]
    lib = ctx.lib
    store, blob_full, offsets, lens, h_gt = heavy_tail_world(torch, ctx, dev)
    G = _native.BLOB_GUARD
    try:
        starts_gt = np.searchsorted(h_gt, np.arange(1, 1_000_002, dtype=np.int64), side="left")
        rng = np.random.Generator(np.random.PCG64(5))
        cap = BloomFilter(10160, 0.01).get_capacity(0.01)
        modulo_m = int(math.ceil(N / float(cap)))
        reqs = (_native.Request * R)()
        claims, raws, off = [], [], 0
        for i in range(R):
            if i % 2 == 0:
                a = int(rng.integers(0, N))
                lo, hi = int(h_gt[a]), int(h_gt[min(a + cap - 1, N - 1)])
                modulo, offset = 1, 0
                rows = np.arange(starts_gt[lo - 1], starts_gt[hi], dtype=np.int64)
            else:
                lo, hi, modulo = 1, 1_000_000, modulo_m
                offset = int(rng.integers(0, modulo))
                first = (modulo - offset) % modulo or modulo
                gs = np.arange(first, 1_000_001, modulo, dtype=np.int64)
                rows = np.concatenate([np.arange(starts_gt[x - 1], starts_gt[x], dtype=np.int64) for x in gs])
            pre = bytes([int(rng.integers(0, 256))])
            bf = BloomFilter(10160, 0.01, pre)
            known = np.ascontiguousarray(rows[rng.random(len(rows)) >= 0.01].astype(np.uint64))
            buf = ctypes.create_string_buffer(bf.bytes, len(bf.bytes))
            if len(known):
                _native.check(lib.dsy_bloom_add_rows(ctx.handle, ctypes.byref(bf.params), store, known.ctypes.data,
                                                     len(known), buf))
            raw = buf.raw + b"\x00" * ((-len(buf.raw)) % 4)
            q = reqs[i]
            q.time_low, q.time_high, q.modulo, q.offset = lo, hi, modulo, offset
            q.filter_offset, q.m_bits, q.k = off, bf.size, bf.functions
            q.hash_kind, q.chunk_bytes = _native.HASH_KINDS[bf.hash_name], bf.chunk_bytes
            q.prefix_len = 1
            q.prefix[0] = pre[0]
            claims.append((rows, bf, off, buf.raw, pre))
            raws.append(raw)
            off += len(raw)
        fblob = b"".join(raws)
        metas = (_native.Meta * 1)()
        metas[0].meta_id, metas[0].direction = 1, _native.DSY_ASC
        h_off = np.zeros(R + 1, dtype=np.uint64)
        h_idx = np.zeros(1 << 24, dtype=np.uint64)
        _native.check(lib.dsy_sync_respond(ctx.handle, store, reqs, R, fblob, len(fblob), metas, 1, 1_000_000, 0,
                                           LIMIT, 99, h_idx.ctypes.data, len(h_idx), h_off.ctypes.data))
        # the oracle over 256 of the claims (both styles: i % 8 in {0, 1}); the saturated largest-style ones walk
        # 10^5-10^6 rows with hashlib
        pick = [i for i in range(R) if i % 8 in (0, 1)]
        rows = np.unique(np.concatenate([claims[i][0] for i in pick]))
        packets, poff = gather_rows(torch, dev, blob_full[G:], offsets, rows)
        want = check_claims([(int(reqs[i].time_low), int(reqs[i].time_high), int(reqs[i].offset), int(reqs[i].modulo),
                              claims[i][3], claims[i][1].functions, claims[i][4]) for i in pick], packets, poff, rows,
                            h_gt.astype(np.uint64), 1_000_000, LIMIT, work=[len(claims[i][0]) for i in pick])
        del packets
        sent = 0
        for j, i in enumerate(pick):
            got = h_idx[h_off[i]:h_off[i + 1]].astype(np.int64).tolist()
            assert got == want[j], (i, len(got), len(want[j]))
            sent += len(got)
        assert sent > 0 and len(pick) == 256
    finally:
        lib.dsy_store_free(store)
        del blob_full, offsets
        torch.cuda.empty_cache()

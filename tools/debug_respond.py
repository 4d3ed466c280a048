#!/usr/bin/env python3
"""Debug aid (not part of the product): the bench's responder claims at a small store size, GPU (dsy_sync_respond)
against the oracle claim by claim, for a few filter shapes; prints the first mismatches."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    import torch
    import bench
    from dispersy_amd import _native
    from oracle import sync_ref
    from oracle.bloom_ref import OracleBloom
    N = int(os.environ.get("N", "300000"))
    R = int(os.environ.get("R", "128"))
    dev = torch.device("cuda", 0)
    ctx = _native.Context(0)
    lib = ctx.lib
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    lengths = torch.randint(100, 1501, (N,), device=dev, generator=g, dtype=torch.int64)
    offsets = torch.zeros(N + 1, device=dev, dtype=torch.int64)
    torch.cumsum(lengths, 0, out=offsets[1:])
    total = int(offsets[-1].item())
    blob_full = torch.randint(0, 256, (total + 2 * _native.BLOB_GUARD,), device=dev, generator=g, dtype=torch.uint8)
    blob = blob_full[_native.BLOB_GUARD:]
    gt = torch.arange(1, N + 1, device=dev, dtype=torch.int64)
    meta = torch.ones(N, device=dev, dtype=torch.int32)
    torch.cuda.synchronize()
    store = ctypes.c_void_p()
    _native.check(lib.dsy_store_attach(ctx.handle, blob.data_ptr(), total, offsets.data_ptr(), N, gt.data_ptr(),
                                       meta.data_ptr(), None, ctypes.byref(store)))
    host_blob = memoryview(blob[:total].cpu().numpy())
    host_off = offsets.cpu().numpy()
    rows = np.arange(N, dtype=np.int64)
    gts = np.arange(1, N + 1, dtype=np.uint64)
    metas = [dict(name="bench", id=1, direction="ASC", priority=128, pruning=None)]
    packet_of = lambda r: host_blob[int(host_off[r]):int(host_off[r + 1])]  # noqa: E731
    for bits, f, prefix in [(10160, 0.01, None), (4096, 0.001, b"x"), (4096, 0.001, None), (10160, 0.01, b"x")]:
        rng = np.random.Generator(np.random.PCG64(8))
        reqs, claims, fblob, d_filters, capacity = bench.make_claims(ctx, lib, store, N, R, rng, bits, f, prefix, dev)
        out_off = np.zeros(R + 1, dtype=np.uint64)
        out = np.zeros(1 << 22, dtype=np.uint64)
        _native.check(lib.dsy_sync_respond(ctx.handle, store, reqs, R, fblob, len(fblob),
                                           (_native.Meta * 1)(_native.Meta(1, 0, 0, 0, 0)), 1, N, 0, 5120, 99,
                                           out.ctypes.data, len(out), out_off.ctypes.data))
        bad = 0
        for i in range(R):
            lo, hi, offset, modulo, kf, pre, raw = claims[i]
            ob = OracleBloom.from_bytes(raw, kf, pre)
            want = sync_ref.respond_arrays(packet_of, {1: (rows, gts)}, metas, (lo, hi, offset, modulo), ob, N, 5120)
            got = out[int(out_off[i]):int(out_off[i + 1])].tolist()
            if got != want:
                bad += 1
                if bad <= 3:
                    print("MISMATCH bits=%d f=%g prefix=%r claim %d lo=%d hi=%d off=%d mod=%d k=%d pre=%r" %
                          (bits, f, prefix, i, lo, hi, offset, modulo, kf, pre))
                    print("  gpu", got[:12], len(got))
                    print("  cpu", want[:12], len(want))
                    extra = sorted(set(got) - set(want))[:5]
                    for r in extra:
                        print("  gpu-only row", r, "in oracle filter:", bytes(packet_of(r)) in ob, "len", len(packet_of(r)))
        print("bits=%d f=%g prefix=%r: %d/%d claims differ" % (bits, f, prefix, bad, R), flush=True)


if __name__ == "__main__":
    main()

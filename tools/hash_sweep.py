#!/usr/bin/env python3
"""Single-filter hashing kernels in isolation (not part of the product): N packets (100-1500 B, seed 1234) generated
in HBM, then dsy_bloom_add_dev / dsy_bloom_test_dev for the MD5 MTU filter and the SHA-1 test-harness filter
(node.py:617), timed with the ctx's HIP events.  Prints Gblk/s and the INT32 VALU fraction per kernel, one JSON line.
Meant to run under rocprofv3 (kernel trace or one --pmc pass at a time).

usage: python tools/hash_sweep.py [--packets N] [--reps R] [--families md5,sha1,sha256] [--ops test,add]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

OPS_PER_BLOCK = {"md5": 500, "sha1": 961, "sha256": 2168}
PEAK_INT32_TOPS = 78.64
FILTERS = {"md5": (10160, 0.01, b"\x00\x01\x02\x03"), "sha1": (4096, 0.001, b"x"), "sha256": (1 << 20, 0.01, b"\x07")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--families", default="md5,sha1")
    ap.add_argument("--ops", default="test,add")
    ap.add_argument("--lo", type=int, default=100)
    ap.add_argument("--hi", type=int, default=1500)
    args = ap.parse_args()
    import torch
    from dispersy_amd import _native
    from dispersy_amd.bloomfilter import BloomFilter
    dev = torch.device("cuda", 0)
    ctx = _native.Context(0)
    lib = ctx.lib
    N = args.packets
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    lengths = torch.randint(args.lo, args.hi + 1, (N,), device=dev, generator=g, dtype=torch.int64)
    offsets = torch.zeros(N + 1, device=dev, dtype=torch.int64)
    torch.cumsum(lengths, 0, out=offsets[1:])
    total = int(offsets[-1].item())
    G = _native.BLOB_GUARD
    blob_full = torch.randint(0, 256, (total + 2 * G,), device=dev, generator=g, dtype=torch.uint8)
    blob = blob_full[G:]
    present = torch.empty(N, dtype=torch.uint8, device=dev)
    out = {"packets": N, "bytes": total}
    for fam in args.families.split(","):
        m, f, prefix = FILTERS[fam]
        bf = BloomFilter(m, f, prefix)
        blk, lb = (64, 8)
        blocks = int(((lengths + len(prefix) + lb) // blk + 1).sum().item())
        filt = torch.zeros(int(lib.dsy_filter_words(m)), dtype=torch.int32, device=dev)
        n_add = min(N, 100_000) if "add" not in args.ops else N
        for op in args.ops.split(","):
            def run():
                if op == "add":
                    _native.check(lib.dsy_bloom_add_dev(ctx.handle, ctypes.byref(bf.params), blob.data_ptr(),
                                                        offsets.data_ptr(), n_add, filt.data_ptr()))
                else:
                    _native.check(lib.dsy_bloom_test_dev(ctx.handle, ctypes.byref(bf.params), blob.data_ptr(),
                                                         offsets.data_ptr(), N, filt.data_ptr(), present.data_ptr()))
            run()
            ctx.synchronize()
            ctx.reset_timing()
            ctx.set_timing(True, only=[_native.TIME_BLOOM])
            t0 = time.perf_counter()
            for _ in range(args.reps):
                run()
            ctx.synchronize()
            wall = (time.perf_counter() - t0) / args.reps
            ctx.set_timing(False)
            kt = ctx.kernel_time(_native.TIME_BLOOM)
            secs = kt["ms"] / 1e3 / max(kt["launches"], 1)
            nb = blocks if op == "test" or n_add == N else None
            out["%s_%s" % (fam, op)] = {
                "kernel_ms": round(secs * 1e3, 3), "wall_ms": round(wall * 1e3, 3),
                "gblocks_per_s": round(nb / secs / 1e9, 2) if nb else None,
                "valu_frac": round(nb * OPS_PER_BLOCK[fam] / secs / 1e12 / PEAK_INT32_TOPS, 4) if nb else None,
                "hbm_gbs": round((total + 17 * N) / secs / 1e9, 1) if nb else None}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""BASELINE config 1 at ONE size, for same-box A/B runs and PMC passes whose per-dispatch averages are not a mix of
sizes: the config-2 store's packets (seed 1234, 100-1500 B, packed in HBM as bench.py builds them),
BloomFilter(10160, 0.01, 4-byte prefix) (MD5) or the reference's test filter BloomFilter(4096, 0.001, "x") (SHA-1,
tests/debugcommunity/node.py:617); add --adds keys, then test all --n keys --reps times.

Every staging variant named in --lines (DSY_BLOOM_LINES values, read when a ctx is created) runs on its own ctx in
this process; their membership bytes must be identical, and the first variant's are checked against the oracle on a
sample (hashlib, oracle/bloom_ref).  Prints one JSON line.

usage: python tools/cfg1_run.py --family md5 --n 10000000 --reps 5 --lines 3,0
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--family", default="md5", choices=["md5", "sha1"])
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--adds", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--lines", default="3,0", help="comma-separated DSY_BLOOM_LINES values, one ctx each")
    ap.add_argument("--check", type=int, default=20_000, help="keys checked against the oracle (0: none)")
    args = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from dispersy_amd import _native
    from dispersy_amd.bloomfilter import BloomFilter
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    N = args.n
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    lengths = torch.randint(100, 1501, (N,), device=dev, generator=g, dtype=torch.int64)
    offsets = torch.zeros(N + 1, device=dev, dtype=torch.int64)
    torch.cumsum(lengths, 0, out=offsets[1:])
    total = int(offsets[-1].item())
    blob_full = torch.randint(0, 256, (total + 2 * _native.BLOB_GUARD,), device=dev, generator=g, dtype=torch.uint8)
    blob = blob_full[_native.BLOB_GUARD:]
    m, f, prefix = {"md5": (10160, 0.01, b"\x00\x01\x02\x03"), "sha1": (4096, 0.001, b"x")}[args.family]
    out = {"family": args.family, "keys": N, "adds": args.adds, "key_bytes": total, "runs": []}
    blocks = bench._blocks(lengths, len(prefix), args.family)
    ref = None
    for lines in args.lines.split(","):
        os.environ["DSY_BLOOM_LINES"] = lines
        ctx = _native.Context(0)
        lib = ctx.lib
        bf = BloomFilter(m, f, prefix)
        filt = torch.zeros(int(lib.dsy_filter_words(m)), dtype=torch.int32, device=dev)
        present = torch.empty(N, dtype=torch.uint8, device=dev)
        add = lambda: _native.check(lib.dsy_bloom_add_dev(ctx.handle, ctypes.byref(bf.params), blob.data_ptr(),  # noqa: E731
                                                          offsets.data_ptr(), args.adds, filt.data_ptr()))
        test = lambda: _native.check(lib.dsy_bloom_test_dev(ctx.handle, ctypes.byref(bf.params), blob.data_ptr(),  # noqa: E731
                                                            offsets.data_ptr(), N, filt.data_ptr(), present.data_ptr()))
        ctx.wait_torch(dev)
        add()
        test()
        k_add, _ = bench._timed_bloom(ctx, add, 3)
        k_test, wall = bench._timed_bloom(ctx, test, args.reps)
        got = present.cpu().numpy()
        fb = filt.cpu().numpy().tobytes()
        same = None
        if ref is None:
            ref = (got, fb)
        else:
            same = bool((got == ref[0]).all() and fb == ref[1])
        rec = {"lines": lines, "test_us": round(k_test * 1e6, 1), "add_us": round(k_add * 1e6, 1),
               "test_keys_per_s": round(N / k_test, 1), "test_wall_keys_per_s": round(N / wall, 1),
               "hbm_alg_tbs": round((total + 17 * N) / k_test / 1e12, 3),
               "int32_frac": round(blocks * bench.OPS_PER_BLOCK[args.family] / k_test / 1e12 / bench.PEAK_INT32_TOPS, 4),
               "present_fraction": round(float(got.mean()), 4), "same_as_first": same}
        if args.check and same is None:
            chk_bf = BloomFilter(m, f, prefix)
            rec["gpu_vs_oracle"] = bench.bloom_vs_oracle(ctx, lib, chk_bf, m, f, prefix, blob, offsets, args.check,
                                                         offsets, min(N, 5 * args.check), dev)
        out["runs"].append(rec)
        ctx.synchronize()
        del ctx
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

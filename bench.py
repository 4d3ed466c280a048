#!/usr/bin/env python3
"""Benchmark of the Bloom-filter sync hot path on MI355X (BASELINE.json configs[1]).

Workload (one step): ONE responder peer holding 10 M stored packets (100-1500 B, global_time 1..N) answers a batch
of 1024 incoming claims -- 512 "largest"-style (modulo 1, a window of ~capacity global times) and 512
"modulo"-style (modulo = ceil(N / capacity), random offset) -- each carrying an MTU bloom filter
(m = 10160, f = 0.01 -> MD5, k = 7, 1-byte prefix) built from the requester's copy of its range with 1 % of the
packets withheld.  The step is the whole batched responder: selection, prefix-salted digest + probe of every
selected packet, byte-limited (5 KiB) compaction -- dsy_sync_respond_dev through the C-ABI.  Packets are
resident in HBM before the timed region.

value = (claim, packet) pairs hashed+tested per second over all ranks.  With N GPUs each rank serves its own
1024 claims against a replica of the store (claims shard, no data-path collective): weak scaling.

Launch:  python bench.py [--gpus N --steps K --warmup W]
     or  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PEAK_INT32_TOPS = 78.64        # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz: one 32-bit VALU op per lane per clock
OPS_PER_BLOCK = {"md5": 500, "sha1": 961, "sha256": 2168, "sha384": 5504, "sha512": 5504}  # SURVEY §8d canonical


# ------------------------------------------------------------------------------------------- CPU legs
def cpu_info():
    """(CPU model, cores this process may use).  On the GPU box the affinity mask shows the whole machine; the
    box's share is OMP_NUM_THREADS (16 per GPU), so that caps the worker count (N = the cores the
    job may use)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    avail = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS") or avail)
    return model, max(1, min(avail, share))


# ------------------------------------------------------------------- the CPU worker pool (forked before any GPU use)
class Shared(object):
    """A read-only numpy array in a file under /dev/shm: it pickles as the file's path, so a pool task attaches to
    it (np.memmap) instead of receiving a copy.  The creating process unlinks the files at exit (Shared.cleanup)."""
    _mine = []

    def __init__(self, arr):
        import tempfile
        base = "/dev/shm" if os.access("/dev/shm", os.W_OK) else None
        fd, self.path = tempfile.mkstemp(prefix="dsy_bench_", suffix=".bin", dir=base)
        arr = np.ascontiguousarray(arr)
        with os.fdopen(fd, "wb") as f:
            f.write(memoryview(arr).cast("B") if arr.size else b"")
        self.dtype, self.shape = arr.dtype.str, arr.shape
        self.a = arr
        Shared._mine.append(self.path)

    def __reduce__(self):
        return (_attach_shared, (self.path, self.dtype, self.shape))

    @classmethod
    def cleanup(cls):
        for p in cls._mine:
            try:
                os.unlink(p)
            except OSError:
                pass
        cls._mine = []


class _Attached(object):
    def __init__(self, a):
        self.a = a


def _attach_shared(path, dtype, shape):
    n = int(np.prod(shape)) if shape else 1
    if n == 0:
        return _Attached(np.zeros(shape, dtype=np.dtype(dtype)))
    return _Attached(np.memmap(path, dtype=np.dtype(dtype), mode="r", shape=shape))


def _pool_task(payload):
    """One pool task: (fn, shard) pickled with cloudpickle (closures included).  fn returns the units done, or
    (units, seconds) when it times its own measured part after a private, untimed setup."""
    import cloudpickle
    fn, shard = cloudpickle.loads(payload)
    t0 = time.perf_counter()
    r = fn(shard)
    return r if isinstance(r, tuple) else (r, time.perf_counter() - t0)


def _pool_call(payload):
    import cloudpickle
    fn, item = cloudpickle.loads(payload)
    return fn(item)


class CpuPool(object):
    """The N-core CPU legs' workers.  They are forked at start-up, before torch is imported or HIP is touched, so
    no worker inherits device files or GPU runtime state; tasks reach them as cloudpickle payloads (large arrays as
    `Shared` files), and they are shut down with close + join (no SIGTERM: a profiler's signal handler in a worker
    would turn that into an abort)."""

    def __init__(self, n):
        import multiprocessing as mp
        self.n = n
        self.pool = mp.get_context("fork").Pool(n)

    def run(self, fn, shards):
        """fn(shard) for every shard at once (len(shards) <= n); returns (units, wall seconds of the slowest)."""
        import cloudpickle
        if len(shards) > self.n:
            raise ValueError("%d shards for %d workers" % (len(shards), self.n))
        res = self.pool.map(_pool_task, [cloudpickle.dumps((fn, s)) for s in shards], chunksize=1)
        return sum(u for u, _ in res), max(t for _, t in res)

    def map(self, fn, items):
        """[fn(item) for item in items] on the workers (the heaviest items first is the caller's choice)."""
        import cloudpickle
        return self.pool.map(_pool_call, [cloudpickle.dumps((fn, it)) for it in items], chunksize=1)

    def close(self):
        self.pool.close()
        self.pool.join()


POOL = None  # the CpuPool of this run (rank 0 at N = 1 with CPU legs), or None


def n_core_leg(fn, shards, unit, sample):
    model, _ = cpu_info()
    if POOL is None:
        return None
    units, secs = POOL.run(fn, shards)
    return {"value": round(units / secs, 1), "unit": unit, "cores": len(shards), "cpu_model": model,
            "sample": sample, "seconds": round(secs, 2),
            "workers": "forked before the first GPU call (CpuPool), one per core of the job's share"}


# ------------------------------------------------------------------------------------- N ranks from one command
def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """`python bench.py --gpus N` without a launcher: start N ranks (one process per GPU) through
    torch.distributed.run as a CHILD process and return its exit code.  This process has not touched the GPU
    (nothing is imported but argparse/numpy) and it never exec's; the ranks find WORLD_SIZE = N in their env."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--packets", type=int, default=10_000_000)
    ap.add_argument("--claims", type=int, default=1024)
    ap.add_argument("--filter-bits", type=int, default=10160)
    ap.add_argument("--error-rate", type=float, default=0.01)
    ap.add_argument("--byte-limit", type=int, default=5120)
    ap.add_argument("--cpu-claims", type=int, default=1, help="0: skip the CPU-baseline legs (and the CPU pool)")
    ap.add_argument("--cpu-pairs", type=int, default=100_000,
                    help="responder CPU baselines: (claim, packet) pairs hashed in the 1-core sample (BASELINE.md:47)")
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--pipeline", type=int, default=3,
                    help="responder legs: batches in flight (dsy_sync_respond_submit / _wait, at most 3); 1 one at a time "
                         "(dsy_sync_respond_dev)")
    ap.add_argument("--pipeline5", type=int, default=1,
                    help="config 5 (heavy tail): batches in flight. Default 1: its calls walk 9 windows each, and "
                         "batches in flight interleave their windows on the stream (each window waits for the host "
                         "to read the previous one's flags), which measured 1-2 %% slower than one call at a time "
                         "(profiles/bulk_parts_ab_r5.json: ms_per_step 3 in flight vs serial_ms_per_step)")
    ap.add_argument("--window", type=int, default=0, help="cap on the responder's window (pairs per claim; 0: default)")
    ap.add_argument("--sim-peers", type=int, default=1_000_000, help="config 3 gossip simulator peers (0: skip)")
    ap.add_argument("--sim-universe", type=int, default=10_000)
    ap.add_argument("--sim-initial", type=int, default=100)
    ap.add_argument("--sim-rounds", type=int, default=10)
    ap.add_argument("--sim-warmup", type=int, default=2)
    ap.add_argument("--sim-chunks", type=int, default=0,
                    help="config 3: each rank's peers in this many chunks, exchanges overlapped with the kernels "
                         "(EpidemicSim.chunks); 0: 4 with more than one rank, else 1 (one rank exchanges nothing)")
    ap.add_argument("--extra", default="claim,dropin,dedup,ingest,sha1,1,3,4,5",
                    help="BASELINE configs measured beside the headline (config 2): 1 single filter, 3 gossip "
                         "simulator, 4 large filters, 5 heavy-tailed packets, ingest: received packets appended to "
                         "the headline store, dedup: duplicate check of received packets against it, claim: modulo and "
                         "largest claims built over it on the device, dropin: SyncCommunity.respond / store_messages "
                         "over it (host buffers); '' for none")
    ap.add_argument("--large-keys", type=int, default=100_000_000, help="config 4: keys added per filter")
    ap.add_argument("--large-tests", type=int, default=10_000_000, help="config 4: keys tested per filter")
    return ap.parse_args()


def main():
    global POOL
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print("bench.py: %d ranks were launched for --gpus %d; refusing to report a wrong n_gpus" % (world, args.gpus),
              file=sys.stderr)
        sys.exit(2)
    if os.environ.get("DSY_BENCH_PROBE"):  # launcher test (tests/test_bench_launch.py): report and stop, no GPU
        print(json.dumps({"probe": True, "rank": rank, "world": world, "local_rank": local, "gpus": args.gpus}))
        return
    if rank == 0 and world == 1 and args.cpu_claims > 0:
        POOL = CpuPool(cpu_info()[1])  # before torch / HIP: the workers inherit no GPU state
    try:
        run(args, rank, world, local)
    finally:
        if POOL is not None:
            POOL.close()
        Shared.cleanup()


def run(args, rank, world, local):
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        # DSY_DIST_BACKEND=gloo rehearses the N > 1 path with several ranks on fewer GPUs (the collectives then
        # stage through host memory, dispersy_amd/shard.py); the driver's multi-GPU runs use RCCL
        torch.cuda.set_device(local % max(torch.cuda.device_count(), 1))
        dist.init_process_group(os.environ.get("DSY_DIST_BACKEND", "nccl"))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from dispersy_amd import _native
    from dispersy_amd.bloomfilter import BloomFilter
    from dispersy_amd.shard import Collectives

    ctx = _native.Context(torch.cuda.current_device())
    lib = ctx.lib
    N, R = args.packets, args.claims

    # ---------------------------------------------------------------- the store, generated in HBM (seed 1234)
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    lengths = torch.randint(100, 1501, (N,), device=dev, generator=g, dtype=torch.int64)
    offsets = torch.zeros(N + 1, device=dev, dtype=torch.int64)
    torch.cumsum(lengths, 0, out=offsets[1:])
    total_bytes = int(offsets[-1].item())
    # DSY_BLOB_GUARD readable bytes before the first and after the last packet (include/dsybloom.h)
    blob_full = torch.randint(0, 256, (total_bytes + 2 * _native.BLOB_GUARD,), device=dev, generator=g, dtype=torch.uint8)
    blob = blob_full[_native.BLOB_GUARD:]
    gt = torch.arange(1, N + 1, device=dev, dtype=torch.int64)
    meta = torch.ones(N, device=dev, dtype=torch.int32)
    torch.cuda.synchronize()
    store = ctypes.c_void_p()
    _native.check(lib.dsy_store_attach(ctx.handle, blob.data_ptr(), total_bytes, offsets.data_ptr(), N, gt.data_ptr(),
                                       meta.data_ptr(), None, ctypes.byref(store)))

    # ---------------------------------------------------------------- the claims (seed 7 + rank)
    rng = np.random.Generator(np.random.PCG64(args.seed + 1000 * rank))
    reqs, claims, fblob, d_filters, capacity = make_claims(ctx, lib, store, N, R, rng, args.filter_bits,
                                                           args.error_rate, None, dev)
    cap_probe = BloomFilter(args.filter_bits, args.error_rate)
    metas = (_native.Meta * 1)()
    metas[0].meta_id, metas[0].direction = 1, _native.DSY_ASC

    if args.window:
        ctx.set_window(args.window)
    batches = Batches(lib, ctx, store, reqs, R, d_filters.data_ptr(), metas, 1, N, args.byte_limit)
    pipe = args.pipeline
    step = batches.step

    batches.run(args.warmup, pipe)
    ctx.synchronize()
    ctx.reset_timing()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    total_pairs = batches.run(args.steps, pipe)
    ctx.synchronize()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    work = ctx.work(_native.TIME_PAIR_TEST)
    # the dominant kernel's launches timed by HIP events in a serial pass (one batch at a time: with two batches in
    # flight a launch's events would also span the other batch's kernels), then the selection / compaction kernels'
    # times from a few more steps; all outside the timed region
    ctx.reset_timing()
    ctx.set_timing(True, only=[_native.TIME_PAIR_TEST])
    t1 = time.perf_counter()
    serial_pairs = batches.run(args.steps, 1)
    serial_s = time.perf_counter() - t1
    ctx.set_timing(False)
    kt = ctx.kernel_time(_native.TIME_PAIR_TEST)
    ctx.reset_timing()
    ctx.set_timing(True, only=[_native.TIME_SELECT, _native.TIME_COMPACT])
    n_side = min(max(args.steps, 1), 5)
    batches.run(n_side, 1)
    ctx.synchronize()
    ctx.set_timing(False)
    sel = ctx.kernel_time(_native.TIME_SELECT)
    cmp_ = ctx.kernel_time(_native.TIME_COMPACT)
    if dist:
        coll = Collectives(dist)
        elapsed = float(coll.scalar(elapsed, "max", device=dev))
        total_pairs = int(coll.scalar(int(total_pairs), "sum", device=dev))
        serial_s = float(coll.scalar(serial_s, "max", device=dev))

    # ---------------------------------------------------------------- roofline of the dominant kernel
    launches = max(kt["launches"], 1)
    avg_s = kt["ms"] / 1e3 / launches
    pairs_per_launch = serial_pairs / max(args.steps, 1)
    blocks_per_launch = kt["blocks"] / launches
    bytes_per_launch = kt["bytes"] / launches + pairs_per_launch * 17  # packet bytes + 16 B task record + miss flag
    hash_name = cap_probe.hash_name
    hbm_frac = bytes_per_launch / avg_s / 1e9 / PEAK_HBM_GBS
    valu_frac = blocks_per_launch * OPS_PER_BLOCK[hash_name] / avg_s / 1e12 / PEAK_INT32_TOPS
    roofline = {
        "kernel": "k_pair_test<%s>" % hash_name,
        # the binding roof is the one the kernel is closer to (the other view is under valu_int32)
        "bound": "hbm" if hbm_frac >= valu_frac else "valu",
        "bound_rule": "the larger of the HBM and INT32-VALU fractions",
        "achieved": round(bytes_per_launch / avg_s / 1e9, 1) if hbm_frac >= valu_frac
        else round(valu_frac * PEAK_INT32_TOPS, 2),
        "peak": PEAK_HBM_GBS if hbm_frac >= valu_frac else PEAK_INT32_TOPS,
        "unit": "GB/s" if hbm_frac >= valu_frac else "Tops/s",
        "frac": round(max(hbm_frac, valu_frac), 4),
        "hbm_gbs": round(bytes_per_launch / avg_s / 1e9, 1),
        "traffic": None,
        "avg_launch_us": round(avg_s * 1e6, 2),
        "launches": kt["launches"],
        "valu_int32": {
            "achieved": round(blocks_per_launch * OPS_PER_BLOCK[hash_name] / avg_s / 1e12, 2),
            "peak": PEAK_INT32_TOPS, "unit": "Tops/s",
            "frac": round(blocks_per_launch * OPS_PER_BLOCK[hash_name] / avg_s / 1e12 / PEAK_INT32_TOPS, 4),
            "ops_per_block": OPS_PER_BLOCK[hash_name], "blocks_per_launch": int(blocks_per_launch)},
        "other_kernels_ms_per_step": {"select": round(sel["ms"] / n_side, 3),
                                      "compact": round(cmp_["ms"] / n_side, 3)},
    }
    # HBM traffic per launch from the committed PMC passes (tools/profile_round.sh -> profiles/pmc_traffic_<hash>.json),
    # reported only when the kernel it measured is the one this run executes: the file carries the sha256 of the
    # kernel's machine code in the library it profiled (tools/kernel_hash.py), compared with this library's
    traffic_file = os.path.join(ROOT, "profiles", "pmc_traffic_%s.json" % hash_name)
    if os.path.isfile(traffic_file):
        from tools.kernel_hash import HEADLINE, kernel_sha
        with open(traffic_file) as f:
            rec = json.load(f)
        now = kernel_sha(_native.LIB_PATH if not os.environ.get("DSY_LIB_PATH") else os.environ["DSY_LIB_PATH"],
                         HEADLINE) if hash_name == "md5" else None
        if now is not None and rec.get("kernel_sha") == now:
            roofline["traffic"] = rec.get("hbm_bytes_per_launch")
            roofline["traffic_source"] = "profiles/pmc_traffic_%s.json (%s; same kernel code, sha256 %s)" % (
                hash_name, rec.get("round"), now[:16])
        else:
            roofline["traffic_source"] = "not reported: profiles/pmc_traffic_%s.json measured another build of the " \
                                         "kernel (sha256 %s, this run %s)" % (hash_name, str(rec.get("kernel_sha"))[:16],
                                                                            str(now)[:16])

    # `work` was read right after the timed steps (reset before them)
    useful = work["useful_pairs"]
    roofline["lane_utilization"] = round(work["blocks"] / max(work["lane_slots"], 1), 4)
    if dist:
        useful = int(coll.scalar(int(useful), "sum", device=dev))

    cpu = None
    if rank == 0 and world == 1 and args.cpu_claims > 0:
        # (every 8th claim of the step, both styles, also checked in full against the oracle: 128 claims; the
        # test suite's test_fullsize_gpu.py checks all 1024)
        cpu = responder_cpu(args, ctx, lib, store, reqs, claims, fblob, blob, offsets,
                            np.arange(1, N + 1, dtype=np.uint64), N, dev, "cfg2 md5", check=list(range(0, R, 8)))

    extra = set(x for x in args.extra.split(",") if x and x != "none")

    # before the legs that append to the store (dropin, dedup, ingest): its CPU check reads the store as generated
    sha1 = None
    if "sha1" in extra:
        sha1 = sha1_respond(args, ctx, lib, store, N, dev, blob, offsets, total_bytes, metas, rank, world, dist)

    ingest = None
    dedup = None
    claim = None
    dropin = None
    if "claim" in extra:
        claim = claim_bench(args, ctx, lib, store, N, capacity, total_bytes / N, cpu_leg=rank == 0 and world == 1)
    if "dropin" in extra:
        dropin = dropin_bench(args, ctx, lib, store, offsets, N, claims)
    if "dedup" in extra:
        dedup = dedup_bench(args, ctx, lib, store, blob, offsets, N, cpu_leg=rank == 0 and world == 1)
    if "ingest" in extra:
        ingest = ingest_bench(args, ctx, lib, store, step, N, cpu_leg=rank == 0 and world == 1)

    gossip = None
    if "3" in extra and args.sim_peers > 0:
        gossip = gossip_sim(args, ctx, dev, rank, world, dist)
    single = large = heavy = None
    if "1" in extra:
        single = single_filter(args, ctx, lib, blob, offsets, N, dev, rank, world)
    if "5" in extra:
        heavy = heavy_tail(args, ctx, lib, dev, rank, world, dist)
    if "4" in extra:
        lib.dsy_store_free(store)
        store = None
        del blob_full, blob, offsets, gt, meta, d_filters
        torch.cuda.empty_cache()
        large = large_filter(args, ctx, lib, dev, rank, world, dist)


    if rank == 0:
        line = {
            "metric": "packets hashed+tested/sec",
            "value": round(useful / elapsed, 1),
            "unit": "packets/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": {"workload": "cfg2: one responder, %d stored packets (100-1500 B) x %d claims per GPU "
                                   "(half largest-style, half modulo-style), m=%d f=%g (%s k=%d), %d B byte limit"
                                   % (N, R, args.filter_bits, args.error_rate, hash_name, cap_probe.functions,
                                      args.byte_limit),
                       "stored_packets": N, "claims_per_gpu": R, "pairs_per_step_per_gpu": int(pairs_per_launch),
                       "parallelism": "claims sharded over %d GPU(s), store replicated" % world},
            "value_counts": "(claim, packet) pairs the reference hashes+tests for these claims: its lazy not_filter "
                            "stops at the packet that spends the 5 KiB budget (community.py:2559-2567)",
            "pairs_hashed_per_s": round(total_pairs / elapsed, 1),
            "pipeline": "%d batches in flight (dsy_sync_respond_submit / _wait): one batch's selection, another's "
                        "compaction and the host's staging overlap the hashing" % pipe if pipe > 1
                        else "one batch at a time (dsy_sync_respond_dev)",
            "serial_ms_per_step": round(serial_s / max(args.steps, 1) * 1e3, 3),
            "claims_per_s": round(R * world * args.steps / elapsed, 1),
            "roofline": roofline,
            "cpu_baseline": cpu,
            "gossip_sim": gossip,
            "single_filter": single,
            "large_filter": large,
            "heavy_tail": heavy,
            "ingest": ingest,
            "dedup": dedup,
            "claim_modulo": claim,
            "dropin": dropin,
            "sha1_respond": sha1,
        }
        line.update(tail_keys(gossip, sha1, heavy, single, large, cpu))
        print(json.dumps(line))
    if store is not None:
        lib.dsy_store_free(store)
    if dist:
        dist.destroy_process_group()


def _get(d, *path):
    for k in path:
        if not isinstance(d, dict) or k not in d:
            return None
        d = d[k]
    return d


def _ok(chk):
    """True / False for a gpu_vs_oracle record (None when the check did not run)."""
    if not isinstance(chk, dict):
        return None
    return bool(chk.get("filter_bytes_equal")) and bool(chk.get("membership_equal"))


def tail_keys(gossip, sha1=None, heavy=None, single=None, large=None, cpu=None):
    """Compact top-level keys printed LAST on the JSON line, so a driver that keeps only the tail of stdout still
    sees BASELINE's second metric (gossip sync rounds/s at N GPUs, config 3) and each leg's headline number.  The
    nested legs above hold the same values with their rooflines and CPU baselines."""
    out = {
        "gossip_n_gpus": _get(gossip, "n_gpus") if gossip else None,
        "gossip_rounds_per_s": _get(gossip, "value"),
        "gossip_ms_per_round": _get(gossip, "ms_per_round"),
        "gossip_store_checksum": _get(gossip, "store_checksum"),
        "gossip_scaling": _get(gossip, "scaling"),
        "sha1_respond_int32_frac": _get(sha1, "roofline", "frac"),
        "sha1_respond_ms_per_step": _get(sha1, "ms_per_step"),
        "cfg5_ms_per_step": _get(heavy, "ms_per_step"),
        "cfg5_hbm_frac": _get(heavy, "roofline", "hbm", "frac"),
        "cfg1_sha1_int32_frac": _get(single, "sha1", "roofline_test", "valu_int32", "frac"),
        "cfg4_sha256_add_int32_frac": {k: v.get("add_valu_frac") for k, v in (_get(large, "filters") or {}).items()}
        or None,
        "cfg1_at_capacity_md5_tests_per_s": _get(single, "md5", "at_capacity", "test_keys_per_s"),
    }
    # (ahead of the gossip keys: the driver's tail of stdout keeps the last few hundred characters)
    out = dict({"cfg2_cpu_1core_pairs_per_s": _get(cpu, "value"),
                "cfg2_cpu_ncore": {"value": _get(cpu, "n_core", "value"), "cores": _get(cpu, "n_core", "cores"),
                                   "unit": _get(cpu, "n_core", "unit")} if _get(cpu, "n_core") else None}, **out)
    # every in-leg GPU == CPU-oracle check that ran (None: the leg or its check did not run)
    checks = {
        "cfg2_responder_sample": _get(cpu, "gpu_matches_cpu_on_sample"),
        "sha1_responder_sample": _get(sha1, "cpu_baseline", "gpu_matches_cpu_on_sample"),
        "cfg5_responder_sample": _get(heavy, "cpu_baseline", "gpu_matches_cpu_on_sample"),
        "cfg2_responder_oracle_128_claims": _get(cpu, "oracle_check", "gpu_matches_oracle"),
        "cfg1_md5": _ok(_get(single, "md5", "gpu_vs_oracle")),
        "cfg1_sha1": _ok(_get(single, "sha1", "gpu_vs_oracle")),
        "cfg1_md5_at_capacity": _ok(_get(single, "md5", "at_capacity", "gpu_vs_oracle")),
        "cfg1_sha1_at_capacity": _ok(_get(single, "sha1", "at_capacity", "gpu_vs_oracle")),
        "cfg4_2^20": _ok(_get(large, "gpu_vs_oracle_2^20")),
    }
    out["gpu_matches_oracle"] = {k: v for k, v in checks.items() if v is not None} or None
    return out


class Batches(object):
    """One batch of R claims served again and again by the responder: step() is the synchronous call
    (dsy_sync_respond_dev); run(k, pipeline) serves k batches, two in flight when pipelined (dsy_sync_respond_submit /
    dsy_sync_respond_wait: batch i+1 is staged and its first window's selection queued before batch i is waited for),
    and returns the (claim, packet) pairs hashed."""

    def __init__(self, lib, ctx, store, reqs, R, d_filters, metas, J, global_time, byte_limit, seed=99):
        self.lib, self.h = lib, ctx.handle
        self.p_out, self.p_off, self.pairs, self.ticket = (ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64(),
                                                           ctypes.c_uint64())
        self.sync_args = (ctx.handle, store, reqs, R, d_filters, metas, J, global_time, 0, byte_limit, seed,
                          ctypes.byref(self.p_out), ctypes.byref(self.p_off), ctypes.byref(self.pairs))
        self.sub_args = (ctx.handle, store, reqs, R, d_filters, metas, J, global_time, 0, byte_limit, seed,
                         ctypes.byref(self.ticket))
        self.wait_tail = (ctypes.byref(self.p_out), ctypes.byref(self.p_off), ctypes.byref(self.pairs))

    def step(self):
        _native.check(self.lib.dsy_sync_respond_dev(*self.sync_args))
        return self.pairs.value

    def submit(self):
        _native.check(self.lib.dsy_sync_respond_submit(*self.sub_args))
        return self.ticket.value

    def wait(self, ticket):
        _native.check(self.lib.dsy_sync_respond_wait(self.h, ticket, *self.wait_tail))
        return self.pairs.value

    def run(self, k, depth=2):
        """k batches, `depth` in flight (1: the synchronous call)."""
        if depth <= 1:
            return sum(self.step() for _ in range(k))
        total, pending = 0, []
        for _ in range(k):
            pending.append(self.submit())
            if len(pending) == depth:
                total += self.wait(pending.pop(0))
        for t in pending:
            total += self.wait(t)
        return total


def sha1_respond(args, ctx, lib, store, N, dev, blob, offsets, total_bytes, metas, rank, world, dist):
    """The headline step with SHA-1 claim filters: BloomFilter(512 * 8, 0.001, prefix="x") -- the filter the
    reference's own test node puts in every introduction request (tests/debugcommunity/node.py:617), k = 10, SHA-1
    '2-byte' chunks -- over the same 10 M-packet store, --claims claims (half largest-style, half modulo-style, 1 %
    of each range missing).  Roofline of k_pair_test<sha1> (INT32 VALU: 961 ops per block), the oracle on a sample
    of the claims beside it."""
    rng = np.random.Generator(np.random.PCG64(args.seed + 1 + 1000 * rank))
    R = args.claims
    reqs, claims, fblob, d_filters, capacity = make_claims(ctx, lib, store, N, R, rng, 512 * 8, 0.001, b"x", dev)
    batches = Batches(lib, ctx, store, reqs, R, d_filters.data_ptr(), metas, 1, N, args.byte_limit)
    pipe = args.pipeline
    steps = max(args.steps, 1)
    batches.run(args.warmup, pipe)
    ctx.synchronize()
    ctx.reset_timing()
    t0 = time.perf_counter()
    total = batches.run(steps, pipe)
    ctx.synchronize()
    elapsed = time.perf_counter() - t0
    work = ctx.work(_native.TIME_PAIR_TEST)
    # the kernel's launches timed by events in a serial pass (see the headline)
    ctx.reset_timing()
    ctx.set_timing(True, only=[_native.TIME_PAIR_TEST])
    t1 = time.perf_counter()
    serial_total = batches.run(steps, 1)
    serial_s = time.perf_counter() - t1
    ctx.set_timing(False)
    kt = ctx.kernel_time(_native.TIME_PAIR_TEST)
    swork = ctx.work(_native.TIME_PAIR_TEST)
    launches = max(kt["launches"], 1)
    avg_s = kt["ms"] / 1e3 / launches
    blocks = kt["blocks"] / launches
    out = {"filter": "BloomFilter(4096, 0.001, b'x'): sha1 k=10, capacity %d" % capacity, "claims": R,
           "ms_per_step": round(elapsed / steps * 1e3, 3), "serial_ms_per_step": round(serial_s / steps * 1e3, 3),
           "pipeline": pipe,
           "pairs_per_s": round(total / elapsed, 1), "useful_pairs_per_s": round(work["useful_pairs"] / elapsed, 1),
           "pairs_per_step": int(total / steps),
           "roofline": {"kernel": "k_pair_test<sha1>", "bound": "valu", "unit": "Tops/s", "peak": PEAK_INT32_TOPS,
                        "achieved": round(blocks * OPS_PER_BLOCK["sha1"] / avg_s / 1e12, 2),
                        "frac": round(blocks * OPS_PER_BLOCK["sha1"] / avg_s / 1e12 / PEAK_INT32_TOPS, 4),
                        "avg_launch_us": round(avg_s * 1e6, 2), "launches": kt["launches"],
                        "gblocks_per_s": round(blocks / avg_s / 1e9, 2),
                        "hbm_gbs": round((kt["bytes"] / launches + serial_total / steps * 17) / avg_s / 1e9, 1),
                        "lane_utilization": round(swork["blocks"] / max(swork["lane_slots"], 1), 4),
                        "measured": "HIP events around each launch in a serial pass (one batch at a time)"}}
    if rank == 0 and world == 1 and args.cpu_claims > 0:
        out["cpu_baseline"] = responder_cpu(args, ctx, lib, store, reqs, claims, fblob, blob, offsets,
                                            np.arange(1, N + 1, dtype=np.uint64), N, dev, "sha1")
    return out


def make_claims(ctx, lib, store, N, R, rng, bits, error_rate, prefix, dev):
    """R claims over the store (global time = row + 1): even ones largest-style (modulo 1, ~capacity consecutive
    global times), odd ones modulo-style (the whole store, one residue class); each filter holds its range but a
    random 1 % (the packets the requester misses).  prefix None: one random byte per claim (community.py:2549),
    else that prefix for every claim.  Returns (dsy_request array, oracle claim tuples, packed filters on the host
    and in HBM, capacity)."""
    import torch
    from dispersy_amd.bloomfilter import BloomFilter
    capacity = BloomFilter(bits, error_rate).get_capacity(error_rate)
    modulo_m = int(math.ceil(N / float(capacity)))
    reqs = (_native.Request * R)()
    filters, claims = [], []
    off = 0
    for i in range(R):
        if i % 2 == 0:  # largest-style: modulo 1, ~capacity consecutive global times
            lo = int(rng.integers(1, N - capacity + 1))
            hi, modulo, offset = lo + capacity - 1, 1, 0
            rows = np.arange(lo - 1, hi, dtype=np.uint64)
        else:  # modulo-style: the whole store, one residue class
            lo, hi, modulo = 1, N, modulo_m
            offset = int(rng.integers(0, modulo))
            first = (modulo - offset) % modulo or modulo  # smallest gt >= 1 with (gt + offset) % modulo == 0
            rows = np.arange(first, N + 1, modulo, dtype=np.uint64) - 1
        pre = bytes([int(rng.integers(0, 256))]) if prefix is None else prefix
        bf = BloomFilter(bits, error_rate, pre)
        known = rows[rng.random(len(rows)) >= 0.01]  # the requester misses 1 % of its range
        buf = ctypes.create_string_buffer(bf.bytes, len(bf.bytes))
        _native.check(lib.dsy_bloom_add_rows(ctx.handle, ctypes.byref(bf.params), store, known.ctypes.data,
                                             len(known), buf))
        raw = buf.raw + b"\x00" * ((-len(buf.raw)) % 4)
        q = reqs[i]
        q.time_low, q.time_high, q.modulo, q.offset = lo, hi, modulo, offset
        q.filter_offset, q.m_bits, q.k = off, bf.size, bf.functions
        q.hash_kind, q.chunk_bytes = _native.HASH_KINDS[bf.hash_name], bf.chunk_bytes
        q.prefix_len = len(pre)
        for j, c in enumerate(pre):
            q.prefix[j] = c
        filters.append(raw)
        claims.append((lo, hi, offset, modulo, bf.functions, pre, buf.raw))
        off += len(raw)
    fblob = b"".join(filters)
    d_filters = torch.frombuffer(bytearray(fblob + bytes(64)), dtype=torch.uint8).to(dev)
    return reqs, claims, fblob, d_filters, capacity


def dropin_bench(args, ctx, lib, store, offsets, N, claims, reps=5, batch=10_000, batches=5):
    """The drop-in surface a Dispersy caller hits, over the headline's 10 M-packet store in HBM:
    - SyncCommunity.respond: the headline's 1024 claims as ClaimRequests with BloomFilter objects -> dsy_sync_respond
      (host buffers: the filters go up the bus, the responses come back) -> per-claim row lists;
    - SyncCommunity.store_messages: batches of received messages INSERTed (SyncStore.append: O(batch) host columns,
      dsy_store_append into HBM) with the community's global time raised (Dispersy._store).
    Wall time per call, PCIe and Python included."""
    from dispersy_amd.bloomfilter import BloomFilter
    from dispersy_amd.community import ClaimRequest, SyncCommunity
    from dispersy_amd.distribution import MetaMessage, SyncDistribution
    from dispersy_amd.store import SyncStore
    lengths = (offsets[1:] - offsets[:-1]).cpu().numpy().astype(np.uint64)
    n0 = int(lib.dsy_store_rows(store))
    st = SyncStore.attach(ctx, store, np.arange(1, n0 + 1, dtype=np.uint64), np.ones(n0, dtype=np.uint32), lengths)
    com = SyncCommunity(st, [MetaMessage("bench", 1, SyncDistribution("ASC", 128))], global_time=N)
    reqs = [ClaimRequest(lo, hi, modulo, offset, BloomFilter(raw, kf, prefix))
            for lo, hi, offset, modulo, kf, prefix, raw in claims]
    com.respond(reqs, byte_limit=args.byte_limit, random_seed=99)
    times, rec_t, rows = [], [], 0
    for _ in range(max(reps, 9)):
        t0 = time.perf_counter()
        got = com.respond(reqs, byte_limit=args.byte_limit, random_seed=99)
        times.append(time.perf_counter() - t0)
        t0 = time.perf_counter()  # respond()'s host part: the claims' ranges and their filters' addresses
        SyncCommunity._claim_columns(reqs)
        rec_t.append(time.perf_counter() - t0)
        rows = sum(len(g) for g in got)
    ms = sorted(times)[len(times) // 2] * 1e3
    rec_ms = sorted(rec_t)[len(rec_t) // 2] * 1e3
    respond = {"call": "SyncCommunity.respond(1024 ClaimRequests) -> dsy_sync_respond_refs (host buffers)",
               "median_ms_per_batch": round(ms, 3), "claims_per_s": round(len(reqs) / (ms / 1e3), 1),
               "rows_returned": rows,
               "host_phases_ms": {"claim ranges + (record, filter) addresses (SyncCommunity._claim_columns)": round(rec_ms, 3),
                                  "dsy_sync_respond_refs (filter gather + upload behind the selection, device step, "
                                  "result download)": round(ms - rec_ms, 3)}}

    class Dist(object):
        def __init__(self, gt):
            self.global_time, self.priority = gt, 128

    meta = com.get_meta_messages()[0]

    class Msg(object):
        """As the reference's Message.Implementation: .meta, and database_id read through it (message.py:265-266)."""

        def __init__(self, gt, packet):
            self.meta, self.distribution, self.packet, self.candidate = meta, Dist(gt), packet, None

        @property
        def database_id(self):
            return self.meta.database_id

    rng = np.random.Generator(np.random.PCG64(314))
    work = []
    for b in range(batches + 1):
        lens = rng.integers(100, 1501, size=batch)
        data = rng.bytes(int(lens.sum()))
        cuts = np.concatenate([[0], np.cumsum(lens)])
        base = n0 + b * batch
        # global time = row + 1, as every row of the headline store (the duplicate-check leg keys rows that way)
        work.append([Msg(base + j + 1, data[int(cuts[j]):int(cuts[j + 1])]) for j in range(batch)])
    com.store_messages(work[0])
    times = []
    for msgs in work[1:]:
        t0 = time.perf_counter()
        com.store_messages(msgs)
        times.append(time.perf_counter() - t0)
    ms2 = sorted(times)[len(times) // 2] * 1e3
    store_msgs = {"call": "SyncCommunity.store_messages(%d messages) -> SyncStore.append -> dsy_store_append" % batch,
                  "median_ms_per_batch": round(ms2, 3), "messages_per_s": round(batch / (ms2 / 1e3), 1),
                  "store_rows_after": int(lib.dsy_store_rows(store))}
    return {"respond": respond, "store_messages": store_msgs}


def dedup_bench(args, ctx, lib, store, blob, offsets, N, batch=10_000, reps=10, cpu_leg=True):
    """SURVEY §8f row 3, the duplicate check of received sync packets (_is_duplicate_sync_message,
    dispersy.py:831-918) against the headline's 10 M-packet store: the (member, global_time) table is built once
    (dsy_store_index_members, every row), then batches of `batch` received messages -- half exact copies of stored
    packets, half new (member, global_time) keys -- go through dsy_dup_check (one wave per message: 64-slot probes,
    64-byte packet compares).  Wall time per call, PCIe upload of the messages included."""
    import torch
    rng = np.random.Generator(np.random.PCG64(123))
    n_rows = int(lib.dsy_store_rows(store))  # the headline's rows plus what the drop-in leg stored (gt = row + 1)
    member = (np.arange(n_rows, dtype=np.uint64) % np.uint64(65536))  # with global_time = row + 1: unique keys
    gt = np.arange(1, n_rows + 1, dtype=np.uint64)
    t0 = time.perf_counter()
    _native.check(lib.dsy_store_index_members(ctx.handle, store, member.ctypes.data, gt.ctypes.data, n_rows))
    build_ms = (time.perf_counter() - t0) * 1e3

    def make():
        dup_rows = rng.integers(0, N, size=batch // 2)
        off_d = offsets[torch.from_numpy(dup_rows).to(offsets.device)].cpu().numpy()
        end_d = offsets[torch.from_numpy(dup_rows + 1).to(offsets.device)].cpu().numpy()
        pk = [bytes(blob[int(a):int(e)].cpu().numpy().tobytes()) for a, e in zip(off_d, end_d)]
        mem = list(member[dup_rows]) + list(rng.integers(70_000, 1 << 30, size=batch - batch // 2))
        gts = list(gt[dup_rows]) + list(rng.integers(1, N + 1, size=batch - batch // 2))
        pk += [rng.bytes(int(x)) for x in rng.integers(100, 1501, size=batch - batch // 2)]
        off = np.zeros(batch + 1, dtype=np.uint64)
        np.cumsum([len(p) for p in pk], out=off[1:])
        return (b"".join(pk), off, np.asarray(mem, dtype=np.uint64), np.asarray(gts, dtype=np.uint64))

    data, off, mem, gts = make()
    sl = np.full(batch, 60, dtype=np.uint32)
    verdict = np.zeros(batch, dtype=np.uint8)
    row = np.zeros(batch, dtype=np.uint64)

    def check():
        _native.check(lib.dsy_dup_check(ctx.handle, store, mem.ctypes.data, gts.ctypes.data, data, len(data),
                                        off.ctypes.data, batch, sl.ctypes.data, verdict.ctypes.data, row.ctypes.data))

    check()
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        check()
        times.append(time.perf_counter() - t0)
    ms = sorted(times)[len(times) // 2] * 1e3
    exact = int((verdict == _native.DSY_DUP_EXACT).sum())
    new = int((verdict == _native.DSY_DUP_NEW).sum())
    cpu = None
    if cpu_leg and args.cpu_claims > 0:  # the reference's SELECT + compare per message over sqlite3 (oracle/sync_ref.py)
        import sqlite3
        from oracle.sync_ref import SYNC_SCHEMA, is_duplicate_sync_message
        conn = sqlite3.connect(":memory:")
        conn.executescript(SYNC_SCHEMA)
        pre = 200_000
        crng = np.random.Generator(np.random.PCG64(6))
        conn.executemany("INSERT INTO sync (community, member, global_time, meta_message, packet) VALUES (1, ?, ?, 1, ?)",
                         ((int(member[i]), int(gt[i]), crng.bytes(int(l)))
                          for i, l in zip(range(pre), crng.integers(100, 1501, size=pre))))
        conn.commit()
        # the first half hits a stored (member, global_time) of the smaller table, the second half misses
        hit_gt = [int(gts[i]) % pre + 1 for i in range(batch // 2)]
        sample = [dict(member=(g - 1) % 65536, gt=g, packet=data[int(off[i]):int(off[i + 1])], signature_length=60,
                       index=i) for i, g in enumerate(hit_gt)]
        sample += [dict(member=int(mem[i]), gt=int(gts[i]), packet=data[int(off[i]):int(off[i + 1])],
                        signature_length=60, index=i) for i in range(batch // 2, batch)]
        sends = []
        t0 = time.perf_counter()
        for m_ in sample:
            is_duplicate_sync_message(conn, 1, m_, sends)
        dt = time.perf_counter() - t0
        model, cores = cpu_info()

        conn.close()

        m_pre, g_pre = member[:pre].copy(), gt[:pre].copy()  # what the workers' tables need (not 10 M rows)

        def table():
            c = sqlite3.connect(":memory:")
            c.executescript(SYNC_SCHEMA)
            r = np.random.Generator(np.random.PCG64(6))
            c.executemany("INSERT INTO sync (community, member, global_time, meta_message, packet) VALUES (1, ?, ?, 1, ?)",
                          ((int(m_pre[i]), int(g_pre[i]), r.bytes(int(l)))
                           for i, l in zip(range(pre), r.integers(100, 1501, size=pre))))
            c.commit()
            return c

        def shard(_):  # every process builds the same table (untimed), then checks the same batch against it
            c = table()
            t1 = time.perf_counter()
            for m_ in sample:
                is_duplicate_sync_message(c, 1, m_, [])
            return len(sample), time.perf_counter() - t1
        ncore = n_core_leg(shard, list(range(cores)), "messages/s",
                           "the same %d messages in every process, each against its own copy of the %d-row table"
                           % (batch, pre))
        cpu = {"value": round(batch / dt, 1), "unit": "messages/s", "cores": 1, "kind": "port", "cpu_model": model,
               "sample": "%d messages through the reference's SELECT packet, undone ... WHERE community, member, "
                         "global_time + packet compare (dispersy.py:868-910) on an in-memory sqlite3 sync table of "
                         "%d rows" % (batch, pre), "n_core": ncore}
    return {"metric": "received messages duplicate-checked/sec", "batch": batch, "store_rows": N,
            "index_build_ms": round(build_ms, 2), "median_ms_per_batch": round(ms, 3),
            "messages_per_s": round(batch / (ms / 1e3), 1), "found_exact": exact, "found_new": new,
            "cpu_baseline": cpu}


def claim_bench(args, ctx, lib, store, N, capacity, mean_len, reps=20, cpu_leg=True):
    """SURVEY §8f row 4, the requester's modulo claim (_dispersy_claim_sync_bloom_filter_modulo,
    community.py:908-933) over the headline's 10 M-packet store: modulo = ceil(N / capacity), a random offset per
    claim; dsy_claim_modulo scans the meta's live index for the residue class and hashes the hits into the MTU filter.
    Wall time per call (filter up and down the bus included).  Algorithmic bytes per claim: 8 B of global_time per
    indexed row + 8 B row id and the packet bytes of every hit."""
    from dispersy_amd.bloomfilter import BloomFilter
    rng = np.random.Generator(np.random.PCG64(77))
    modulo = int(np.ceil(N / float(capacity)))
    ids = np.asarray([1], dtype=np.uint32)
    count = ctypes.c_uint64(0)
    times, hits = [], []
    for r in range(reps + 2):
        bf = BloomFilter(args.filter_bits, args.error_rate, bytes([int(rng.integers(0, 256))]))
        buf = ctypes.create_string_buffer(bytes(bf._raw), len(bf._raw))
        offset = int(rng.integers(0, modulo))
        t0 = time.perf_counter()
        _native.check(lib.dsy_claim_modulo(ctx.handle, ctypes.byref(bf.params), store, ids.ctypes.data, 1, offset,
                                           modulo, buf, ctypes.byref(count)))
        if r >= 2:
            times.append(time.perf_counter() - t0)
            hits.append(count.value)
    ms = sorted(times)[len(times) // 2] * 1e3
    hit = float(np.mean(hits))
    alg_bytes = 8.0 * N + hit * (8 + mean_len)
    cpu = cpu_largest = None
    if cpu_leg and args.cpu_claims > 0:  # the reference's SELECT (community.py:918) in sqlite + hashlib add_keys
        import sqlite3
        from oracle import sync_ref
        from oracle.bloom_ref import OracleBloom
        from oracle.sync_ref import SYNC_SCHEMA
        pre = 1_000_000
        crng = np.random.Generator(np.random.PCG64(8))
        conn = sqlite3.connect(":memory:")
        conn.executescript(SYNC_SCHEMA)
        conn.executemany("INSERT INTO sync (community, member, global_time, meta_message, packet) VALUES (1, ?, ?, 1, ?)",
                         ((i, i + 1, crng.bytes(int(l))) for i, l in enumerate(crng.integers(100, 1501, size=pre))))
        conn.commit()
        cmod = int(np.ceil(pre / float(capacity)))
        t0 = time.perf_counter()
        nclaims = 3
        for c in range(nclaims):
            ob = OracleBloom.from_m_f(args.filter_bits, args.error_rate, bytes([c]))
            ob.add_keys([bytes(p) for p, in conn.execute(
                "SELECT sync.packet FROM sync WHERE meta_message IN (1) AND sync.undone = 0 "
                "AND (sync.global_time + ?) % ? = 0", (c, cmod))])
        dt = time.perf_counter() - t0
        # the largest strategy's reference path on the same table: its SELECT ... ORDER BY global_time LIMIT
        # (community.py:884-888) twice per claim + add_keys, through oracle/sync_ref.claim_largest
        import random as _r
        lmetas = [dict(name="bench", id=1, direction="ASC", priority=128, pruning=None)]
        t1 = time.perf_counter()
        n_large = 20
        for c in range(n_large):
            sync_ref.claim_largest(conn, lmetas, args.filter_bits, args.error_rate, pre, pre + 10000, pre,
                                   _r.Random(c), OracleBloom)
        dt_large = time.perf_counter() - t1
        conn.close()
        model, _ = cpu_info()
        cpu = {"value": round(nclaims * pre / dt, 1), "unit": "indexed rows/s", "cores": 1, "kind": "port",
               "cpu_model": model,
               "sample": "row-rate comparison, not the same workload: %d modulo claims (modulo %d) through the "
                         "reference's SELECT (community.py:918) on an in-memory sqlite3 sync table of %d rows + hashlib "
                         "add_keys of the hits; the GPU line scans a %d-row store, so compare indexed rows/s"
                         % (nclaims, cmod, pre, N)}
        cpu_largest = {"value": round(n_large / dt_large, 2), "unit": "largest claims/s", "cores": 1, "kind": "port",
                       "cpu_model": model,
                       "sample": "%d claims through oracle/sync_ref.claim_largest (the reference's ORDER BY global_time "
                                 "LIMIT capacity+1 SELECTs, community.py:839-903, + hashlib add_keys) over the %d-row "
                                 "sqlite3 table; the SELECTs walk the (meta, undone, global_time) index, so their cost "
                                 "does not grow with the table" % (n_large, pre)}
    largest = claim_largest_bench(args, ctx, lib, store, N, capacity, cpu_largest)
    return {"metric": "modulo claims built/sec", "store_rows": N, "modulo": modulo, "mean_hits": round(hit, 1),
            "median_ms_per_claim": round(ms, 3), "claims_per_s": round(1e3 / ms, 1),
            "indexed_rows_per_s": round(N / (ms / 1e3), 1),
            "achieved_gbs": round(alg_bytes / (ms / 1e3) / 1e9, 1), "cpu_baseline": cpu, "largest": largest}


def claim_largest_bench(args, ctx, lib, store, N, capacity, cpu, reps=20):
    """The default (largest) claim strategy on the device (dsy_claim_largest, community.py:763-903): pivots drawn as
    the reference draws them (gt - expovariate(2 / gt)) over the 10 M-row store, capacity rows selected on each side,
    the wider range's rows hashed into the MTU filter.  Wall time per call (filter over the bus included)."""
    import random as _r
    from dispersy_amd.bloomfilter import BloomFilter
    rng = _r.Random(2718)
    ids = np.asarray([1], dtype=np.uint32)
    out = (ctypes.c_uint64 * 4)()
    times, added = [], []
    for r in range(reps + 2):
        bf = BloomFilter(args.filter_bits, args.error_rate, bytes([rng.randrange(256)]))
        buf = ctypes.create_string_buffer(bytes(bf._raw), len(bf._raw))
        pivot = N - int(rng.expovariate(1.0 / (N / 2.0)))
        if pivot < 1:
            pivot = int(rng.random() * N)
        t0 = time.perf_counter()
        _native.check(lib.dsy_claim_largest(ctx.handle, ctypes.byref(bf.params), store, ids.ctypes.data, 1, pivot,
                                            capacity, N, N + 10000, buf, out))
        if r >= 2:
            times.append(time.perf_counter() - t0)
            added.append(out[2])
    ms = sorted(times)[len(times) // 2] * 1e3
    return {"metric": "largest claims built/sec", "store_rows": N, "median_ms_per_claim": round(ms, 3),
            "claims_per_s": round(1e3 / ms, 1), "mean_rows_hashed": round(float(np.mean(added)), 1),
            "cpu_baseline": cpu}


def ingest_bench(args, ctx, lib, store, step, N, batch=10_000, batches=10, cpu_leg=True):
    """SURVEY §8f row 1, requester-side ingest: `Dispersy._store` INSERTs each batch of received sync packets
    (dispersy.py:1475-1612).  Here batches of `batch` packets (100-1500 B, global times spread over the store's
    range, so they land everywhere in the index and tie with stored rows) go into the headline's 10 M-packet store
    through dsy_store_append: host buffers -> HBM, line copy, row records; the rows' (meta, global_time, rowid) index
    entries are queued and merged into the index by its next reader (k_ingest_*: 16 B read + 16 B written per
    indexed row, once for all the batches appended since).  The first append moves the caller-owned
    (attached) store into grow-able buffers of its own and is reported apart.  A responder step runs on the grown
    store afterwards.  Wall time per call, PCIe upload of the packets included."""
    import torch
    rng = np.random.Generator(np.random.PCG64(99))

    top = [N]  # the highest global time stored so far

    def make(kind):
        lens = rng.integers(100, 1501, size=batch)
        off = np.zeros(batch + 1, dtype=np.uint64)
        np.cumsum(lens, out=off[1:])
        data = rng.bytes(int(off[-1]))
        if kind == "new":  # messages created after everything stored (the Lamport global time only grows)
            gts = rng.integers(top[0] + 1, top[0] + 1 + batch, size=batch).astype(np.uint64)
            top[0] += batch
        elif kind == "recent":  # received messages of the last 10 k global times and above
            gts = rng.integers(top[0] - 10_000, top[0] + batch, size=batch).astype(np.uint64)
            top[0] += batch
        else:  # old messages (a peer catching up): anywhere in the history
            gts = rng.integers(1, N + 1, size=batch).astype(np.uint64)
        metas = np.ones(batch, dtype=np.uint32)
        return data, off, gts, metas

    member_next = [1 << 40]  # members of the appended rows (the store may hold a duplicate table by now)

    def append(b):
        data, off, gts, metas = b
        mem = np.arange(member_next[0], member_next[0] + batch, dtype=np.uint64)
        member_next[0] += batch
        _native.check(lib.dsy_store_append(ctx.handle, store, data, len(data), off.ctypes.data, batch,
                                           gts.ctypes.data, metas.ctypes.data, mem.ctypes.data))

    def ix_stats():
        out = np.zeros(6, dtype=np.uint64)
        _native.check(lib.dsy_store_index_stats(store, out.ctypes.data))
        return out.astype(np.int64)

    def timed_step():
        ctx.synchronize()
        t0 = time.perf_counter()
        pairs = step()
        ctx.synchronize()
        return (time.perf_counter() - t0) * 1e3, pairs

    first_ms = None
    work_legs = {}
    after_pairs = 0
    for kind in ("history", "recent", "new"):
        work = [make(kind) for _ in range(batches + (1 if first_ms is None else 0))]
        if first_ms is None:  # the first append moves the attached store into buffers of its own
            t0 = time.perf_counter()
            append(work.pop(0))
            first_ms = (time.perf_counter() - t0) * 1e3
            timed_step()  # merges it
        # interleaved, as a Dispersy peer runs: one received batch stored, then the next responder step reads the
        # index (store_flush merges the batch)
        s0, t_app, t_read = ix_stats(), [], []
        for b in work:
            t0 = time.perf_counter()
            append(b)
            t_app.append(time.perf_counter() - t0)
            t_read.append(timed_step()[0])
        s1 = ix_stats()
        base_ms, after_pairs = timed_step()  # a step with nothing to merge
        work_legs[kind] = {
            "global_times": {"history": "anywhere in the store's history [1, %d]" % N,
                             "recent": "the newest 10 k and above (received recent messages)",
                             "new": "above every stored one (messages created since)"}[kind],
            "median_ms_per_append": round(sorted(t_app)[len(t_app) // 2] * 1e3, 3),
            "median_responder_step_after_an_append_ms": round(sorted(t_read)[len(t_read) // 2], 3),
            "responder_step_without_merge_ms": round(base_ms, 3),
            "in_place_tail_merges": int(s1[2] - s0[2]), "whole_index_merges": int(s1[3] - s0[3]),
            "index_bytes_per_append": int((s1[4] - s0[4]) // len(work)),
            "index_bytes_per_append_over_batch_index_bytes": round(float(s1[4] - s0[4]) / len(work) / (16 * batch), 2),
            "index_entries_live_and_slack": [int(s1[0]), int(s1[1])]}
        ms_list = t_app
    ms = sorted(ms_list)[len(ms_list) // 2] * 1e3
    rows = int(lib.dsy_store_rows(store))
    pkt_bytes = float(np.mean([len(w[0]) for w in work]))
    torch.cuda.synchronize()
    cpu = None
    if cpu_leg and args.cpu_claims > 0:  # the CPU baseline leg: the reference's INSERT through sqlite3 (oracle/sync_ref.py)
        import sqlite3
        from oracle.sync_ref import SYNC_SCHEMA, insert_packets
        conn = sqlite3.connect(":memory:")
        conn.executescript(SYNC_SCHEMA)
        pre = 200_000
        crng = np.random.Generator(np.random.PCG64(5))
        plens = crng.integers(100, 1501, size=pre)
        conn.executemany("INSERT INTO sync (community, member, global_time, meta_message, packet) VALUES (1, ?, ?, 1, ?)",
                         ((i, int(g), crng.bytes(int(l))) for i, (g, l) in
                          enumerate(zip(crng.integers(1, N + 1, size=pre), plens))))
        conn.commit()
        data, off, gts, _ = work[1]
        msgs = [(pre + i, int(gts[i]), 1, data[int(off[i]):int(off[i + 1])]) for i in range(batch)]
        t0 = time.perf_counter()
        insert_packets(conn, 1, msgs)
        conn.commit()
        dt = time.perf_counter() - t0
        conn.close()
        model, cores = cpu_info()

        def shard(_):  # every process fills its own table (untimed), then INSERTs the same batch
            c = sqlite3.connect(":memory:")
            c.executescript(SYNC_SCHEMA)
            r = np.random.Generator(np.random.PCG64(5))
            pl = r.integers(100, 1501, size=pre)
            c.executemany("INSERT INTO sync (community, member, global_time, meta_message, packet) VALUES (1, ?, ?, 1, ?)",
                          ((i, int(g), r.bytes(int(l))) for i, (g, l) in enumerate(zip(r.integers(1, N + 1, size=pre), pl))))
            c.commit()
            t1 = time.perf_counter()
            insert_packets(c, 1, msgs)
            c.commit()
            return len(msgs), time.perf_counter() - t1
        ncore = n_core_leg(shard, list(range(cores)), "packets/s",
                           "the same %d-packet batch in every process, each into its own %d-row table" % (batch, pre))
        cpu = {"value": round(batch / dt, 1), "unit": "packets/s", "cores": 1, "kind": "port", "cpu_model": model,
               "sample": "one batch of %d packets INSERTed one statement each (dispersy.py:1523-1533) into an "
                         "in-memory sqlite3 sync table with its index, pre-filled with %d rows" % (batch, pre),
               "n_core": ncore}
    return {"metric": "received packets stored/sec", "batch": batch, "batches": batches, "cpu_baseline": cpu,
            "store_rows_after": rows, "median_ms_per_batch": round(ms, 3),
            "packets_per_s": round(batch / (ms / 1e3), 1),
            "first_append_ms": round(first_ms, 2), "packet_bytes_per_append": int(pkt_bytes),
            "index_maintenance": "an append queues its rows' (meta, global_time, row) entries (16 B each) on the "
                                 "device; the next read of the index orders them (radix sort) and merges each meta's "
                                 "tail from its first new entry in place into the slack of its region, or merges the "
                                 "whole index once (32 B per entry) when the tails would move more",
            "index_bytes_per_append": work_legs["new"]["index_bytes_per_append"],
            "workloads": work_legs,
            "roofline": {"kernel": "the whole append call: packet upload (PCIe), line copy, row records",
                         "bound": "hbm", "unit": "GB/s", "peak": PEAK_HBM_GBS,
                         "achieved": round((16 * batch + pkt_bytes) / (ms / 1e3) / 1e9, 1),
                         "frac": round((16 * batch + pkt_bytes) / (ms / 1e3) / 1e9 / PEAK_HBM_GBS, 4),
                         "traffic": None},
            "respond_after_ingest_pairs": int(after_pairs)}


def gossip_sim(args, ctx, dev, rank, world, dist):
    """BASELINE config 3: the epidemic-sync simulator (dispersy_amd/sim.py) -- P peers block-sharded over the
    ranks, one gossip round = every peer claims (MTU filter over its store), every claim is answered, every peer
    stores what it got; two RCCL all-to-all(v) exchanges per round.  Total work is fixed (strong scaling)."""
    import torch
    from dispersy_amd.sim import EpidemicSim, GpuEngine, make_config, make_universe
    blob, offs = make_universe(args.sim_universe, seed=11)
    chunks = args.sim_chunks or (4 if world > 1 else 1)
    cfg = make_config(args.sim_peers, args.sim_universe, rank, world, seed=11, chunks=chunks)
    eng = GpuEngine(cfg, blob, offs, dev, ctx=ctx)
    eng.seed(args.sim_initial)
    sim = EpidemicSim(eng, cfg, rank, world, dist, dev, chunks=chunks)
    held0 = sim.global_stats()[0]
    for r in range(args.sim_warmup):
        sim.round(r)
    eng.sync()
    ex0 = (sim.exchanged_bytes, sim.exchanged_remote)
    ctx.reset_timing()
    ctx.set_timing(True, only=[_native.TIME_SIM_BUILD, _native.TIME_SIM_RESPOND])
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for r in range(args.sim_warmup, args.sim_warmup + args.sim_rounds):
        sim.round(r)
    eng.sync()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    ctx.set_timing(False)
    kernels = {}
    for name, cls in (("k_sim_build_claims<md5>", _native.TIME_SIM_BUILD), ("k_sim_respond<md5>", _native.TIME_SIM_RESPOND)):
        kt, wk = ctx.kernel_time(cls), ctx.work(cls)
        secs = kt["ms"] / 1e3
        kernels[name] = {
            "ms_per_round": round(kt["ms"] / max(args.sim_rounds, 1), 3),
            "gblocks_per_s": round(wk["blocks"] / secs / 1e9, 2) if secs else None,
            "valu_int32": {"achieved": round(wk["blocks"] * OPS_PER_BLOCK["md5"] / secs / 1e12, 2) if secs else None,
                           "peak": PEAK_INT32_TOPS, "unit": "Tops/s",
                           "frac": round(wk["blocks"] * OPS_PER_BLOCK["md5"] / secs / 1e12 / PEAK_INT32_TOPS, 4)
                           if secs else None},
            "lane_utilization": round(wk["blocks"] / max(wk["lane_slots"], 1), 4),
            "blocks_per_round": int(wk["blocks"] / max(args.sim_rounds, 1))}
    # per rank and round: record bytes this rank sent (claims + responses), and the part that left the rank
    mine = torch.tensor([(sim.exchanged_bytes - ex0[0]) // max(args.sim_rounds, 1),
                         (sim.exchanged_remote - ex0[1]) // max(args.sim_rounds, 1)], dtype=torch.int64, device=dev)
    per_rank = [mine.tolist()]
    if sim.coll is not None:
        dt = float(sim.coll.scalar(dt, "max", device=dev))
        every = torch.zeros(2 * world, dtype=torch.int64, device=dev)
        sim.coll.all_gather_into(every, mine)
        per_rank = every.view(world, 2).tolist()
    held, chk = sim.global_stats()
    return {"metric": "gossip sync rounds/sec", "value": round(args.sim_rounds / dt, 3), "unit": "rounds/s",
            "n_gpus": world, "scaling": "strong", "rounds": args.sim_rounds, "warmup_rounds": args.sim_warmup,
            "ms_per_round": round(dt / args.sim_rounds * 1e3, 3),
            "config": {"peers": args.sim_peers, "universe": args.sim_universe, "initial_packets": args.sim_initial,
                       "filter": "m=%d k=%d md5" % (cfg.m_bits, cfg.k), "byte_limit": cfg.byte_limit},
            "packets_held_start": held0, "packets_held_end": held, "store_checksum": "%016x" % chk,
            "exchange_bytes_rank0": sim.exchanged_bytes, "kernels": kernels, "chunks": chunks,
            "exchange_per_round": {"bytes_sent_per_rank": [r[0] for r in per_rank],
                                   "bytes_to_other_ranks_per_rank": [r[1] for r in per_rank],
                                   "how": "two all-to-all(v) per round (claims %d B, responses %d B per peer)%s"
                                          % (cfg.claim_bytes, cfg.resp_bytes,
                                             ", overlapped with the kernels in %d chunks" % chunks
                                             if chunks > 1 and world > 1 else "")},
            "cpu_baseline": gossip_cpu(args, blob, offs) if rank == 0 and world == 1 and args.cpu_claims > 0 else None}


def gossip_cpu(args, blob, offs, peers=10_000):
    """oracle/sim_ref's CPU engine (hashlib + Python, the reference's per-packet work) runs ONE round of a
    `peers`-peer simulation from the seeded state; a round of the benchmarked args.sim_peers peers is that work
    times args.sim_peers / peers (stated as an extrapolation).  N cores: one independent
    `peers`-peer round per process."""
    from dispersy_amd.sim import EpidemicSim, make_config
    from oracle.sim_ref import OracleEngine
    scale = args.sim_peers / float(peers)

    def one_round(seed):
        cfg = make_config(peers, args.sim_universe, 0, 1, seed=seed)
        eng = OracleEngine(cfg, blob, offs, arrays="numpy")
        eng.seed(args.sim_initial)
        sim = EpidemicSim(eng, cfg)
        t0 = time.perf_counter()
        sim.round(0)
        return time.perf_counter() - t0, sim.tested

    dt, tested = one_round(11)
    model, cores = cpu_info()
    ncore = n_core_leg(lambda seed: one_round(seed) and 1, [11 + w for w in range(cores)], "rounds of %d peers/s" % peers,
                       "one %d-peer round per process" % peers)
    return {"value": round(1.0 / (dt * scale), 5), "unit": "rounds/s (extrapolated to %d peers)" % args.sim_peers,
            "cores": 1, "kind": "port", "cpu_model": model,
            "sample": "one round of a %d-peer simulation (universe %d, %d initial packets per peer) through "
                      "oracle/sim_ref.OracleEngine: %.2f s, %d (claim, packet) pairs tested; x %g for %d peers"
                      % (peers, args.sim_universe, args.sim_initial, dt, tested, scale, args.sim_peers),
            "n_core": dict(ncore, value_extrapolated=round(ncore["value"] / scale, 5),
                           unit_extrapolated="rounds/s (extrapolated to %d peers)" % args.sim_peers)}


def _blocks(lengths, plen, hash_name):
    """Compression blocks of prefix || key per key (SURVEY §8 conventions): floor((p+L+8)/64)+1, or /128 with a
    16-byte length field for SHA-384/512."""
    blk, lb = (128, 16) if hash_name in ("sha384", "sha512") else (64, 8)
    return int(((lengths + plen + lb) // blk + 1).sum().item())


def _timed_bloom(ctx, fn, reps):
    """Run fn() reps times on the ctx stream with HIP-event timing of the bloom kernel class; returns (avg kernel
    seconds, wall seconds per rep)."""
    ctx.synchronize()
    ctx.reset_timing()
    ctx.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    ctx.synchronize()
    wall = (time.perf_counter() - t0) / reps
    ctx.set_timing(False)
    kt = ctx.kernel_time(_native.TIME_BLOOM)
    return kt["ms"] / 1e3 / max(kt["launches"], 1), wall


def bloom_vs_oracle(ctx, lib, bf, m, f, prefix, blob, add_off, n_add, test_off, n_test, dev):
    """In-leg parity check of the single-filter kernels: a fresh filter built on the GPU from the n_add keys at
    add_off, then n_test keys at test_off tested; the same through oracle/bloom_ref (hashlib, bloomfilter.py:160-197)
    on host copies.  Filter bytes and every membership verdict must be equal."""
    import torch
    from oracle.bloom_ref import OracleBloom
    filt = torch.zeros(int(lib.dsy_filter_words(m)), dtype=torch.int32, device=dev)
    present = torch.empty(max(n_test, 1), dtype=torch.uint8, device=dev)
    ctx.wait_torch(dev)
    _native.check(lib.dsy_bloom_add_dev(ctx.handle, ctypes.byref(bf.params), blob.data_ptr(), add_off.data_ptr(), n_add,
                                        filt.data_ptr()))
    _native.check(lib.dsy_bloom_test_dev(ctx.handle, ctypes.byref(bf.params), blob.data_ptr(), test_off.data_ptr(),
                                         n_test, filt.data_ptr(), present.data_ptr()))
    ctx.synchronize()
    got_bytes = filt.cpu().numpy().view(np.uint8)[:m // 8].tobytes()
    got = present[:n_test].cpu().numpy()
    ob = OracleBloom.from_m_f(m, f, prefix)
    def keys(off, n):  # the n keys at off as bytes (one host copy of just their span)
        o = off[:n + 1].cpu().numpy()
        lo = int(o[0])
        host = blob[lo:int(o[-1])].cpu().numpy().tobytes()
        return [host[int(o[i]) - lo:int(o[i + 1]) - lo] for i in range(n)]
    ob.add_keys(keys(add_off, n_add))
    want = np.fromiter((k in ob for k in keys(test_off, n_test)), dtype=np.uint8, count=n_test)
    return {"adds": n_add, "tests": n_test, "filter_bytes_equal": got_bytes == ob.to_bytes(),
            "membership_equal": bool(np.array_equal(got, want)), "present_fraction": round(float(got.mean()), 4)}


def single_filter(args, ctx, lib, blob, offsets, N, dev, rank, world):
    """BASELINE config 1 at GPU scale: BloomFilter(10160, 0.01, 4-byte prefix) (MD5, k=7) and the reference's test
    filter BloomFilter(4096, 0.001, b"x") (SHA-1, k=10, tests/debugcommunity/node.py:617): add 100 k packets, then
    test all N packets of the config-2 store (already in HBM) -- dsy_bloom_add_dev / dsy_bloom_test_dev."""
    import torch
    from dispersy_amd.bloomfilter import BloomFilter
    n_add = min(100_000, N)
    lengths = offsets[1:] - offsets[:-1]
    out = {}
    present = torch.empty(N, dtype=torch.uint8, device=dev)
    for name, m, f, prefix in (("md5", 10160, 0.01, b"\x00\x01\x02\x03"), ("sha1", 4096, 0.001, b"x")):
        bf = BloomFilter(m, f, prefix)
        assert bf.hash_name == name
        filt = torch.zeros(int(lib.dsy_filter_words(m)), dtype=torch.int32, device=dev)
        add = lambda: _native.check(lib.dsy_bloom_add_dev(ctx.handle, ctypes.byref(bf.params), blob.data_ptr(),  # noqa: E731
                                                          offsets.data_ptr(), n_add, filt.data_ptr()))
        test = lambda: _native.check(lib.dsy_bloom_test_dev(ctx.handle, ctypes.byref(bf.params), blob.data_ptr(),  # noqa: E731
                                                            offsets.data_ptr(), N, filt.data_ptr(), present.data_ptr()))
        ctx.wait_torch(dev)  # the zeroed filter (torch's stream) before the ctx stream's build
        add()
        test()  # warm-up
        k_add, _ = _timed_bloom(ctx, add, 3)
        k_test, wall = _timed_bloom(ctx, test, 5)
        blocks = _blocks(lengths, len(prefix), name)
        nbytes = int(lengths.sum().item())
        ops = blocks * OPS_PER_BLOCK[name]
        out[name] = {
            "filter": "BloomFilter(%d, %g, prefix=%r): %s k=%d" % (m, f, prefix, name, bf.functions),
            "add_keys_per_s": round(n_add / k_add, 1), "test_keys": N,
            "test_keys_per_s": round(N / k_test, 1), "test_wall_keys_per_s": round(N / wall, 1),
            "present_fraction": round(float(present.float().mean().item()), 4),
            "roofline_test": {"kernel": "k_bloom_test<%s>" % name, "avg_launch_us": round(k_test * 1e6, 1),
                              "gblocks_per_s": round(blocks / k_test / 1e9, 2),
                              "hbm": {"achieved": round((nbytes + 16 * N + N) / k_test / 1e9, 1), "peak": PEAK_HBM_GBS,
                                      "unit": "GB/s", "frac": round((nbytes + 17 * N) / k_test / 1e9 / PEAK_HBM_GBS, 4)},
                              "valu_int32": {"achieved": round(ops / k_test / 1e12, 2), "peak": PEAK_INT32_TOPS,
                                             "unit": "Tops/s", "frac": round(ops / k_test / 1e12 / PEAK_INT32_TOPS, 4),
                                             "ops_per_block": OPS_PER_BLOCK[name]}},
        }
        # the leg above fills the filter far past its capacity (every bit set): a GPU == oracle check of the same
        # kernels on 20 k adds and 50 k tests, then SURVEY §8(d) row 1's at-capacity variant -- get_capacity(f) adds
        # (1059 for the MTU filter), 1 M tests, false positives ~f -- timed and checked against the oracle in full
        out[name]["gpu_vs_oracle"] = bloom_vs_oracle(ctx, lib, bf, m, f, prefix, blob, offsets, 20_000, offsets,
                                                     50_000, dev)
        cap = bf.get_capacity(f)
        n_t = min(1_000_000, N)
        filt.zero_()
        ctx.wait_torch(dev)
        add_cap = lambda: _native.check(lib.dsy_bloom_add_dev(ctx.handle, ctypes.byref(bf.params), blob.data_ptr(),  # noqa: E731
                                                              offsets.data_ptr(), cap, filt.data_ptr()))
        test_cap = lambda: _native.check(lib.dsy_bloom_test_dev(ctx.handle, ctypes.byref(bf.params), blob.data_ptr(),  # noqa: E731
                                                                offsets.data_ptr(), n_t, filt.data_ptr(),
                                                                present.data_ptr()))
        add_cap()
        test_cap()
        k_cap, wall_cap = _timed_bloom(ctx, test_cap, 5)
        chk = bloom_vs_oracle(ctx, lib, bf, m, f, prefix, blob, offsets, cap, offsets, n_t, dev) \
            if rank == 0 and world == 1 and args.cpu_claims > 0 else None
        out[name]["at_capacity"] = {
            "adds": cap, "tests": n_t, "test_keys_per_s": round(n_t / k_cap, 1),
            "test_wall_keys_per_s": round(n_t / wall_cap, 1),
            "present_fraction": round(float(present[:n_t].float().mean().item()), 4),
            "expected_present_fraction": round(cap / n_t + f * (1 - cap / n_t), 4),
            "avg_launch_us": round(k_cap * 1e6, 1), "gpu_vs_oracle": chk}
    # HBM traffic of the test launches from the committed single-size PMC passes (tools/cfg1_run.py under rocprofv3,
    # profiles/pmc_traffic_cfg1.json), reported only for the kernel code they measured (tools/kernel_hash.py)
    traffic_file = os.path.join(ROOT, "profiles", "pmc_traffic_cfg1.json")
    if os.path.isfile(traffic_file):
        from tools.kernel_hash import kernel_sha
        with open(traffic_file) as f:
            recs = json.load(f)
        lib_path = os.environ.get("DSY_LIB_PATH") or _native.LIB_PATH
        for name in ("md5", "sha1"):
            rec, rt = recs.get(name), out.get(name, {}).get("roofline_test")
            if not rec or rt is None:
                continue
            now = kernel_sha(lib_path, rec["symbol"])
            alg = int(lengths.sum().item()) + 17 * N
            if now is not None and now == rec.get("kernel_sha") and int(rec.get("keys", -1)) == N:
                rt["traffic"] = rec["hbm_bytes_per_launch"]
                rt["traffic_over_algorithmic"] = round(rec["hbm_bytes_per_launch"] / alg, 3)
                rt["traffic_source"] = "profiles/pmc_traffic_cfg1.json (%s; same kernel code, sha256 %s)" % (
                    rec.get("round"), now[:16])
            else:
                rt["traffic"] = None
                rt["traffic_source"] = "not reported: profiles/pmc_traffic_cfg1.json measured another build or size"
    if rank == 0 and world == 1:
        out["cpu_baseline"] = single_filter_cpu(blob, offsets)
    return out


def host_keys(blob, offsets, n):
    """The first n packets of a device store as (Shared blob, Shared offsets) on the host."""
    end = int(offsets[n].item())
    return Shared(blob[:end].cpu().numpy()), Shared(offsets[:n + 1].cpu().numpy())


def key_list(s_blob, s_off, lo=0, hi=None):
    """bytes objects of packets [lo, hi) of a host_keys pair (the reference's keys are py2 str)."""
    b, o = s_blob.a, s_off.a
    hi = len(o) - 1 if hi is None else hi
    return [bytes(b[int(o[i]):int(o[i + 1])]) for i in range(lo, hi)]


def single_filter_cpu(blob, offsets, n_add=100_000, n_test=1_000_000):
    """BASELINE config 1 in full on the CPU (BASELINE.md:46): oracle/bloom_ref (hashlib + Python int bit array)
    adds 100 k packets and tests 1 M (the first 1 M packets of the store, the 100 k added among them), one core;
    then one process per core, each building the same filter (untimed) and testing its disjoint share of the 1 M."""
    from oracle.bloom_ref import OracleBloom
    s_blob, s_off = host_keys(blob, offsets, n_test)
    keys = key_list(s_blob, s_off)
    res = {}
    fams = (("md5", 10160, 0.01, b"\x00\x01\x02\x03"), ("sha1", 4096, 0.001, b"x"))
    for name, m, f, prefix in fams:
        ob = OracleBloom.from_m_f(m, f, prefix)
        t0 = time.perf_counter()
        ob.add_keys(keys[:n_add])
        t1 = time.perf_counter()
        hits = sum(1 for k in keys if k in ob)
        t2 = time.perf_counter()
        res[name] = {"add_keys_per_s": round(n_add / (t1 - t0), 1), "test_keys_per_s": round(n_test / (t2 - t1), 1),
                     "present": hits, "seconds": round(t2 - t0, 2)}
    del keys
    model, cores = cpu_info()
    for name, m, f, prefix in fams:
        def test(w, m=m, f=f, prefix=prefix):
            lo, hi = w * n_test // cores, (w + 1) * n_test // cores
            ob = OracleBloom.from_m_f(m, f, prefix)
            ob.add_keys(key_list(s_blob, s_off, 0, n_add))
            mine = key_list(s_blob, s_off, lo, hi)
            t1 = time.perf_counter()
            for k in mine:
                k in ob  # noqa: B015 -- the membership test is the work
            return hi - lo, time.perf_counter() - t1
        res[name]["n_core"] = n_core_leg(test, list(range(cores)), "tests/s",
                                         "the %d tests split over the processes (disjoint shares), each against its "
                                         "own copy of the filter of the %d adds" % (n_test, n_add))
    return {"kind": "port", "cores": 1, "cpu_model": model,
            "sample": "the full config: %d adds + %d tests (the first %d packets of the store) per filter"
                      % (n_add, n_test, n_test), "results": res}


def large_filter(args, ctx, lib, dev, rank, world, dist=None):
    """BASELINE config 4: BloomFilter(2**b, 0.01, b"\x07") for b in (20, 22, 24) -- SHA-256, 'L' chunks, k=7 --
    filled with --large-keys packets (100-1500 B, seed 99, generated in HBM) and probed with --large-tests other
    packets.  The filters (128 KB - 2 MB) exceed LDS: the build ORs bits into the L2/HBM-resident array.
    With N ranks every rank adds its own --large-keys packets (weak scaling); the partial filters are all-gathered
    over RCCL and OR-ed on the GPU (dsy_filter_or_reduce) into the filter of all N x keys, which every
    rank then probes with its own test packets."""
    import torch
    from dispersy_amd.bloomfilter import BloomFilter
    from dispersy_amd.shard import Collectives, union_filter
    G = _native.BLOB_GUARD
    n_add, n_test = args.large_keys, args.large_tests
    n = n_add + n_test
    g = torch.Generator(device=dev)
    g.manual_seed(99 + 1000 * rank)
    lengths = torch.randint(100, 1501, (n,), device=dev, generator=g, dtype=torch.int64)
    offsets = torch.zeros(n + 1, device=dev, dtype=torch.int64)
    torch.cumsum(lengths, 0, out=offsets[1:])
    total = int(offsets[-1].item())
    blob_full = torch.randint(0, 256, (total + 2 * G,), device=dev, generator=g, dtype=torch.uint8)
    blob = blob_full[G:]
    test_off = offsets[n_add:]
    present = torch.empty(n_test, dtype=torch.uint8, device=dev)
    out = {"keys_added": n_add, "keys_tested": n_test, "key_bytes_added": int(offsets[n_add].item()), "filters": {}}
    add_blocks = _blocks(lengths[:n_add], 1, "sha256")
    test_blocks = _blocks(lengths[n_add:], 1, "sha256")
    for bits in (20, 22, 24):
        m = 1 << bits
        bf = BloomFilter(m, 0.01, b"\x07")
        filt = torch.zeros(int(lib.dsy_filter_words(m)), dtype=torch.int32, device=dev)
        add = lambda: _native.check(lib.dsy_bloom_add_dev(ctx.handle, ctypes.byref(bf.params), blob.data_ptr(),  # noqa: E731
                                                          offsets.data_ptr(), n_add, filt.data_ptr()))
        test = lambda: _native.check(lib.dsy_bloom_test_dev(ctx.handle, ctypes.byref(bf.params), blob.data_ptr(),  # noqa: E731
                                                            test_off.data_ptr(), n_test, filt.data_ptr(),
                                                            present.data_ptr()))
        filt.zero_()
        ctx.wait_torch(dev)  # torch's zeroing before the ctx stream's build
        k_add, wall_add = _timed_bloom(ctx, add, 1)
        union = None
        if dist is not None and world > 1:
            # the whole build as a job: every rank adds its shard, then all-gather + OR of the partial filters
            coll = Collectives(dist)
            filt.zero_()
            torch.cuda.synchronize()
            coll.barrier()
            t0 = time.perf_counter()
            add()
            union = union_filter(ctx, coll, filt)
            torch.cuda.synchronize()  # union_filter returns with the OR queued on torch's stream
            t_job = coll.scalar(time.perf_counter() - t0, "max", device=dev)
            filt.copy_(union)
            torch.cuda.synchronize()
        k_test, wall_test = _timed_bloom(ctx, test, 3)
        ones = int(np.unpackbits(filt.cpu().numpy().view(np.uint8)[:m // 8]).sum())
        if union is not None:
            out.setdefault("sharded_build", {})["2^%d" % bits] = {
                "ranks": world, "keys_all_ranks": world * n_add, "job_s": round(t_job, 4),
                "add_keys_per_s_all_ranks": round(world * n_add / t_job, 1),
                "exchange": "%s all-gather of %d x %d B partial filters + dsy_filter_or_reduce"
                            % ("RCCL" if dist.get_backend() == "nccl" else dist.get_backend(), world, 4 * filt.numel())}
        out["filters"]["2^%d" % bits] = {
            "hash": "%s k=%d chunk=%d" % (bf.hash_name, bf.functions, bf.chunk_bytes),
            "add_keys_per_s": round(n_add / k_add, 1), "add_ms": round(k_add * 1e3, 2),
            "add_wall_keys_per_s": round(n_add / wall_add, 1),
            "add_gblocks_per_s": round(add_blocks / k_add / 1e9, 2),
            "add_valu_frac": round(add_blocks * OPS_PER_BLOCK["sha256"] / k_add / 1e12 / PEAK_INT32_TOPS, 4),
            "test_keys_per_s": round(n_test / k_test, 1), "test_ms": round(k_test * 1e3, 2),
            "test_wall_keys_per_s": round(n_test / wall_test, 1),
            "test_gblocks_per_s": round(test_blocks / k_test / 1e9, 2),
            "bits_set": ones, "present_fraction": round(float(present.float().mean().item()), 4),
        }
    # the legs above saturate every filter (100 M keys): a GPU == oracle check of the HBM-resident-filter kernels at
    # 2^20 on 20 k adds and 20 k tests (oracle/bloom_ref: hashlib SHA-256, 'L' chunks)
    bf = BloomFilter(1 << 20, 0.01, b"\x07")
    out["gpu_vs_oracle_2^20"] = bloom_vs_oracle(ctx, lib, bf, 1 << 20, 0.01, b"\x07", blob, offsets, 20_000, test_off,
                                                20_000, dev)
    if rank == 0 and world == 1:
        out["cpu_baseline"] = large_filter_cpu(blob, offsets)
    del blob_full, blob, offsets, lengths
    torch.cuda.empty_cache()
    return out


def large_filter_cpu(blob, offsets, n_add=100_000, n_test=100_000):
    """oracle/bloom_ref at m = 2^20 (hashlib + Python int bit array: O(m) per set bit, the reference's cost
    model), one core, on 10^5 adds and 10^5 tests (BASELINE.md:50; the cost per op does not depend on the fill, so
    the 100 M-key figure is an extrapolation); then one process per core adding its disjoint share of the 10^5
    into its own partial filter, as a sharded build."""
    from oracle.bloom_ref import OracleBloom
    s_blob, s_off = host_keys(blob, offsets, n_add + n_test)
    keys = key_list(s_blob, s_off)
    ob = OracleBloom.from_m_f(1 << 20, 0.01, b"\x07")
    t0 = time.perf_counter()
    ob.add_keys(keys[:n_add])
    t1 = time.perf_counter()
    sum(1 for k in keys[n_add:] if k in ob)
    t2 = time.perf_counter()
    del keys
    model, cores = cpu_info()

    def adds(w):
        lo, hi = w * n_add // cores, (w + 1) * n_add // cores
        mine = key_list(s_blob, s_off, lo, hi)
        part = OracleBloom.from_m_f(1 << 20, 0.01, b"\x07")
        t3 = time.perf_counter()
        part.add_keys(mine)
        return hi - lo, time.perf_counter() - t3
    ncore = n_core_leg(adds, list(range(cores)), "adds/s",
                       "the %d adds split over the processes (disjoint shares), each into its own 2^20 filter" % n_add)
    return {"kind": "port", "cores": 1, "filter": "2^20", "cpu_model": model,
            "sample": "%d adds + %d tests, extrapolated per key" % (n_add, n_test),
            "add_keys_per_s": round(n_add / (t1 - t0), 1), "test_keys_per_s": round(n_test / (t2 - t1), 1),
            "seconds": round(t2 - t0, 2), "n_core": ncore}


def heavy_tail(args, ctx, lib, dev, rank, world, dist):
    """BASELINE config 5: one responder, 10 M packets with discretised Pareto(1.2) lengths clipped to [60, 65476]
    (the UDP cap, endpoint.py:263) and Zipf(1.1) global times over 1..10^6, serving 1024 claims as in config 2.
    Rows sharing a global time are many (gt = 1 holds ~9 %), so claims vary from a few hundred to ~10^6 rows."""
    import torch
    from dispersy_amd.bloomfilter import BloomFilter
    G = _native.BLOB_GUARD
    N, R = args.packets, args.claims
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    u = torch.rand(N, device=dev, generator=g, dtype=torch.float64)
    lengths = torch.clamp(torch.floor(60.0 * u.pow(-1.0 / 1.2)), max=65476).to(torch.int64)
    del u
    offsets = torch.zeros(N + 1, device=dev, dtype=torch.int64)
    torch.cumsum(lengths, 0, out=offsets[1:])
    total = int(offsets[-1].item())
    blob_full = torch.randint(0, 256, (total + 2 * G,), device=dev, generator=g, dtype=torch.uint8)
    blob = blob_full[G:]
    G_MAX = 1_000_000
    w = torch.arange(1, G_MAX + 1, device=dev, dtype=torch.float64).pow(-1.1)
    cdf = torch.cumsum(w, 0)
    cdf /= cdf[-1].clone()
    gt = torch.searchsorted(cdf, torch.rand(N, device=dev, generator=g, dtype=torch.float64)) + 1
    gt = torch.clamp(gt, max=G_MAX).sort().values.contiguous()
    meta = torch.ones(N, device=dev, dtype=torch.int32)
    torch.cuda.synchronize()
    store = ctypes.c_void_p()
    _native.check(lib.dsy_store_attach(ctx.handle, blob.data_ptr(), total, offsets.data_ptr(), N, gt.data_ptr(),
                                       meta.data_ptr(), None, ctypes.byref(store)))
    h_gt = gt.cpu().numpy()
    # row range of every distinct global time (for residue-class selection without scanning 10 M rows per claim)
    starts = np.searchsorted(h_gt, np.arange(1, G_MAX + 2, dtype=np.int64), side="left")
    rng = np.random.Generator(np.random.PCG64(5 + 1000 * rank))
    cap = BloomFilter(args.filter_bits, args.error_rate).get_capacity(args.error_rate)
    modulo_m = int(math.ceil(N / float(cap)))
    reqs = (_native.Request * R)()
    filters, off, sel_rows, claims = [], 0, 0, []
    for i in range(R):
        if i % 2 == 0:
            a = int(rng.integers(0, N))
            lo, hi = int(h_gt[a]), int(h_gt[min(a + cap - 1, N - 1)])
            modulo, offset = 1, 0
            rows = np.arange(starts[lo - 1], starts[hi], dtype=np.uint64)
        else:
            lo, hi, modulo = 1, G_MAX, modulo_m
            offset = int(rng.integers(0, modulo))
            first = (modulo - offset) % modulo or modulo
            gs = np.arange(first, G_MAX + 1, modulo, dtype=np.int64)
            rows = np.concatenate([np.arange(starts[x - 1], starts[x], dtype=np.uint64) for x in gs]) if len(gs) \
                else np.zeros(0, dtype=np.uint64)
        sel_rows += len(rows)
        prefix = bytes([int(rng.integers(0, 256))])
        bf = BloomFilter(args.filter_bits, args.error_rate, prefix)
        known = np.ascontiguousarray(rows[rng.random(len(rows)) >= 0.01])
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
        q.prefix[0] = prefix[0]
        filters.append(raw)
        claims.append((lo, hi, offset, modulo, bf.functions, prefix, buf.raw))
        off += len(raw)
    fblob = b"".join(filters)
    d_filters = torch.frombuffer(bytearray(fblob + bytes(64)), dtype=torch.uint8).to(dev)
    metas = (_native.Meta * 1)()
    metas[0].meta_id, metas[0].direction = 1, _native.DSY_ASC
    if args.window:
        ctx.set_window(args.window)
    batches = Batches(lib, ctx, store, reqs, R, d_filters.data_ptr(), metas, 1, G_MAX, args.byte_limit)
    pipe = args.pipeline5
    batches.run(2, pipe)
    steps = max(3, args.steps // 4)
    ctx.synchronize()
    ctx.reset_timing()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    hashed = batches.run(steps, pipe)
    ctx.synchronize()
    dt = time.perf_counter() - t0
    work = ctx.work(_native.TIME_PAIR_TEST)
    # kernel times from a serial pass (events of overlapping batches would overlap)
    ctx.reset_timing()
    ctx.set_timing(True)
    t1 = time.perf_counter()
    batches.run(steps, 1)
    serial_dt = time.perf_counter() - t1
    ctx.set_timing(False)
    kt = ctx.kernel_time(_native.TIME_PAIR_TEST)
    swork = ctx.work(_native.TIME_PAIR_TEST)
    useful = work["useful_pairs"]
    if dist is not None and world > 1:  # the whole job: every rank's pairs over the slowest rank's time
        from dispersy_amd.shard import Collectives
        coll = Collectives(dist)
        dt = float(coll.scalar(dt, "max", device=dev))
        useful = int(coll.scalar(int(useful), "sum", device=dev))
        hashed = int(coll.scalar(int(hashed), "sum", device=dev))
    cpu = None
    if rank == 0 and world == 1 and args.cpu_claims > 0:
        cpu = responder_cpu(args, ctx, lib, store, reqs, claims, fblob, blob, offsets, h_gt.astype(np.uint64), G_MAX,
                            dev, "cfg5 heavy tail", check=[i for i in range(R) if i % 16 in (0, 1)])
    lib.dsy_store_free(store)
    secs = kt["ms"] / 1e3
    out = {"metric": "packets hashed+tested/sec", "value": round(useful / dt, 1), "unit": "packets/s", "n_gpus": world,
           "cpu_baseline": cpu,
           "roofline": {"kernel": "k_pair_test<md5>", "bound": "valu+hbm",
                        "valu_int32": {"achieved": round(swork["blocks"] * OPS_PER_BLOCK["md5"] / secs / 1e12, 2)
                                       if secs else None, "peak": PEAK_INT32_TOPS, "unit": "Tops/s",
                                       "frac": round(swork["blocks"] * OPS_PER_BLOCK["md5"] / secs / 1e12 /
                                                     PEAK_INT32_TOPS, 4) if secs else None},
                        "hbm": {"achieved": round(swork["bytes"] / secs / 1e9, 1) if secs else None,
                                "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                "frac": round(swork["bytes"] / secs / 1e9 / PEAK_HBM_GBS, 4) if secs else None}},
           "pairs_hashed_per_s": round(hashed / dt, 1), "ms_per_step": round(dt / steps * 1e3, 3), "steps": steps,
           "serial_ms_per_step": round(serial_dt / steps * 1e3, 3), "pipeline": pipe,
           "stored_packets": N, "stored_bytes": total, "mean_packet_bytes": round(total / N, 1),
           "max_packet_bytes": int(lengths.max().item()), "selected_rows_per_step": int(sel_rows),
           "lane_utilization": round(swork["blocks"] / max(swork["lane_slots"], 1), 4),
           "pair_test": {"avg_launch_us": round(kt["ms"] * 1e3 / max(kt["launches"], 1), 1),
                         "launches_per_step": round(kt["launches"] / steps, 1),
                         "gblocks_per_s": round(swork["blocks"] / (kt["ms"] / 1e3) / 1e9, 2) if kt["ms"] else None,
                         "hbm_gbs": round(swork["bytes"] / (kt["ms"] / 1e3) / 1e9, 1) if kt["ms"] else None}}
    del blob_full, blob, offsets, lengths, gt, meta, d_filters
    torch.cuda.empty_cache()
    return out


def responder_cpu(args, ctx, lib, store, reqs, claims, fblob, blob, offsets, h_gts, g_time, dev, label,
                  max_claims=1024, check=None):
    """The responder's CPU baseline (configs 2 and 5, the SHA-1 leg): oracle/sync_ref.respond_arrays -- numpy for
    the range / modulo predicate (faster than the reference's sqlite scan, so generous to the CPU), hashlib + Python
    for the lazy not_filter / byte-limit loop exactly as the reference (community.py:2555-2567) -- over the first
    claims of the step until >= --cpu-pairs (claim, packet) pairs are hashed (BASELINE.md:47), 1 core; the GPU's
    answers for the same claims (host-buffer dsy_sync_respond) checked against it; then every worker of the pool
    runs the same sample (rotated), one process per core.

    Only the packets the lazy loop touches travel to the host: a claim walks its selected rows in send order up to
    the packet that spends the budget (all of them when the budget is never spent), which the GPU's answer fixes.
    They are gathered on the GPU into one compact blob shared with the workers through /dev/shm."""
    import torch
    from oracle import sync_ref
    from oracle.bloom_ref import OracleBloom
    n_try = min(max_claims, len(claims))
    sub = (type(reqs[0]) * n_try)(*[reqs[i] for i in range(n_try)])
    out_off = np.zeros(n_try + 1, dtype=np.uint64)
    out = np.zeros(1 << 24, dtype=np.uint64)
    _native.check(lib.dsy_sync_respond(ctx.handle, store, sub, n_try, fblob, len(fblob),
                                       (_native.Meta * 1)(_native.Meta(1, 0, 0, 0, 0)), 1, g_time, 0, args.byte_limit,
                                       99, out.ctypes.data, len(out), out_off.ctypes.data))
    gpu = [out[int(out_off[j]):int(out_off[j + 1])].tolist() for j in range(n_try)]
    h_off = offsets.cpu().numpy()
    def walked(i):  # the rows the reference's lazy loop hashes for claim i (ASC meta, gt sorted by row)
        lo, hi, offset, modulo = claims[i][:4]
        a = int(np.searchsorted(h_gts, lo, side="left"))
        b = int(np.searchsorted(h_gts, hi, side="right"))
        sel = np.arange(a, b, dtype=np.int64)
        if modulo > 1 and b > a:
            sel = sel[(h_gts[a:b] + np.uint64(offset)) % np.uint64(modulo) == 0]
        sent = gpu[i]
        if sent and int((h_off[np.asarray(sent) + 1] - h_off[np.asarray(sent)]).sum()) >= args.byte_limit:
            sel = sel[:int(np.searchsorted(sel, sent[-1])) + 1]
        return sel

    touched, sample, pairs = [], [], 0
    for i in range(n_try):
        sel = walked(i)
        touched.append(sel)
        sample.append(i)
        pairs += len(sel)
        if pairs >= args.cpu_pairs:
            break
    work = {}
    if check:  # the claims the pool checks against the oracle as well (not timed)
        check = [i for i in check if i < n_try]
        for i in check:
            sel = walked(i)
            work[i] = len(sel)
            if i not in sample:
                touched.append(sel)
    rows = np.unique(np.concatenate(touched)) if touched else np.zeros(0, np.int64)
    d_rows = torch.from_numpy(rows).to(dev)
    st = offsets[d_rows]
    ln = offsets[d_rows + 1] - st
    co = torch.zeros(len(rows) + 1, dtype=torch.int64, device=dev)
    torch.cumsum(ln, 0, out=co[1:])
    total = int(co[-1].item())
    idx = torch.arange(total, device=dev, dtype=torch.int64) + torch.repeat_interleave(st - co[:-1], ln)
    s_blob, s_off, s_rows, s_gts = (Shared(blob[idx].cpu().numpy()), Shared(co.cpu().numpy()), Shared(rows),
                                    Shared(h_gts))
    del idx, d_rows, st, ln, co
    metas = [dict(name="bench", id=1, direction="ASC", priority=128, pruning=None)]
    byte_limit = args.byte_limit

    def prepare():
        cb, co_, rw, gts = s_blob.a, s_off.a, s_rows.a, s_gts.a
        pos = dict(zip(rw.tolist(), range(len(rw))))
        mv = memoryview(cb)
        packet_of = lambda r: mv[int(co_[pos[r]]):int(co_[pos[r] + 1])]  # noqa: E731
        return packet_of, {1: (np.arange(len(gts), dtype=np.int64), gts)}

    def run(order, packet_of, gt_by_meta, counter):
        return [sync_ref.respond_arrays(packet_of, gt_by_meta, metas, claims[i][:4],
                                        OracleBloom.from_bytes(claims[i][6], claims[i][4], claims[i][5]), g_time,
                                        byte_limit, False, counter) for i in order]

    packet_of, gt_by_meta = prepare()
    counter = [0]
    t0 = time.perf_counter()
    outs = run(sample, packet_of, gt_by_meta, counter)
    dt = time.perf_counter() - t0
    match = outs == gpu[:len(sample)]
    model, cores = cpu_info()

    def shard(w):
        p_of, gbm = prepare()
        order = sample[w % len(sample):] + sample[:w % len(sample)]
        cnt = [0]
        t1 = time.perf_counter()
        run(order, p_of, gbm, cnt)
        return cnt[0], time.perf_counter() - t1
    ncore = n_core_leg(shard, list(range(cores)), "packets/s",
                       "the same %d claims in every process (rotated), one process per core, same port"
                       % len(sample)) if match else None
    oracle_check = None
    if check and POOL is not None:
        # every checked claim through the oracle, one claim per worker task (heaviest first), against the GPU's answer
        def one(i):
            cb, co_, rw, gts = s_blob.a, s_off.a, s_rows.a, s_gts.a
            mv = memoryview(cb)

            def p_of(r):  # (the rows are sorted: a binary search, no per-task dict over millions of rows)
                j = int(np.searchsorted(rw, r))
                return mv[int(co_[j]):int(co_[j + 1])]

            class Rows(object):  # the store's rows are its index order
                def __getitem__(self, k):
                    return k
            cnt = [0]
            return i, run([i], p_of, {1: (Rows(), gts)}, cnt)[0], cnt[0]
        t1 = time.perf_counter()
        res = POOL.map(one, sorted(check, key=lambda i: -work[i]))
        oracle_check = {"claims": len(res), "pairs_hashed": int(sum(c for _, _, c in res)),
                        "gpu_matches_oracle": all(ans == gpu[i] for i, ans, _ in res),
                        "seconds": round(time.perf_counter() - t1, 2),
                        "how": "oracle/sync_ref.respond_arrays (hashlib) on the CpuPool workers, one claim per task"}
    return {"value": round(counter[0] / dt, 1), "unit": "packets/s", "cores": 1, "kind": "port", "cpu_model": model,
            "oracle_check": oracle_check,
            "sample": "%s: the first %d of the step's claims, %d (claim, packet) pairs hashed lazily as the reference "
                      "does (it stops at the packet that spends the %d B budget), through oracle/sync_ref.respond_arrays "
                      "+ oracle/bloom_ref (hashlib), %.1f s" % (label, len(sample), counter[0], byte_limit, dt),
            "pairs": counter[0], "seconds": round(dt, 2),
            "gpu_matches_cpu_on_sample": match, "n_core": ncore}


from dispersy_amd import _native  # noqa: E402  (module-level name used in cpu_baseline)

if __name__ == "__main__":
    main()

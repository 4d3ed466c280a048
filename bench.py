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
    ap.add_argument("--cpu-claims", type=int, default=96, help="claims in the CPU-baseline sample (0: skip)")
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--sim-peers", type=int, default=1_000_000, help="config 3 gossip simulator peers (0: skip)")
    ap.add_argument("--sim-universe", type=int, default=10_000)
    ap.add_argument("--sim-initial", type=int, default=100)
    ap.add_argument("--sim-rounds", type=int, default=10)
    ap.add_argument("--sim-warmup", type=int, default=2)
    return ap.parse_args()


def main():
    args = parse()
    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from dispersy_amd import _native
    from dispersy_amd.bloomfilter import BloomFilter

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
    cap_probe = BloomFilter(args.filter_bits, args.error_rate)
    capacity = cap_probe.get_capacity(args.error_rate)
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
        prefix = bytes([int(rng.integers(0, 256))])
        bf = BloomFilter(args.filter_bits, args.error_rate, prefix)
        known = rows[rng.random(len(rows)) >= 0.01]  # the requester misses 1 % of its range
        buf = ctypes.create_string_buffer(bf.bytes, len(bf.bytes))
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

    p_out, p_off, pairs = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()

    def step():
        _native.check(lib.dsy_sync_respond_dev(ctx.handle, store, reqs, R, d_filters.data_ptr(), metas, 1, N, 0,
                                               args.byte_limit, 99, ctypes.byref(p_out), ctypes.byref(p_off),
                                               ctypes.byref(pairs)))

    for _ in range(args.warmup):
        step()
    ctx.synchronize()
    ctx.reset_timing()
    ctx.set_timing(True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    total_pairs = 0
    for _ in range(args.steps):
        step()
        total_pairs += pairs.value
    ctx.synchronize()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_timing(False)
    kt = ctx.kernel_time(_native.TIME_PAIR_TEST)
    sel = ctx.kernel_time(_native.TIME_SELECT)
    cmp_ = ctx.kernel_time(_native.TIME_COMPACT)
    if dist:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        p = torch.tensor([total_pairs], device=dev, dtype=torch.int64)
        dist.all_reduce(p, op=dist.ReduceOp.SUM)
        total_pairs = int(p.item())

    # ---------------------------------------------------------------- roofline of the dominant kernel
    launches = max(kt["launches"], 1)
    avg_s = kt["ms"] / 1e3 / launches
    pairs_per_launch = total_pairs / max(args.steps, 1) / max(world, 1)
    blocks_per_launch = kt["blocks"] / launches
    bytes_per_launch = kt["bytes"] / launches + pairs_per_launch * 25  # packet bytes + offsets/row/flag per pair
    hash_name = cap_probe.hash_name
    roofline = {
        "kernel": "k_pair_test<%s>" % hash_name,
        "bound": "hbm",
        "achieved": round(bytes_per_launch / avg_s / 1e9, 1),
        "peak": PEAK_HBM_GBS,
        "unit": "GB/s",
        "frac": round(bytes_per_launch / avg_s / 1e9 / PEAK_HBM_GBS, 4),
        "traffic": None,
        "avg_launch_us": round(avg_s * 1e6, 2),
        "launches": kt["launches"],
        "valu_int32": {
            "achieved": round(blocks_per_launch * OPS_PER_BLOCK[hash_name] / avg_s / 1e12, 2),
            "peak": PEAK_INT32_TOPS, "unit": "Tops/s",
            "frac": round(blocks_per_launch * OPS_PER_BLOCK[hash_name] / avg_s / 1e12 / PEAK_INT32_TOPS, 4),
            "ops_per_block": OPS_PER_BLOCK[hash_name], "blocks_per_launch": int(blocks_per_launch)},
        "other_kernels_ms_per_step": {"select": round(sel["ms"] / max(args.steps, 1), 3),
                                      "compact": round(cmp_["ms"] / max(args.steps, 1), 3)},
    }
    traffic_file = os.path.join(ROOT, "profiles", "pmc_traffic_%s.json" % hash_name)
    if os.path.isfile(traffic_file):
        with open(traffic_file) as f:
            roofline["traffic"] = json.load(f).get("hbm_bytes_per_launch")

    gossip = None
    if args.sim_peers > 0:
        gossip = gossip_sim(args, ctx, dev, rank, world, dist)

    cpu = None
    if rank == 0 and world == 1 and args.cpu_claims > 0:
        cpu = cpu_baseline(args, ctx, lib, store, reqs, claims, blob, offsets, total_bytes, N, fblob)

    if rank == 0:
        line = {
            "metric": "packets hashed+tested/sec",
            "value": round(total_pairs / elapsed, 1),
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
            "roofline": roofline,
            "cpu_baseline": cpu,
            "gossip_sim": gossip,
        }
        print(json.dumps(line))
    lib.dsy_store_free(store)
    if dist:
        dist.destroy_process_group()


def gossip_sim(args, ctx, dev, rank, world, dist):
    """BASELINE config 3: the epidemic-sync simulator (dispersy_amd/sim.py) -- P peers block-sharded over the
    ranks, one gossip round = every peer claims (MTU filter over its store), every claim is answered, every peer
    stores what it got; two RCCL all-to-all(v) exchanges per round.  Total work is fixed (strong scaling)."""
    import torch
    from dispersy_amd.sim import EpidemicSim, GpuEngine, make_config, make_universe
    blob, offs = make_universe(args.sim_universe, seed=11)
    cfg = make_config(args.sim_peers, args.sim_universe, rank, world, seed=11)
    eng = GpuEngine(cfg, blob, offs, dev, ctx=ctx)
    eng.seed(args.sim_initial)
    sim = EpidemicSim(eng, cfg, rank, world, dist, dev)
    held0 = sim.global_stats()[0]
    for r in range(args.sim_warmup):
        sim.round(r)
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
    if dist:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    held, chk = sim.global_stats()
    return {"metric": "gossip sync rounds/sec", "value": round(args.sim_rounds / dt, 3), "unit": "rounds/s",
            "n_gpus": world, "scaling": "strong", "rounds": args.sim_rounds, "warmup_rounds": args.sim_warmup,
            "ms_per_round": round(dt / args.sim_rounds * 1e3, 3),
            "config": {"peers": args.sim_peers, "universe": args.sim_universe, "initial_packets": args.sim_initial,
                       "filter": "m=%d k=%d md5" % (cfg.m_bits, cfg.k), "byte_limit": cfg.byte_limit},
            "packets_held_start": held0, "packets_held_end": held, "store_checksum": "%016x" % chk,
            "exchange_bytes_rank0": sim.exchanged_bytes}


def cpu_baseline(args, ctx, lib, store, reqs, claims, blob, offsets, total_bytes, N, fblob):
    """The oracle's CPU port of the responder (hashlib + Python, one core) on a bounded sample of the same claims,
    with the GPU's answers for those claims checked against it."""
    from oracle import sync_ref
    from oracle.bloom_ref import OracleBloom
    host_blob = memoryview(blob[:total_bytes].cpu().numpy())
    host_off = offsets.cpu().numpy()
    rows = np.arange(N, dtype=np.int64)
    gts = np.arange(1, N + 1, dtype=np.uint64)
    gt_by_meta = {1: (rows, gts)}
    packet_of = lambda r: host_blob[int(host_off[r]):int(host_off[r + 1])]  # noqa: E731
    metas = [dict(name="bench", id=1, direction="ASC", priority=128, pruning=None)]
    k = args.cpu_claims
    sample = list(range(0, min(k, len(claims))))
    counter = [0]
    outs = []
    t0 = time.perf_counter()
    for i in sample:
        lo, hi, offset, modulo, kf, prefix, raw = claims[i]
        ob = OracleBloom.from_bytes(raw, kf, prefix)
        outs.append(sync_ref.respond_arrays(packet_of, gt_by_meta, metas, (lo, hi, offset, modulo), ob, N,
                                            args.byte_limit, False, counter))
    dt = time.perf_counter() - t0
    # the GPU's answer for the same claims, through the host-buffer C-ABI entry point
    sub = (type(reqs[0]) * len(sample))(*[reqs[i] for i in sample])
    out_off = np.zeros(len(sample) + 1, dtype=np.uint64)
    out = np.zeros(1 << 20, dtype=np.uint64)
    _native.check(lib.dsy_sync_respond(ctx.handle, store, sub, len(sample), fblob, len(fblob),
                                       (_native.Meta * 1)(_native.Meta(1, 0, 0, 0, 0)), 1, N, 0, args.byte_limit, 99,
                                       out.ctypes.data, len(out), out_off.ctypes.data))
    gpu = [out[int(out_off[j]):int(out_off[j + 1])].tolist() for j in range(len(sample))]
    return {"value": round(counter[0] / dt, 1), "unit": "packets/s", "cores": 1, "kind": "port",
            "sample": "%d of the step's claims (%d pairs hashed lazily, as the reference stops at the byte limit) "
                      "through oracle/sync_ref.respond_arrays + oracle/bloom_ref (hashlib), %.1f s"
                      % (len(sample), counter[0], dt),
            "gpu_matches_cpu_on_sample": gpu == outs}


from dispersy_amd import _native  # noqa: E402  (module-level name used in cpu_baseline)

if __name__ == "__main__":
    main()

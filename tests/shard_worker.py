"""One rank of test_shard_gpu.py's two-rank run (test infrastructure): gloo over 127.0.0.1, both ranks on cuda:0.
Runs the three sharded jobs of dispersy_amd/shard.py through the HIP path and writes what it saw to $SHARD_OUT
(JSON); rank 0 also runs each job as a single process and records whether the two agree.

cfg4: 40 k keys split over the ranks, add_sharded into MD5 / SHA-1 / SHA-256 (2^20, 2^24) filters -> the union.
cfg2: 48 claims split over the ranks, SyncCommunity.respond on the replicated store -> rows in rank order.
cfg3: EpidemicSim with GpuEngines on block-sharded peers, two all-to-all(v) exchanges per round."""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(HERE, "golden"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FILTERS = [(10160, 0.01, b"\x00\x01\x02\x03"), (4096, 0.001, b"x"), (1 << 20, 0.01, b"\x07"), (1 << 24, 0.01, b"\x07")]


def cfg4(ctx, coll, dev):
    from dispersy_amd import BloomFilter, _native
    from dispersy_amd.shard import add_sharded
    from keys import random_packets
    blob, offs = random_packets(77, 40_000, 60, 1500)
    G = _native.BLOB_GUARD
    d_blob = torch.zeros(len(blob) + 2 * G, dtype=torch.uint8, device=dev)
    d_blob[G:G + len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
    d_offs = torch.from_numpy(offs.astype(np.int64)).to(dev)
    out = {}
    for m, f, prefix in FILTERS:
        bf = BloomFilter(m, f, prefix)
        filt = torch.zeros(int(ctx.lib.dsy_filter_words(m)), dtype=torch.int32, device=dev)
        union = add_sharded(ctx, bf.params, d_blob[G:], d_offs, len(offs) - 1, coll, filt)
        got = union.cpu().numpy().tobytes()[:m // 8]
        row = {"sha": hashlib.sha256(got).hexdigest(), "bits": int(np.unpackbits(np.frombuffer(got, np.uint8)).sum()),
               "partial_bits": int(np.unpackbits(filt.cpu().numpy().view(np.uint8)[:m // 8]).sum())}
        if coll.rank == 0:
            whole = BloomFilter(m, f, prefix)
            whole.add_packed(blob, offs)
            row["equal_single"] = whole.bytes == got
        out["%d/%s" % (m, f)] = row
    return out


def cfg2(coll):
    from dispersy_amd import BloomFilter
    from dispersy_amd.community import ClaimRequest, SyncCommunity
    from dispersy_amd.distribution import MetaMessage, SyncDistribution
    from dispersy_amd.shard import shard_range
    from dispersy_amd.store import SyncStore
    rng = np.random.Generator(np.random.PCG64(41))
    n = 30_000
    gts = rng.integers(1, 20_000, size=n)
    rows = [(i + 1, int(gts[i]), 1 + int(i % 3 == 0), 0, i.to_bytes(4, "big") + rng.bytes(int(rng.integers(20, 400))))
            for i in range(n)]
    store = SyncStore.from_rows(rows)
    metas = [MetaMessage("a", 1, SyncDistribution("ASC", 128)), MetaMessage("d", 2, SyncDistribution("DESC", 200))]
    com = SyncCommunity(store, metas, global_time=20_000)
    claims = []
    for i in range(48):
        lo = int(rng.integers(1, 19_000))
        hi = lo + int(rng.integers(100, 3000))
        modulo = int(rng.integers(1, 5))
        bf = BloomFilter(10160, 0.01, bytes([i]))
        sel = [r[4] for r in rows if lo <= r[1] <= hi]
        bf.add_keys(sel[::3])
        claims.append(ClaimRequest(lo, hi, modulo, int(rng.integers(0, modulo)), bf))
    lo, hi = shard_range(len(claims), coll.rank, coll.world)
    mine = [store.rowid[r].tolist() for r in com.respond(claims[lo:hi], byte_limit=20_000)]
    gathered = coll.all_gather_object(mine)
    out = {"claims": [lo, hi], "rows_sent": sum(map(len, mine))}
    if coll.rank == 0:
        single = [store.rowid[r].tolist() for r in com.respond(claims, byte_limit=20_000)]
        out["equal_single"] = [x for per in gathered for x in per] == single
        out["rows_all"] = sum(map(len, single))
    return out


def cfg3(coll, dev):
    from dispersy_amd.sim import EpidemicSim, GpuEngine, make_config, make_universe
    P, U, INITIAL, ROUNDS = 1500, 3000, 40, 4
    blob, offs = make_universe(U, seed=4)

    def run(rank, world, d, chunks=1):
        cfg = make_config(P, U, rank, world, seed=13, chunks=chunks)
        eng = GpuEngine(cfg, blob, offs, dev)
        eng.seed(INITIAL)
        sim = EpidemicSim(eng, cfg, rank, world, d, dev, chunks=chunks)
        hist = [list(sim.global_stats())]
        for r in range(ROUNDS):
            sim.round(r)
            hist.append(list(sim.global_stats()))
        return hist, sim.exchanged_bytes

    hist, moved = run(coll.rank, coll.world, dist)
    chunked, _ = run(coll.rank, coll.world, dist, chunks=3)  # peers in chunks as virtual ranks (gloo: synchronous)
    out = {"history": hist, "exchanged_bytes": moved, "chunked_equal": chunked == hist}
    if coll.rank == 0:
        single, _ = run(0, 1, None)
        out["equal_single"] = hist == single
    return out


def main():
    from dispersy_amd import _native
    from dispersy_amd.shard import Collectives
    dist.init_process_group("gloo")
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        ctx = _native.default_context()
        coll = Collectives(dist)
        res = {"rank": coll.rank, "world": coll.world, "cfg4": cfg4(ctx, coll, dev), "cfg2": cfg2(coll),
               "cfg3": cfg3(coll, dev)}
        coll.barrier()
    finally:
        dist.destroy_process_group()
    with open(os.environ["SHARD_OUT"], "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()

"""The sharded jobs' host logic (dispersy_amd/shard.py) on CPU: the block split, and world_size 2 over
gloo for cfg2 (claims split over the ranks, store replicated: the ranks' answers in rank order are the single
process's) and cfg4 (keys split, partial filters all-gathered and OR-ed: the union is the filter of all keys).
The per-rank compute here is the oracle -- the HIP path of the same jobs runs two ranks on one GPU in
test_shard_gpu.py."""
import os
import socket
import sqlite3

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dispersy_amd.shard import Collectives, shard_range
from keys import packet_list
from oracle import sync_ref
from oracle.bloom_ref import OracleBloom
from golden_util import SYNC_SCHEMA


@pytest.mark.parametrize("n", [0, 1, 7, 64, 1000, 1023])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_range_partitions(n, world):
    spans = [shard_range(n, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    sizes = [hi - lo for lo, hi in spans]
    assert max(sizes) - min(sizes) <= 1 and sizes == sorted(sizes, reverse=True)


def test_shard_range_rejects_bad_rank():
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


METAS = [dict(name="a", id=1, direction="ASC", priority=128, pruning=None)]


def _store(n):
    rng = np.random.Generator(np.random.PCG64(17))
    conn = sqlite3.connect(":memory:")
    conn.executescript(SYNC_SCHEMA)
    conn.executemany("INSERT INTO sync(id, community, member, global_time, meta_message, undone, packet, sequence) "
                     "VALUES (?, 1, ?, ?, 1, 0, ?, 0)",
                     [(i + 1, i + 1, int(rng.integers(1, 400)), rng.bytes(int(rng.integers(20, 200))))
                      for i in range(n)])
    return conn


def _claims(conn, n):
    rng = np.random.Generator(np.random.PCG64(23))
    out = []
    for i in range(n):
        lo = int(rng.integers(1, 300))
        modulo = int(rng.integers(1, 4))
        bloom = OracleBloom.from_m_f(1024, 0.01, bytes([i & 0xFF]))
        known = [bytes(p) for (p,) in conn.execute("SELECT packet FROM sync WHERE global_time BETWEEN ? AND ?",
                                                    (lo, lo + 60))]
        bloom.add_keys(known[::2])
        out.append(((lo, lo + 80, int(rng.integers(0, modulo)), modulo), bloom))
    return out


def cfg2_answers(rank, world, n_claims=37):
    conn = _store(2000)
    claims = _claims(conn, n_claims)
    lo, hi = shard_range(n_claims, rank, world)
    return [sync_ref.respond_lists(conn, METAS, req, bloom, 400, 5000) for req, bloom in claims[lo:hi]]


def cfg4_partial(rank, world, m=10160, n_keys=3001):
    keys = packet_list(31, n_keys, 40, 600)
    lo, hi = shard_range(n_keys, rank, world)
    ref = OracleBloom.from_m_f(m, 0.01, b"\x07")
    ref.add_keys(keys[lo:hi])
    raw = ref.to_bytes() + b"\x00" * ((-(m // 8)) % 4)
    return torch.from_numpy(np.frombuffer(raw, dtype=np.int32).copy())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        coll = Collectives(dist)
        answers = coll.all_gather_object(cfg2_answers(rank, world))
        partial = cfg4_partial(rank, world)
        parts = torch.empty(world * partial.numel(), dtype=torch.int32)
        coll.all_gather_into(parts, partial)
        union = np.bitwise_or.reduce(parts.view(world, -1).numpy(), axis=0)
        pairs = coll.scalar(sum(len(a) for a in answers[rank]), "sum")
        slowest = coll.scalar(float(rank + 1), "max")
        if rank == 0:
            q.put(([x for per in answers for x in per], union.tobytes(), pairs, slowest))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_ranks_equal_one(world):
    """2, 4 and 8 ranks (the driver's 8-GPU shape) over gloo: cfg2's answers in rank order and cfg4's union filter are
    the single process's."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    answers, union, pairs, slowest = q.get(timeout=600)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single = cfg2_answers(0, 1)
    assert answers == single and sum(map(len, single)) > 50
    assert pairs == sum(map(len, single)) and slowest == float(world)
    assert union == cfg4_partial(0, 1).numpy().tobytes()

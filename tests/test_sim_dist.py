"""The epidemic simulator's multi-rank path (block-sharded peers, two all-to-all(v) exchanges per round) on CPU:
world sizes 2, 4 and 8 (the driver's 8-GPU shape) over gloo with the oracle CPU engine must reproduce world_size 1
exactly, with whole rounds and with the chunked round (peers in chunks as virtual ranks, EpidemicSim.chunks)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dispersy_amd.sim import EpidemicSim, make_config, make_universe
from oracle.sim_ref import OracleEngine

P, U, INITIAL, ROUNDS = 240, 600, 12, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def run_sim(rank, world, dist_mod=None, byte_limit=2000, chunks=1, exchanged=None):
    blob, offs = make_universe(U, seed=3)
    cfg = make_config(P, U, rank, world, bits=2048, error_rate=0.01, byte_limit=byte_limit, seed=5, chunks=chunks)
    eng = OracleEngine(cfg, blob, offs)
    eng.seed(INITIAL)
    sim = EpidemicSim(eng, cfg, rank, world, dist_mod, torch.device("cpu"), chunks=chunks)
    history = [sim.global_stats()]
    for r in range(ROUNDS):
        sim.round(r)
        history.append(sim.global_stats())
    if exchanged is not None:
        exchanged.append((sim.exchanged_bytes, sim.exchanged_remote))
    return history


def _worker(rank, world, port, q, chunks):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ex = []
        h = run_sim(rank, world, dist, chunks=chunks, exchanged=ex)
        q.put((rank, h, ex[0]))
    finally:
        dist.destroy_process_group()


_SINGLE = {}


def _single():
    if "h" not in _SINGLE:
        _SINGLE["h"] = run_sim(0, 1)
    return _SINGLE["h"]


@pytest.mark.parametrize("world,chunks", [(2, 1), (4, 1), (8, 1), (2, 3), (8, 2)])
def test_ranks_equal_one(world, chunks):
    single = _single()
    assert single[-1][0] > single[0][0]  # packets spread
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, chunks)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (h, ex)) for r, h, ex in (q.get(timeout=600) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert got[r][0] == single, (world, chunks, r)
    # every claim and response record crosses once: what the ranks sent is the whole round's records
    sent = sum(got[r][1][0] for r in range(world))
    blob, offs = make_universe(U, seed=3)
    cfg = make_config(P, U, 0, 1, bits=2048, seed=5)
    assert sent == ROUNDS * P * (cfg.claim_bytes + cfg.resp_bytes)
    assert 0 < sum(got[r][1][1] for r in range(world)) < sent


@pytest.mark.parametrize("chunks", [2, 4, 5])
def test_chunked_round_one_rank_equals_whole(chunks):
    """The chunked round at one rank (no exchange): chunk-wise builds over virtual ranks, responds and one merge at
    the end give the whole round's stores."""
    assert run_sim(0, 1, chunks=chunks) == _single()


def test_sim_config_matches_community_filter():
    cfg = make_config(1_000_000, 10_000, 0, 8)
    assert (cfg.m_bits, cfg.k, cfg.hash_kind, cfg.chunk_bytes) == (10160, 7, 0, 2)  # MD5 MTU filter
    assert cfg.capacity == 1059
    assert cfg.peers_per_rank == 125_000 and cfg.peer_end == 125_000


def test_claim_matrix_rows_are_each_ranks_counts():
    """Every rank computes the same [src, dst] matrix (dsy_sim_claim_matrix restated): row r is what rank r's
    claim_counts returns, column r what it receives, so the exchange needs no count all-to-all."""
    blob, offs = make_universe(50, seed=3)
    for world in (1, 2, 3):
        engs = [OracleEngine(make_config(P, 50, r, world, bits=2048, seed=5), blob, offs) for r in range(world)]
        for rnd in range(3):
            mats = [e.claim_matrix(rnd, world) for e in engs]
            for m in mats[1:]:
                assert (m == mats[0]).all()
            for r, e in enumerate(engs):
                assert (mats[0][r] == e.claim_counts(rnd, world)).all()
            assert int(mats[0].sum()) == P

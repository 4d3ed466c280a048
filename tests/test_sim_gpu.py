"""The epidemic simulator's HIP kernels (dsy_sim_*) against the oracle CPU engine, peer by peer, and a two-rank
exchange emulated in one process (records routed by hand) against the single-rank run."""
import numpy as np
import pytest
import torch

from dispersy_amd.sim import EpidemicSim, GpuEngine, make_config, make_universe
from oracle.sim_ref import OracleEngine

pytestmark = pytest.mark.gpu

P, U, INITIAL, ROUNDS = 1500, 3000, 40, 4


def test_gpu_engine_matches_oracle_engine():
    blob, offs = make_universe(U, seed=3)
    dev = torch.device("cuda", 0)
    cg = make_config(P, U, 0, 1, seed=9)
    co = make_config(P, U, 0, 1, seed=9)
    g, o = GpuEngine(cg, blob, offs, dev), OracleEngine(co, blob, offs)
    g.seed(INITIAL)
    o.seed(INITIAL)
    sg, so = EpidemicSim(g, cg, device=dev), EpidemicSim(o, co)
    assert sg.global_stats() == so.global_stats()
    for r in range(ROUNDS):
        sg.round(r)
        so.round(r)
        assert sg.global_stats() == so.global_stats(), r
    gb = g.bits.cpu().numpy().view(np.uint32).reshape(P, cg.words)
    assert (gb == o.bitsets()).all()
    # the GPU tests whole 64-packet chunks before it stops at the budget; the CPU engine stops packet by packet
    assert sg.tested >= so.tested


def test_gpu_engine_matches_oracle_at_bench_shape():
    """The bench's gossip configuration (universe 10 000 packets, 100 initial per peer, MTU filters, 5 KiB budget) at
    20 000 peers -- 13x the peers above, where every peer's store is near the filter's capacity by the second round --
    against the oracle engine, peer by peer, for two rounds (the 1 M-peer bench run is checked by its store checksum
    only; the oracle takes ~18 s per round here)."""
    p, u, initial = 20_000, 10_000, 100
    blob, offs = make_universe(u, seed=5)
    dev = torch.device("cuda", 0)
    cg = make_config(p, u, 0, 1, seed=21)
    co = make_config(p, u, 0, 1, seed=21)
    g, o = GpuEngine(cg, blob, offs, dev), OracleEngine(co, blob, offs)
    g.seed(initial)
    o.seed(initial)
    sg, so = EpidemicSim(g, cg, device=dev), EpidemicSim(o, co)
    for r in range(2):
        sg.round(r)
        so.round(r)
        assert sg.global_stats() == so.global_stats(), r
    gb = g.bits.cpu().numpy().view(np.uint32).reshape(p, cg.words)
    assert (gb == o.bitsets()).all()


def test_two_rank_routing_in_one_process():
    """Two GpuEngines own halves of the peers; their records are exchanged by slicing, as all_to_all_single does."""
    blob, offs = make_universe(U, seed=4)
    dev = torch.device("cuda", 0)
    single_cfg = make_config(P, U, 0, 1, seed=13)
    single = GpuEngine(single_cfg, blob, offs, dev)
    single.seed(INITIAL)
    ss = EpidemicSim(single, single_cfg, device=dev)
    cfgs = [make_config(P, U, r, 2, seed=13) for r in range(2)]
    engs = [GpuEngine(c, blob, offs, dev) for c in cfgs]
    for e in engs:
        e.seed(INITIAL)

    def exchange(bufs, counts, rec):
        # bufs[r] holds records grouped by destination; counts[r][d] records from r to d
        out = []
        for d in range(2):
            parts = []
            for r in range(2):
                start = int(sum(counts[r][:d])) * rec
                parts.append(bufs[r][start:start + int(counts[r][d]) * rec])
            out.append(torch.cat(parts) if sum(p.numel() for p in parts) else torch.empty(1, dtype=torch.uint8, device=dev))
        return out, [int(sum(counts[r][d] for r in range(2))) for d in range(2)]

    for rnd in range(ROUNDS):
        ss.round(rnd)
        counts = [e.claim_counts(rnd, 2) for e in engs]
        # the matrix every rank computes for itself holds each rank's send counts as its row
        for e in engs:
            assert (e.claim_matrix(rnd, 2) == np.stack(counts)).all()
        bufs = [e.build_claims(rnd, np.concatenate([[0], np.cumsum(c)[:-1]]), int(c.sum())) for e, c in zip(engs, counts)]
        for e in engs:  # the calls only enqueue on each engine's stream; the hand-made exchange below runs on torch's
            e.sync()
        claims_in, n_in = exchange(bufs, counts, cfgs[0].claim_bytes)
        pcounts = [e.resp_counts(ci, n, 2) for e, ci, n in zip(engs, claims_in, n_in)]
        # one response per claim: the counts going back are the received claims' counts by source rank
        assert [list(pc) for pc in pcounts] == [[int(counts[r][d]) for r in range(2)] for d in range(2)]
        rbufs = [e.respond(ci, n, np.concatenate([[0], np.cumsum(pc)[:-1]]), int(pc.sum()))[0]
                 for e, ci, n, pc in zip(engs, claims_in, n_in, pcounts)]
        for e in engs:
            e.sync()
        resps_in, r_in = exchange(rbufs, pcounts, cfgs[0].resp_bytes)
        for e, ri, n in zip(engs, resps_in, r_in):
            e.merge(ri, n)
        held = sum(e.stats()[0] for e in engs)
        chk = 0
        for e in engs:
            chk ^= e.stats()[1] & 0x7fffffffffffffff
        assert (held, chk) == ss.global_stats(), rnd


@pytest.mark.parametrize("chunks", [2, 3])
def test_chunked_round_gpu_equals_whole(chunks):
    """The chunked round (EpidemicSim.chunks: chunk-wise claim builds over virtual ranks, dsy_sim_build_claims on a
    chunk's config and bits) on the GPU engine at one rank gives the whole round's stores, round after round."""
    blob, offs = make_universe(U, seed=5)
    dev = torch.device("cuda", 0)
    cw, cc = make_config(P, U, 0, 1, seed=17), make_config(P, U, 0, 1, seed=17, chunks=chunks)
    ew, ec = GpuEngine(cw, blob, offs, dev), GpuEngine(cc, blob, offs, dev)
    ew.seed(INITIAL)
    ec.seed(INITIAL)
    sw, sc = EpidemicSim(ew, cw, device=dev), EpidemicSim(ec, cc, device=dev, chunks=chunks)
    for r in range(ROUNDS):
        sw.round(r)
        sc.round(r)
        assert sc.global_stats() == sw.global_stats(), r
    assert (ec.bits.cpu().numpy() == ew.bits.cpu().numpy()).all()

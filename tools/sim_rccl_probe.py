#!/usr/bin/env python3
"""The simulator's overlapped round over RCCL on a one-GPU box (not part of the product): a one-rank torchrun job
joins an "nccl" (RCCL) group and runs EpidemicSim with chunks (exchanges on a communication stream, the engine's
kernels waiting on per-exchange events, dsy_ctx_wait_event) and exchange_always, so every claim and response record
goes through RCCL all-to-all(v) even at one rank; the per-round (packets held, checksum) history must equal the plain
one-process round's.  Prints one JSON line.
    python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 --master-port P tools/sim_rccl_probe.py"""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dispersy_amd.sim import EpidemicSim, GpuEngine, make_config, make_universe  # noqa: E402

P, U, INITIAL, ROUNDS = 3000, 3000, 40, 5


def run(dev, chunks, d):
    blob, offs = make_universe(U, seed=4)
    cfg = make_config(P, U, 0, 1, seed=13, chunks=chunks)
    eng = GpuEngine(cfg, blob, offs, dev)
    eng.seed(INITIAL)
    sim = EpidemicSim(eng, cfg, 0, 1, d, dev, chunks=chunks, exchange_always=d is not None)
    hist = [list(sim.global_stats())]
    for r in range(ROUNDS):
        sim.round(r)
        hist.append(list(sim.global_stats()))
    eng.sync()
    return hist, sim.exchanged_bytes, sim._overlapped()


def main():
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl")
    whole, _, _ = run(dev, 1, None)
    out = {"backend": dist.get_backend(), "whole": whole}
    for chunks in (1, 4):
        hist, moved, overlapped = run(dev, chunks, dist)
        out["chunks%d" % chunks] = {"equal": hist == whole, "exchanged_bytes": moved, "overlapped": overlapped}
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

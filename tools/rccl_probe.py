#!/usr/bin/env python3
"""RCCL probe on a one-GPU box (not part of the product): every rank of a torchrun job binds cuda:0, joins an "nccl"
(RCCL) group and runs the collectives dispersy_amd.shard.Collectives issues, with the dtypes the jobs pass (int64 /
float64 scalars, int32 and int64 all-gathers, uint8 all-to-all(v) with byte splits).  Prints one JSON line per rank.
Two ranks on one GPU show whether this RCCL build accepts them at all; one rank checks the calls and dtypes.
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P tools/rccl_probe.py"""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dispersy_amd.shard import Collectives  # noqa: E402


def main():
    torch.cuda.set_device(0)
    dist.init_process_group("nccl")
    coll = Collectives(dist)
    r, w = coll.rank, coll.world
    dev = torch.device("cuda", 0)
    out = {"rank": r, "world": w, "backend": dist.get_backend()}
    out["sum_i64"] = coll.scalar(r + 1, "sum", device=dev)
    out["max_f64"] = coll.scalar(0.5 + r, "max", device=dev)
    parts = torch.empty(w * 3, dtype=torch.int32, device=dev)
    coll.all_gather_into(parts, torch.tensor([r, 10 + r, 20 + r], dtype=torch.int32, device=dev))
    out["gather_i32"] = parts.tolist()
    p64 = torch.empty(w, dtype=torch.int64, device=dev)
    coll.all_gather_into(p64, torch.tensor([2 ** 40 + r], dtype=torch.int64, device=dev))
    out["gather_i64"] = p64.tolist()
    # all-to-all(v) of bytes: rank r sends (d + 1) * 3 + r bytes of value 16 r + d to rank d
    send = [(d + 1) * 3 + r for d in range(w)]
    recv = [(r + 1) * 3 + s for s in range(w)]
    inp = torch.cat([torch.full((send[d],), 16 * r + d, dtype=torch.uint8, device=dev) for d in range(w)])
    got = torch.empty(sum(recv), dtype=torch.uint8, device=dev)
    coll.all_to_all_single(got, inp, recv, send)
    want = torch.cat([torch.full((recv[s],), 16 * s + r, dtype=torch.uint8, device=dev) for s in range(w)])
    out["a2av_ok"] = bool(torch.equal(got, want))
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

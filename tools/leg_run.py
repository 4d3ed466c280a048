#!/usr/bin/env python3
"""Run ONE of bench.py's legs alone, so a rocprofv3 pass sees only that leg's launches (config 5's k_pair_test<md5> is
the same kernel as the headline's).  Prints the leg's JSON record.

usage: python tools/leg_run.py 5 [bench.py options]     (config 5, the heavy-tailed store; --cpu-claims 0 implied)
       DSY_LEG_RANK=r: the claims rank r of a multi-GPU run draws (its seed), in this one process
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    leg = sys.argv[1]
    sys.argv = [sys.argv[0]] + sys.argv[2:] + ["--cpu-claims", "0"]
    import bench
    args = bench.parse()
    import torch
    from dispersy_amd import _native
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    ctx = _native.Context(0)
    if leg == "5":
        out = bench.heavy_tail(args, ctx, ctx.lib, dev, int(os.environ.get("DSY_LEG_RANK", "0")), 1, None)
    else:
        raise SystemExit("unknown leg %r" % leg)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

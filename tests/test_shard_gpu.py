"""The sharded jobs (dispersy_amd/shard.py) with two ranks on the MI355X: tests/shard_worker.py is
started twice as a child process (gloo over 127.0.0.1, both ranks on cuda:0 -- the exchange is staged through host
memory, the hashing, OR-reduce, responder and simulator kernels run on the GPU), and every job must equal the
single-process run: cfg4's union filter bytes (MD5, SHA-1, SHA-256 at 2^20 and 2^24), cfg2's answers in claim
order, cfg3's per-round (packets held, checksum) history."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.fixture(scope="module")
def two_ranks(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("shard")
    port = str(_free_port())
    procs, outs = [], []
    for rank in range(2):
        out = str(tmp / ("rank%d.json" % rank))
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port, SHARD_OUT=out)
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "shard_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
        outs.append(out)
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=100)[0].decode(errors="replace"))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]
    res = []
    for out in outs:
        with open(out) as f:
            res.append(json.load(f))
    return res


def test_cfg4_union_equals_single_build(two_ranks):
    r0, r1 = two_ranks
    for name, row in r0["cfg4"].items():
        assert row["equal_single"], name
        assert row["sha"] == r1["cfg4"][name]["sha"], name  # every rank holds the same union
        assert row["bits"] >= max(row["partial_bits"], r1["cfg4"][name]["partial_bits"]), name


def test_cfg2_claims_sharded_equal_single(two_ranks):
    r0, r1 = two_ranks
    assert r0["cfg2"]["equal_single"]
    assert r0["cfg2"]["claims"][1] == r1["cfg2"]["claims"][0] and r1["cfg2"]["claims"][1] == 48
    assert r0["cfg2"]["rows_sent"] + r1["cfg2"]["rows_sent"] == r0["cfg2"]["rows_all"] > 0


def test_cfg3_sim_two_ranks_equal_one(two_ranks):
    r0, r1 = two_ranks
    assert r0["cfg3"]["equal_single"]
    assert r0["cfg3"]["history"] == r1["cfg3"]["history"]
    assert r0["cfg3"]["history"][-1][0] > r0["cfg3"]["history"][0][0]
    assert r0["cfg3"]["exchanged_bytes"] > 0 and r1["cfg3"]["exchanged_bytes"] > 0
    assert r0["cfg3"]["chunked_equal"] and r1["cfg3"]["chunked_equal"]


def test_cfg4_one_rank_add_sharded_equals_single_build():
    """The world == 1 path of add_sharded / union_filter (no collective): the filter torch zeroed is built on the
    ctx stream and cloned on torch's stream, ordered by device events both ways."""
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from dispersy_amd import BloomFilter, _native
    from dispersy_amd.shard import add_sharded
    from keys import random_packets
    dev = torch.device("cuda", 0)
    ctx = _native.default_context()
    blob, offs = random_packets(78, 30_000, 60, 1500)
    G = _native.BLOB_GUARD
    d_blob = torch.zeros(len(blob) + 2 * G, dtype=torch.uint8, device=dev)
    d_blob[G:G + len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
    d_offs = torch.from_numpy(offs.astype(np.int64)).to(dev)
    for m, f, prefix in [(10160, 0.01, b"\x00\x01\x02\x03"), (1 << 20, 0.01, b"\x07")]:
        bf = BloomFilter(m, f, prefix)
        filt = torch.full((int(ctx.lib.dsy_filter_words(m)),), -1, dtype=torch.int32, device=dev)
        filt.zero_()  # queued on torch's stream right before the build
        union = add_sharded(ctx, bf.params, d_blob[G:], d_offs, len(offs) - 1, None, filt)
        whole = BloomFilter(m, f, prefix)
        whole.add_packed(blob, offs)
        assert union.cpu().numpy().tobytes()[:m // 8] == whole.bytes


def test_sim_overlapped_round_over_rccl_one_rank():
    """The simulator's chunked round with its exchanges on a communication stream (RCCL all-to-all(v), per-exchange
    events the engine's kernels wait on) in a one-rank "nccl" job: every record goes through RCCL, and the per-round
    history equals the plain round's (tools/sim_rccl_probe.py).  The driver's 8-GPU run takes this path."""
    port = str(_free_port())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", port, os.path.join(os.path.dirname(HERE), "tools", "sim_rccl_probe.py")]
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=180)
    log = p.stdout.decode(errors="replace")
    assert p.returncode == 0, log[-3000:]
    row = json.loads([ln for ln in log.splitlines() if ln.startswith("{")][-1])
    assert row["backend"] == "nccl" and row["whole"][-1][0] > row["whole"][0][0]
    for key in ("chunks1", "chunks4"):
        assert row[key]["equal"] and row[key]["exchanged_bytes"] > 0, (key, row[key])
    assert row["chunks4"]["overlapped"]


def test_rccl_collectives_one_rank():
    """The collectives Collectives issues over RCCL ("nccl"), with the dtypes the jobs pass -- int64 / float64
    scalars (all-reduce SUM / MAX), int32 and int64 all-gathers, a uint8 all-to-all(v) with byte splits -- in a
    one-rank torchrun job on cuda:0 (tools/rccl_probe.py).  Two ranks cannot share one GPU under RCCL ("Duplicate GPU
    detected"), so the two-rank exchanges above run over gloo; this pins the RCCL calls themselves."""
    port = str(_free_port())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", port, os.path.join(os.path.dirname(HERE), "tools", "rccl_probe.py")]
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=120)
    log = p.stdout.decode(errors="replace")
    assert p.returncode == 0, log[-3000:]
    row = json.loads([ln for ln in log.splitlines() if ln.startswith("{")][-1])
    assert row == {"rank": 0, "world": 1, "backend": "nccl", "sum_i64": 1, "max_f64": 0.5, "gather_i32": [0, 10, 20],
                   "gather_i64": [2 ** 40], "a2av_ok": True}

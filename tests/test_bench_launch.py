"""bench.py's process plumbing, on the CPU: `--gpus N` starts N ranks itself (through torch.distributed.run, as a
child process, before anything touches the GPU), a rank refuses a world size that differs from --gpus, and the
N-core CPU legs run in a pool forked before the GPU is used, reading large arrays from /dev/shm."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(kw)
    return env


def test_gpus_n_launches_n_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--steps", "1"], env=_env(DSY_BENCH_PROBE="1"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    probes = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(p["rank"] for p in probes) == [0, 1, 2]
    assert {p["world"] for p in probes} == {3}
    assert sorted(p["local_rank"] for p in probes) == [0, 1, 2]


def test_single_gpu_runs_in_process():
    r = subprocess.run([sys.executable, BENCH], env=_env(DSY_BENCH_PROBE="1"), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    probes = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert probes == [{"probe": True, "rank": 0, "world": 1, "local_rank": 0, "gpus": 1}]


def test_world_mismatch_is_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4"], env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0",
                                                                        DSY_BENCH_PROBE="1"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "--gpus 4" in r.stderr


def test_tail_keys_close_the_line():
    """The gossip rounds/s (BASELINE's second metric) and each leg's headline number are the LAST keys of the JSON
    line, read from the legs' nested records (shapes of a real run: profiles/bench_r3_n1_v4.json), so a driver that
    stores only the tail of stdout still holds them."""
    sys.path.insert(0, ROOT)
    import bench
    with open(os.path.join(ROOT, "profiles", "bench_r3_n1_v4.json")) as f:
        rec = json.load(f)
    rec = rec.get("parsed", rec)
    line = {"metric": "x", "value": 1.0, "gossip_sim": rec["gossip_sim"]}
    tail = bench.tail_keys(rec["gossip_sim"], rec["sha1_respond"], rec["heavy_tail"], rec["single_filter"],
                           rec["large_filter"], rec["cpu_baseline"])
    line.update(tail)
    text = json.dumps(line)
    keys = list(line)
    assert keys[-len(tail):] == list(tail)
    for k in ("gossip_rounds_per_s", "gossip_ms_per_round", "gossip_store_checksum", "gossip_n_gpus"):
        assert k in tail and tail[k] is not None, k
        assert '"%s"' % k in text[-600:], k
    assert tail["gossip_rounds_per_s"] == rec["gossip_sim"]["value"]
    assert tail["gossip_store_checksum"] == rec["gossip_sim"]["store_checksum"]
    assert tail["sha1_respond_int32_frac"] == rec["sha1_respond"]["roofline"]["frac"]
    assert tail["cfg5_ms_per_step"] == rec["heavy_tail"]["ms_per_step"]
    assert tail["cfg1_sha1_int32_frac"] == rec["single_filter"]["sha1"]["roofline_test"]["valu_int32"]["frac"]
    assert set(tail["cfg4_sha256_add_int32_frac"]) == {"2^20", "2^22", "2^24"}
    # the in-leg GPU == oracle checks of that run (round 3 had only the responder samples)
    assert tail["gpu_matches_oracle"]["cfg2_responder_sample"] is True
    assert tail["gpu_matches_oracle"]["sha1_responder_sample"] is True
    assert tail["gpu_matches_oracle"]["cfg5_responder_sample"] is True
    # legs that did not run leave None, never a KeyError
    assert set(bench.tail_keys(None).values()) == {None}


def test_cpu_pool_runs_closures_over_shared_arrays():
    sys.path.insert(0, ROOT)
    import bench
    arr = np.arange(1000, dtype=np.uint64)
    sh = bench.Shared(arr)
    scale = 3
    pool = bench.CpuPool(2)
    try:
        def fn(w):  # a closure: cloudpickle carries it, the array travels as its /dev/shm path
            return int(sh.a[w::2].sum()) * scale, 0.5
        units, secs = pool.run(fn, [0, 1])
        assert units == int(arr.sum()) * scale
        assert secs == 0.5
    finally:
        pool.close()
        path = sh.path
        bench.Shared.cleanup()
    assert not os.path.exists(path)

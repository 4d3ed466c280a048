"""Helpers shared by tests that read tests/golden/*.json (test infrastructure)."""
import functools
import gzip
import json
import os
import sqlite3

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@functools.lru_cache(maxsize=None)
def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def expected_bytes(expect):
    if "bytes_hex" in expect:
        return bytes.fromhex(expect["bytes_hex"])
    with gzip.open(os.path.join(GOLDEN, expect["bytes_file"]), "rb") as f:
        return f.read()


def keys_for(spec):
    from keys import named_packets, packet_list
    kind = spec["kind"]
    if kind == "named":
        return named_packets(spec["n"], spec.get("start", 0), spec.get("fmt", "packet-%d").encode())
    if kind == "random":
        return packet_list(spec["seed"], spec["n"], spec["lo"], spec["hi"])
    if kind == "str_int":
        return [str(i).encode() for i in range(spec["start"], spec["stop"])]
    if kind == "ragged":
        import numpy as np
        rng = np.random.Generator(np.random.PCG64(spec["seed"]))
        return [rng.bytes(n) for n in spec["lengths"]]
    raise ValueError(kind)


from oracle.sync_ref import SYNC_SCHEMA  # noqa: E402  (dispersydatabase.py:53-64)


def sqlite_from_rows(rows):
    conn = sqlite3.connect(":memory:")
    conn.executescript(SYNC_SCHEMA)
    conn.executemany("INSERT INTO sync(id, community, member, global_time, meta_message, undone, packet, sequence) "
                     "VALUES (?, 1, ?, ?, ?, ?, ?, 0)",
                     [(r["id"], r["member"], r["gt"], r["meta"], r["undone"], bytes.fromhex(r["packet"])) for r in rows])
    return conn


class Replay(object):
    """Replays the random draws the reference made (recorded by gen_sync_golden.DrawLog)."""

    def __init__(self, log):
        self.log = list(log)

    def _next(self, kind):
        k, v = self.log.pop(0)
        assert k == kind, (k, kind)
        return v

    def random(self):
        return self._next("random")

    def expovariate(self, lambd):
        return self._next("expovariate")

    def randint(self, a, b):
        return self._next("randint")

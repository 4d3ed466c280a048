#!/usr/bin/env python3
"""Where SyncCommunity.store_messages' time goes (GPU box): a 1 M-row store in HBM, batches of 10 k received messages
(100-1500 B) stored as bench.py's drop-in leg does, timed whole and under cProfile (top functions by own time), plus
the bare dsy_store_append call on the same columns.  Prints one JSON line."""
import cProfile
import io
import json
import os
import pstats
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dispersy_amd import _native  # noqa: E402
from dispersy_amd.community import SyncCommunity  # noqa: E402
from dispersy_amd.distribution import MetaMessage, SyncDistribution  # noqa: E402
from dispersy_amd.store import SyncStore  # noqa: E402


class Dist(object):
    def __init__(self, gt):
        self.global_time, self.priority = gt, 128


class Msg(object):
    """As the reference's Message.Implementation: .meta, and database_id read through it (message.py:265-266)."""

    def __init__(self, gt, packet, meta):
        self.meta, self.distribution, self.packet, self.candidate = meta, Dist(gt), packet, None

    @property
    def database_id(self):
        return self.meta.database_id


def main():
    rng = np.random.Generator(np.random.PCG64(1))
    n0, batch = 1_000_000, 10_000
    lens = rng.integers(100, 1501, size=n0)
    blob = rng.bytes(int(lens.sum()))
    cuts = np.concatenate([[0], np.cumsum(lens)])
    rows = [(i + 1, i + 1, 1, 0, blob[int(cuts[i]):int(cuts[i + 1])]) for i in range(n0)]
    store = SyncStore.from_rows(rows)
    store.handle  # noqa: B018
    meta = MetaMessage("bench", 1, SyncDistribution("ASC", 128))
    com = SyncCommunity(store, [meta], global_time=n0)
    work = []
    for b in range(12):
        bl = rng.integers(100, 1501, size=batch)
        data = rng.bytes(int(bl.sum()))
        c = np.concatenate([[0], np.cumsum(bl)])
        work.append([Msg(n0 + b * batch + j + 1, data[int(c[j]):int(c[j + 1])], meta) for j in range(batch)])
    com.store_messages(work[0])
    times = []
    for msgs in work[1:6]:
        t0 = time.perf_counter()
        com.store_messages(msgs)
        times.append(time.perf_counter() - t0)
    prof = cProfile.Profile()
    prof.enable()
    for msgs in work[6:11]:
        com.store_messages(msgs)
    prof.disable()
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(14)
    # the bare C call on ready columns
    msgs = work[11]
    packets = [m.packet for m in msgs]
    data = b"".join(packets)
    off = np.zeros(batch + 1, dtype=np.uint64)
    np.cumsum(np.fromiter(map(len, packets), dtype=np.uint64, count=batch), out=off[1:])
    gts = np.arange(n0 + 2_000_000, n0 + 2_000_000 + batch, dtype=np.uint64)
    metas = np.ones(batch, dtype=np.uint32)
    lib, ctx = store.ctx.lib, store.ctx
    bare = []
    for _ in range(5):
        t0 = time.perf_counter()
        _native.check(lib.dsy_store_append(ctx.handle, store.handle, data, len(data), off.ctypes.data, batch,
                                           gts.ctypes.data, metas.ctypes.data, None))
        bare.append(time.perf_counter() - t0)
        gts += batch
    print(json.dumps({"store_messages_ms": [round(x * 1e3, 3) for x in times],
                      "dsy_store_append_ms": [round(x * 1e3, 3) for x in bare],
                      "profile_tottime_top": s.getvalue().splitlines()[:40]}))


if __name__ == "__main__":
    main()

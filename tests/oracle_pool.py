"""Full-size parity through the CPU oracle, fanned out over worker processes (test infrastructure, no GPU).

oracle/sync_ref.respond_arrays is the reference's responder restated over in-memory columns: the claim's candidates in
send order (community.py:2746-2811 -- here one ASC meta), each hashed with hashlib through oracle/bloom_ref's lazy
not_filter, and the byte-limited walk that stops at the packet spending the budget (community.py:2555-2567).  At
BASELINE's full sizes (10 M stored packets, 1024 claims) that is minutes of one core, so the claims are spread over
spawned workers: fresh interpreters that import numpy, hashlib and oracle/ only (no torch, no HIP -- spawning a child
process is how a GPU process starts another program), attached to the data through read-only files:

    packets   the bytes of every candidate row the claims may touch, back to back (a row's packet is found through
              `rows`, the sorted row numbers, and `offsets`)
    gts       the store's global_time column (rows are 0..N-1, one meta, in index order)

check_claims() returns each claim's answer: the store rows sent, in order."""
import multiprocessing as mp
import os
import tempfile

import numpy as np

_WORKERS = 16  # the GPU box's CPU share (os.cpu_count() there reports the whole machine)
_STATE = {}


class _Identity(object):
    """rows[i] == i: the store's rows are its index order (one meta, every row live)."""

    def __getitem__(self, i):
        return i


def _attach(paths):
    if _STATE.get("paths") != paths:
        blob_p, off_p, rows_p, gts_p = paths
        _STATE.update(paths=paths, blob=np.load(blob_p, mmap_mode="r"), off=np.load(off_p, mmap_mode="r"),
                      rows=np.load(rows_p, mmap_mode="r"), gts=np.load(gts_p, mmap_mode="r"))
    return _STATE


def _one(task):
    """One claim through the oracle: (index, rows sent)."""
    import sys
    paths, root, idx, claim, global_time, byte_limit = task
    if root not in sys.path:
        sys.path.insert(0, root)
    from oracle import sync_ref
    from oracle.bloom_ref import OracleBloom
    st = _attach(paths)
    blob, off, rows = st["blob"], st["off"], st["rows"]

    def packet_of(r):
        i = int(np.searchsorted(rows, r))
        return blob[int(off[i]):int(off[i + 1])].tobytes()

    time_low, time_high, offset, modulo, raw, k, prefix = claim
    bloom = OracleBloom.from_bytes(raw, k, prefix)
    metas = [dict(name="fullsize", id=1, direction="ASC", priority=128, pruning=None)]
    sent = sync_ref.respond_arrays(packet_of, {1: (_Identity(), st["gts"])}, metas,
                                   (time_low, time_high, offset, modulo), bloom, global_time, byte_limit)
    return idx, sent


def check_claims(claims, packets, offsets, rows, gts, global_time, byte_limit, work=None):
    """claims: (time_low, time_high, offset, modulo, filter bytes, k, prefix) each; packets / offsets / rows: the
    candidate rows' bytes (see the module doc); gts: the global_time column; work: optional per-claim cost estimate
    (the heaviest go first).  Returns the oracle's answer for every claim, in order."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    base = "/dev/shm" if os.access("/dev/shm", os.W_OK) else None
    tmp = tempfile.mkdtemp(prefix="dsy_oracle_", dir=base)
    try:
        paths = []
        for name, arr in (("blob", packets), ("off", offsets), ("rows", rows), ("gts", gts)):
            p = os.path.join(tmp, name + ".npy")
            np.save(p, np.ascontiguousarray(arr))
            paths.append(p)
        paths = tuple(paths)
        order = list(range(len(claims)))
        if work is not None:
            order.sort(key=lambda i: -work[i])
        tasks = [(paths, root, i, claims[i], global_time, byte_limit) for i in order]
        out = [None] * len(claims)
        with mp.get_context("spawn").Pool(min(_WORKERS, max(1, len(claims)))) as pool:
            for i, sent in pool.imap_unordered(_one, tasks, chunksize=1):
                out[i] = sent
        return out
    finally:
        for f in os.listdir(tmp):
            os.unlink(os.path.join(tmp, f))
        os.rmdir(tmp)

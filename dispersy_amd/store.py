"""`SyncStore`: the packed HBM export of Dispersy's `sync` table (dispersydatabase.py:53-64).

Rows are kept in the order of the reference's `sync_meta_message_undone_global_time_index`
(meta_message, global_time, rowid) -- the order SQLite walks when it serves a sync range -- as columns:

    blob        u8[sum L]   packets back to back        offsets   u64[N+1]
    global_time u64[N]      meta u32[N]                 undone    i64[N]     rowid  i64[N]
    member      u64[N]      (optional: the (member, global_time) duplicate check, dispersy.py:831-918)

`undone` is the reference's column: 0, or the id of the undo message whose packet is the proof.

The device copy (dsy_store_upload) holds the packets as a line copy plus a live-row index (undone != 0 excluded)
with per-meta segments; the host copy of the small columns serves the claim-side range selection
(community.py:881-933) and maps responder output rows back to packets.

`append` is the requester-side ingest (`INSERT INTO sync` of Dispersy._store, dispersy.py:1475-1612): received
packets take the next row positions, in insertion (rowid) order, and join the index by (meta_message,
global_time, rowid) -- on the device by dsy_store_append's merge, on the host per meta.  Rows past the constructor's
are therefore no longer in index order; `live_rows` always is.  `dup_check` / `replace_packet` are the duplicate
check of received packets and its UPDATE (dispersy.py:831-918).
"""
import ctypes

import numpy as np

from . import _native


class SyncStore(object):
    def __init__(self, blob, offsets, global_time, meta, undone=None, rowid=None, ctx=None, member=None):
        self.offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        self.n = len(self.offsets) - 1
        self.blob = blob if isinstance(blob, (bytes, bytearray, memoryview, np.ndarray)) else bytes(blob)
        self.global_time = np.ascontiguousarray(global_time, dtype=np.uint64)
        self.meta = np.ascontiguousarray(meta, dtype=np.uint32)
        self.undone = (np.zeros(self.n, dtype=np.int64) if undone is None
                       else np.ascontiguousarray(undone, dtype=np.int64))
        self.rowid = (np.arange(1, self.n + 1, dtype=np.int64) if rowid is None
                      else np.ascontiguousarray(rowid, dtype=np.int64))
        self.member = None if member is None else np.ascontiguousarray(member, dtype=np.uint64)
        assert len(self.global_time) == len(self.meta) == len(self.undone) == len(self.rowid) == self.n
        assert self.member is None or len(self.member) == self.n
        if self.n > 1:
            m, g = self.meta, self.global_time
            bad = (m[1:] < m[:-1]) | ((m[1:] == m[:-1]) & (g[1:] < g[:-1]))
            if bad.any():
                raise ValueError("SyncStore rows must be sorted by (meta_message, global_time, rowid)")
        self._ctx = ctx
        self._handle = None
        self._n_sorted = self.n  # rows in index order, uploaded by dsy_store_upload; later rows are appends
        self._row_of_id = None
        self._replaced = {}  # row -> packet after an UPDATE (dsy_store_replace); the packed blob keeps the original
        self._dup_indexed = False
        self._prunes = []  # (meta, max_global_time) DELETEs, replayed on the device after a lazy upload
        # live (undone == 0) rows per meta, in global_time order: the claim side's index range scans
        live = np.flatnonzero(self.undone == 0)
        self._live = {}
        if len(live):
            lm = self.meta[live]
            cuts = np.flatnonzero(lm[1:] != lm[:-1]) + 1
            for seg in np.split(live, cuts):
                self._live[int(self.meta[seg[0]])] = seg
        self._empty = np.zeros(0, dtype=np.int64)

    # ------------------------------------------------------------------------------------ constructors
    @classmethod
    def from_rows(cls, rows, ctx=None):
        """rows: iterable of (rowid, global_time, meta_message, undone, packet[, member])."""
        rows = sorted(rows, key=lambda r: (r[2], r[1], r[0]))
        n = len(rows)
        offsets = np.zeros(n + 1, dtype=np.uint64)
        if n:
            np.cumsum([len(r[4]) for r in rows], out=offsets[1:])
        member = [r[5] for r in rows] if rows and len(rows[0]) > 5 else None
        return cls(b"".join(bytes(r[4]) for r in rows), offsets, [r[1] for r in rows], [r[2] for r in rows],
                   [r[3] for r in rows], [r[0] for r in rows], ctx=ctx, member=member)

    @classmethod
    def from_sqlite(cls, conn, community=None, ctx=None):
        """Export a Dispersy database's `sync` table (optionally one community) in index order."""
        sql = "SELECT id, global_time, meta_message, undone, packet, member FROM sync"
        args = ()
        if community is not None:
            sql += " WHERE community = ?"
            args = (community,)
        sql += " ORDER BY meta_message, global_time, id"
        return cls.from_rows([(i, g, m, u, bytes(p), mb) for i, g, m, u, p, mb in conn.execute(sql, args)], ctx=ctx)

    # --------------------------------------------------------------------------------------- accessors
    def packet(self, i):
        if self._replaced:
            p = self._replaced.get(int(i))
            if p is not None:
                return p
        a, b = int(self.offsets[i]), int(self.offsets[i + 1])
        return bytes(self.blob[a:b])

    def packets(self, rows):
        return [self.packet(int(i)) for i in rows]

    def length(self, i):
        if self._replaced and int(i) in self._replaced:
            return len(self._replaced[int(i)])
        return int(self.offsets[i + 1] - self.offsets[i])

    def row_of_id(self, rowid):
        if self._row_of_id is None:
            self._row_of_id = {int(r): i for i, r in enumerate(self.rowid)}
        return self._row_of_id[int(rowid)]

    def live_rows(self, meta_id):
        """Store rows of one meta with undone == 0, in (global_time, rowid) order."""
        return self._live.get(int(meta_id), self._empty)

    def count_live(self, meta_ids):
        return int(sum(len(self.live_rows(m)) for m in meta_ids))

    # ------------------------------------------------------------------------------------------ ingest
    def append(self, packets, global_time, meta, rowid=None, member=None):
        """INSERT INTO sync of a batch of received packets (dispersy.py:1475-1612), undone = 0.

        packets: list of bytes; global_time / meta (/ member): one per packet; rowid: increasing ids above every
        stored one (default: the next ids, as SQLite assigns them).  Returns the new rows' positions.  When the store
        is on the device already, the batch goes there in one dsy_store_append call."""
        a = len(packets)
        gts = np.ascontiguousarray(global_time, dtype=np.uint64)
        metas = np.ascontiguousarray(meta, dtype=np.uint32)
        if len(gts) != a or len(metas) != a:
            raise ValueError("append: one global_time and one meta per packet")
        top = int(self.rowid.max()) if self.n else 0
        ids = (np.arange(top + 1, top + 1 + a, dtype=np.int64) if rowid is None
               else np.ascontiguousarray(rowid, dtype=np.int64))
        if len(ids) != a or (a and (ids[0] <= top or (a > 1 and (ids[1:] <= ids[:-1]).any()))):
            raise ValueError("append: rowids must increase and exceed every stored rowid")
        if self.n and (self.member is None) != (member is None):
            raise ValueError("append: give members exactly when the store has a member column")
        mem = None if member is None else np.ascontiguousarray(member, dtype=np.uint64)
        rows = np.arange(self.n, self.n + a, dtype=np.int64)
        if a == 0:
            return rows
        lens = np.fromiter((len(p) for p in packets), dtype=np.uint64, count=a)
        new_off = np.zeros(a + 1, dtype=np.uint64)
        np.cumsum(lens, out=new_off[1:])
        data = b"".join(bytes(p) for p in packets)
        if self._handle is not None:
            lib = self.ctx.lib
            _native.check(lib.dsy_store_append(self.ctx.handle, self._handle, data, len(data), new_off.ctypes.data, a,
                                               gts.ctypes.data, metas.ctypes.data,
                                               mem.ctypes.data if self._dup_indexed else None))
        # host columns
        base = self.offsets[-1]
        self.offsets = np.concatenate([self.offsets, base + new_off[1:]])
        if isinstance(self.blob, np.ndarray):
            self.blob = np.concatenate([self.blob, np.frombuffer(data, dtype=np.uint8)])
        else:
            if not isinstance(self.blob, bytearray):
                self.blob = bytearray(self.blob)
            self.blob += data
        self.global_time = np.concatenate([self.global_time, gts])
        self.meta = np.concatenate([self.meta, metas])
        self.undone = np.concatenate([self.undone, np.zeros(a, dtype=np.int64)])
        self.rowid = np.concatenate([self.rowid, ids])
        if mem is not None:
            self.member = mem if self.member is None else np.concatenate([self.member, mem])
        self.n += a
        self._row_of_id = None
        # per-meta live rows: old rows first on equal global times (smaller rowid), new ones in insertion order
        for m in np.unique(metas):
            seg = np.concatenate([self._live.get(int(m), self._empty).astype(np.int64), rows[metas == m]])
            self._live[int(m)] = seg[np.argsort(self.global_time[seg], kind="stable")]
        return rows

    def prune(self, meta_id, max_global_time):
        """DELETE FROM sync WHERE meta_message = ? AND global_time <= ? (community.py:1092-1096, GlobalTimePruning):
        the rows leave the live index (host and device).  Returns the number of rows deleted."""
        seg = self._live.get(int(meta_id))
        if seg is None or not len(seg) or max_global_time < 0:
            return 0
        k = int(np.searchsorted(self.global_time[seg], np.uint64(max_global_time), side="right"))
        if not k:
            return 0
        self._live[int(meta_id)] = seg[k:]
        self._prunes.append((int(meta_id), int(max_global_time), self.n))
        if self._handle is not None:
            out = ctypes.c_uint64()
            _native.check(self.ctx.lib.dsy_store_prune(self.ctx.handle, self._handle, int(meta_id),
                                                       int(max_global_time), ctypes.byref(out)))
            assert out.value == k, (out.value, k)
        return k

    # ------------------------------------------------------------------------------- duplicate check
    def dup_check(self, members, global_times, packets, signature_lengths):
        """(verdict, row) per received message against the stored (member, global_time) rows (dsy_dup_check,
        _is_duplicate_sync_message dispersy.py:831-918): verdicts are _native.DSY_DUP_*; row -1 when new."""
        if self.member is None:
            raise ValueError("dup_check needs the store's member column")
        h = self.handle
        lib = self.ctx.lib
        if not self._dup_indexed:
            _native.check(lib.dsy_store_index_members(self.ctx.handle, h, self.member.ctypes.data,
                                                      self.global_time.ctypes.data, self.n))
            self._dup_indexed = True
        m = len(packets)
        mem = np.ascontiguousarray(members, dtype=np.uint64)
        gts = np.ascontiguousarray(global_times, dtype=np.uint64)
        sl = np.ascontiguousarray(signature_lengths, dtype=np.uint32)
        off = np.zeros(m + 1, dtype=np.uint64)
        if m:
            np.cumsum([len(p) for p in packets], out=off[1:])
        data = b"".join(bytes(p) for p in packets)
        verdict = np.zeros(m, dtype=np.uint8)
        row = np.zeros(m, dtype=np.uint64)
        if m:
            _native.check(lib.dsy_dup_check(self.ctx.handle, h, mem.ctypes.data, gts.ctypes.data, data, len(data),
                                            off.ctypes.data, m, sl.ctypes.data, verdict.ctypes.data, row.ctypes.data))
        return verdict, row.astype(np.int64)

    def replace_packet(self, rows, packets, device=True):
        """UPDATE sync SET packet = ? (dispersy.py:903) for the given rows: same row, index place and rowid.
        device=False changes only the host copy (the caller updates HBM with a later call)."""
        for r, p in zip(rows, packets):
            self._replaced[int(r)] = bytes(p)
        if device and self._handle is not None and len(rows):
            self._replace_device(rows, packets)

    def _replace_device(self, rows, packets):
        rws = np.ascontiguousarray(rows, dtype=np.uint64)
        off = np.zeros(len(packets) + 1, dtype=np.uint64)
        np.cumsum([len(p) for p in packets], out=off[1:])
        data = b"".join(bytes(p) for p in packets)
        _native.check(self.ctx.lib.dsy_store_replace(self.ctx.handle, self._handle, rws.ctypes.data, data, len(data),
                                                     off.ctypes.data, len(packets)))

    # ------------------------------------------------------------------------------------------ device
    @property
    def ctx(self):
        if self._ctx is None:
            self._ctx = _native.default_context()
        return self._ctx

    @property
    def handle(self):
        """dsy_store* on the device (uploaded on first use)."""
        if self._handle is None:
            ctx = self.ctx
            blob = self.blob if isinstance(self.blob, bytes) else bytes(self.blob)
            h = ctypes.c_void_p()
            n0 = self._n_sorted
            blob0 = blob[:int(self.offsets[n0])] if n0 < self.n else blob
            undone = (self.undone != 0).astype(np.uint8)
            _native.check(ctx.lib.dsy_store_upload(ctx.handle, blob0, len(blob0), self.offsets.ctypes.data, n0,
                                                   self.global_time.ctypes.data, self.meta.ctypes.data,
                                                   undone.ctypes.data, ctypes.byref(h)))
            self._handle = h
            # rows appended and DELETEs made before the first upload, replayed in their order (a DELETE never
            # reaches rows appended after it)
            done = n0
            for meta_id, max_gt, n_at in self._prunes + [(None, None, self.n)]:
                if n_at > done:
                    off = np.ascontiguousarray(self.offsets[done:n_at + 1] - self.offsets[done])
                    tail = blob[int(self.offsets[done]):int(self.offsets[n_at])]
                    _native.check(ctx.lib.dsy_store_append(ctx.handle, h, tail, len(tail), off.ctypes.data,
                                                           n_at - done, self.global_time[done:n_at].ctypes.data,
                                                           self.meta[done:n_at].ctypes.data, None))
                    done = n_at
                if meta_id is not None:
                    out = ctypes.c_uint64()
                    _native.check(ctx.lib.dsy_store_prune(ctx.handle, h, meta_id, max_gt, ctypes.byref(out)))
            if self._replaced:  # UPDATEs made before the first upload
                rows = sorted(self._replaced)
                self._replace_device(rows, [self._replaced[r] for r in rows])
        return self._handle

    def close(self):
        if self._handle is not None and self._ctx is not None and self._ctx.handle:
            self._ctx.lib.dsy_store_free(self._handle)
        self._handle = None

    __del__ = close

"""`SyncStore`: the packed HBM export of Dispersy's `sync` table (dispersydatabase.py:53-64).

Rows are kept in the order of the reference's `sync_meta_message_undone_global_time_index`
(meta_message, global_time, rowid) -- the order SQLite walks when it serves a sync range -- as columns:

    blob        u8[sum L]   packets back to back        offsets   u64[N+1]
    global_time u64[N]      meta u32[N]                 undone    i64[N]     rowid  i64[N]
    member      u64[N]      (optional: the (member, global_time) duplicate check, dispersy.py:831-918)
    sequence    i64[N]      the sequence number of sequence-numbered FullSync messages, 0 for NULL (dispersy.py:1529)
    deleted     bool[N]     rows a DELETE removed (pruning, sequence conflicts, LastSync history)

`undone` is the reference's column: 0, or the id of the undo message whose packet is the proof.

The device copy (dsy_store_upload) holds the packets as a line copy plus a live-row index (undone != 0 and deleted rows
excluded) with per-meta segments; the host copy of the small columns serves the claim-side range selection
(community.py:881-933) and maps responder output rows back to packets.

`append` is the requester-side ingest (`INSERT INTO sync` of Dispersy._store, dispersy.py:1475-1612): received
packets take the next row positions, in insertion (rowid) order, and join the index by (meta_message,
global_time, rowid) -- on the device by dsy_store_append's merge.  The host side is O(batch): columns grow
geometrically and the per-meta live arrays take the new rows as a pending delta, merged only when a host-side reader
asks for that meta's rows (live_rows).  Rows past the constructor's are therefore no longer in index order;
`live_rows` always is.  `dup_check` / `replace_packet` are the duplicate check of received packets and its UPDATE
(dispersy.py:831-918); `prune` and `delete_rows` are the DELETEs.
"""
import bisect
import ctypes

import numpy as np

from . import _native

_COLUMNS = ("global_time", "meta", "undone", "rowid", "member", "sequence", "deleted")


def _room(buf, used, need):
    """buf with capacity >= need (geometric growth, the first `used` entries kept)."""
    if need <= len(buf):
        return buf
    out = np.empty(max(need, 2 * len(buf), 1024), dtype=buf.dtype)
    out[:used] = buf[:used]
    return out


def _bytes_data_offset():
    """Offset of a CPython bytes object's data from its id() (the object header; 32 on 64-bit CPython 3), checked on
    live objects -- or None, and the appends join their packets instead."""
    off = bytes.__basicsize__ - 1
    try:
        for probe in (b"\x01\x02probe", bytes(range(256)) * 3, b"x"):
            if ctypes.string_at(id(probe) + off, len(probe)) != probe:
                return None
    except Exception:  # noqa: BLE001 -- any failure: take the join path
        return None
    return off


_BYTES_DATA = _bytes_data_offset()
_ONLY_BYTES = {bytes}


class _LiveRows(object):
    """One meta's live rows (undone == 0, not deleted) in the index order (global_time, row): a sorted base array
    (its global times beside it) whose removed rows are tombstones, and the rows added since (appended, or live again
    after a redo), merged on read.  Every change is O(its rows) -- a DELETE or an undo of 100 rows does not copy a
    10 M-row segment, a GlobalTimePruning cut is a binary search and a slice (round-4 verdict); rows() materialises
    the order (O(segment), only when a host-side reader asks for it)."""
    __slots__ = ("base", "gbase", "dead_base", "added", "dead_added", "n")

    def __init__(self, base, gbase):
        self.base = base
        self.gbase = gbase         # global_time of base's rows (ascending)
        self.dead_base = set()     # tombstones: rows of base no longer live
        self.added = []            # arrays of rows added since base was built
        self.dead_added = set()    # rows of `added` no longer live
        self.n = len(base)

    def _in_base(self, rows, gt):
        """Whether each of `rows` sits in base (else: in added): its global time's run of base, searched."""
        g = gt[rows]
        lo = np.searchsorted(self.gbase, g, side="left")
        hi = np.searchsorted(self.gbase, g, side="right")
        out = np.zeros(len(rows), dtype=bool)
        for j in np.flatnonzero(hi > lo).tolist():
            run = self.base[lo[j]:hi[j]]  # rows of one global time, ascending
            i = int(np.searchsorted(run, rows[j]))
            out[j] = i < len(run) and run[i] == rows[j]
        return out

    def add(self, rows, gt):
        if self.dead_base or self.dead_added:  # live again where they still sit (a redo of a row undone earlier)
            back_b = [r for r in rows.tolist() if r in self.dead_base]
            back_a = [r for r in rows.tolist() if r in self.dead_added]
            if back_b or back_a:
                self.dead_base.difference_update(back_b)
                self.dead_added.difference_update(back_a)
                self.n += len(back_b) + len(back_a)
                rows = rows[~np.isin(rows, back_b + back_a)]
        if len(rows):
            self.added.append(rows)
            self.n += len(rows)
            self._amortise(gt)

    def remove(self, rows, gt):
        where = self._in_base(rows, gt)
        self.dead_base.update(rows[where].tolist())
        self.dead_added.update(rows[~where].tolist())
        self.n -= len(rows)
        self._amortise(gt)

    # count_upto / cut (every GlobalTimePruning raise) walk the added arrays and the tombstones: keep both small
    # against the segment.  Added arrays are joined once there are kMaxParts of them (O(added rows), so O(1) per row
    # over kMaxParts batches); rows() merges everything into base once the pending rows or tombstones reach
    # 1/kMergeFrac of the segment (O(segment), paid once per segment/kMergeFrac changed rows: O(kMergeFrac) per row)
    kMaxParts = 16
    kMergeFrac = 8
    kMergeMin = 4096

    def _pending(self):
        return sum(len(a) for a in self.added) + len(self.dead_base) + len(self.dead_added)

    def _amortise(self, gt):
        if self._pending() >= max(self.kMergeMin, len(self.base) // self.kMergeFrac):
            self.rows(gt)
        elif len(self.added) > self.kMaxParts:
            self.added = [np.concatenate(self.added)]

    @staticmethod
    def _arr(s):
        return np.fromiter(s, dtype=np.int64, count=len(s))

    def rows(self, gt):
        """The live rows in (global_time, row) order."""
        if self.dead_base:
            keep = ~np.isin(self.base, self._arr(self.dead_base))
            self.base, self.gbase = self.base[keep], self.gbase[keep]
            self.dead_base = set()
        if self.added:
            new = np.concatenate(self.added)
            if self.dead_added:
                new = new[~np.isin(new, self._arr(self.dead_added))]
                self.dead_added = set()
            new = new[np.lexsort((new, gt[new]))]
            base, g, gn = self.base, self.gbase, gt[new]
            lo = np.searchsorted(g, gn, side="left")
            at = np.searchsorted(g, gn, side="right")
            # a row added among stored rows of its global time (a redone one) goes by row; an appended row's is larger
            # than every stored row's, so `at` (after them) is its place
            tie = np.flatnonzero(at > lo)  # (at > lo: base is not empty there)
            for j in tie[new[tie] < base[at[tie] - 1]].tolist():
                at[j] = lo[j] + int(np.searchsorted(base[lo[j]:at[j]], new[j]))
            self.base = np.insert(base, at, new)
            self.gbase = np.insert(g, at, gn)
            self.added = []
        return self.base

    def count_upto(self, gt, max_gt):
        """Live rows with global_time <= max_gt: O(log segment + tombstones + rows added since the last merge)."""
        mg = np.uint64(max_gt)
        k = int(np.searchsorted(self.gbase, mg, side="right"))
        if self.dead_base:
            k -= int((gt[self._arr(self.dead_base)] <= mg).sum())
        for a in self.added:
            k += int((gt[a] <= mg).sum())
        if self.dead_added:
            k -= int((gt[self._arr(self.dead_added)] <= mg).sum())
        return k

    def cut(self, gt, max_gt):
        """Remove and return the live rows with global_time <= max_gt (a GlobalTimePruning DELETE): O(log segment +
        rows cut + tombstones + rows added since the last merge)."""
        mg = np.uint64(max_gt)
        pos = int(np.searchsorted(self.gbase, mg, side="right"))
        gone = self.base[:pos]
        self.base, self.gbase = self.base[pos:], self.gbase[pos:]
        if self.dead_base:
            d = self._arr(self.dead_base)
            d = d[gt[d] <= mg]
            if len(d):
                gone = gone[~np.isin(gone, d)]
                self.dead_base.difference_update(d.tolist())
        if self.added:
            parts, keep = [gone], []
            for a in self.added:
                low = gt[a] <= mg
                parts.append(a[low])
                if not low.all():
                    keep.append(a[~low])
            self.added = keep
            gone = np.concatenate(parts)
            if self.dead_added:
                d = self._arr(self.dead_added)
                d = d[gt[d] <= mg]
                if len(d):
                    gone = gone[~np.isin(gone, d)]
                    self.dead_added.difference_update(d.tolist())
        self.n -= len(gone)
        return gone


class SyncStore(object):
    def __init__(self, blob, offsets, global_time, meta, undone=None, rowid=None, ctx=None, member=None,
                 communities=None, sequence=None):
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = self.n = len(offsets) - 1
        self._buf = dict(
            offsets=offsets.copy(),
            global_time=np.ascontiguousarray(global_time, dtype=np.uint64).copy(),
            meta=np.ascontiguousarray(meta, dtype=np.uint32).copy(),
            undone=(np.zeros(n, dtype=np.int64) if undone is None else np.ascontiguousarray(undone, dtype=np.int64).copy()),
            rowid=(np.arange(1, n + 1, dtype=np.int64) if rowid is None
                   else np.ascontiguousarray(rowid, dtype=np.int64).copy()),
            member=None if member is None else np.ascontiguousarray(member, dtype=np.uint64).copy(),
            sequence=(np.zeros(n, dtype=np.int64) if sequence is None
                      else np.ascontiguousarray([x or 0 for x in sequence], dtype=np.int64)),
            deleted=np.zeros(n, dtype=bool))
        self.blob = blob if isinstance(blob, (bytes, bytearray, memoryview, np.ndarray)) else bytes(blob)
        assert all(len(self._buf[c]) == n for c in _COLUMNS if self._buf[c] is not None)
        # communities the rows belong to (sync.community): the duplicate table is keyed (member, global_time), which
        # is the reference's UNIQUE(community, member, global_time) only within one community
        self.communities = None if communities is None else frozenset(communities)
        if n > 1:
            m, g = self.meta, self.global_time
            bad = (m[1:] < m[:-1]) | ((m[1:] == m[:-1]) & (g[1:] < g[:-1]))
            if bad.any():
                raise ValueError("SyncStore rows must be sorted by (meta_message, global_time, rowid)")
        self._ctx = ctx
        self._handle = None
        self._n_sorted = n  # rows in index order, uploaded by dsy_store_upload; later rows are appends
        self._row_of_id = None
        self._replaced = {}  # row -> packet after an UPDATE (dsy_store_replace); the packed blob keeps the original
        self._dup_indexed = False
        self._ops = []  # ("prune", meta, max_gt, n_at) / ("delete", rows, n_at): replayed on the device after a lazy upload
        # live (undone == 0, not deleted) rows per meta (_LiveRows), and the undone rows per meta (a DELETE reaches
        # them too; the index does not hold them)
        self._live = {}
        self._undone_rows = {}
        live = np.flatnonzero(self.undone == 0)
        if len(live):
            lm = self.meta[live]
            cuts = np.flatnonzero(lm[1:] != lm[:-1]) + 1
            for seg in np.split(live, cuts):
                self._live[int(self.meta[seg[0]])] = _LiveRows(seg, self.global_time[seg])
        und = np.flatnonzero(self.undone != 0)
        for r, m in zip(und.tolist(), self.meta[und].tolist()):
            self._undone_rows.setdefault(int(m), set()).add(r)
        self._empty = np.zeros(0, dtype=np.int64)
        self._groups = None  # (meta, member) -> rows, built on first use (member_rows)
        self._keys = None    # (member, global_time) -> row, built on first use (rows_of_keys)
        self._gpending = {}
        self._blob_base = 0  # offsets[] of the host blob's first byte (attach: earlier packets are device-only)
        # packets appended later, per batch: its joined bytes, or the list of the caller's packet objects when they
        # went to the device as a gather list (appending to one growing buffer copied it every batch: 8 MB per 10 k
        # packets); _tail_at[i] = offsets[] of batch i's first byte, _tail_row[i] = its first row
        self._tail, self._tail_at, self._tail_row = [], [], []
        self._pair_groups = {}  # (meta, member1, member2) -> rows: the double_signed_sync table (set_pairs)
        # whether the constructor's rows came with their double_signed_sync table (an empty store trivially did)
        self._pairs_exported = n == 0
        self._owns_handle = True

    # ------------------------------------------------------------------------------------------ columns
    def _col(self, name):
        b = self._buf[name]
        return None if b is None else b[:self.n]

    offsets = property(lambda self: self._buf["offsets"][:self.n + 1])
    global_time = property(lambda self: self._col("global_time"))
    meta = property(lambda self: self._col("meta"))
    undone = property(lambda self: self._col("undone"))
    rowid = property(lambda self: self._col("rowid"))
    member = property(lambda self: self._col("member"))
    sequence = property(lambda self: self._col("sequence"))
    deleted = property(lambda self: self._col("deleted"))

    # ------------------------------------------------------------------------------------ constructors
    @classmethod
    def from_rows(cls, rows, ctx=None, communities=None, pairs=None):
        """rows: iterable of (rowid, global_time, meta_message, undone, packet[, member[, sequence]]).
        pairs: the double_signed_sync table of these rows, (sync id, member1, member2) each (dispersy.py:1537-1541);
        None: not exported (a double-member-signed meta with stored rows then cannot keep its history, see
        pairs_exported)."""
        rows = sorted(rows, key=lambda r: (r[2], r[1], r[0]))
        n = len(rows)
        offsets = np.zeros(n + 1, dtype=np.uint64)
        if n:
            np.cumsum([len(r[4]) for r in rows], out=offsets[1:])
        member = [r[5] for r in rows] if rows and len(rows[0]) > 5 else None
        sequence = [r[6] for r in rows] if rows and len(rows[0]) > 6 else None
        st = cls(b"".join(bytes(r[4]) for r in rows), offsets, [r[1] for r in rows], [r[2] for r in rows],
                 [r[3] for r in rows], [r[0] for r in rows], ctx=ctx, member=member, communities=communities,
                 sequence=sequence)
        if pairs is not None:
            st._load_pairs(pairs)
        return st

    @classmethod
    def from_sqlite(cls, conn, community=None, ctx=None):
        """Export a Dispersy database's `sync` table (optionally one community) in index order, with its
        double_signed_sync rows (the member pairs of double-member-signed messages) when the database has that table."""
        sql = "SELECT id, global_time, meta_message, undone, packet, member, community, sequence FROM sync"
        args = ()
        if community is not None:
            sql += " WHERE community = ?"
            args = (community,)
        sql += " ORDER BY meta_message, global_time, id"
        rows = list(conn.execute(sql, args))
        pairs = None
        if conn.execute("SELECT name FROM sqlite_master WHERE type = 'table' AND name = 'double_signed_sync'").fetchone():
            psql = "SELECT double_signed_sync.sync, member1, member2 FROM double_signed_sync"
            if community is not None:
                psql += " JOIN sync ON sync.id = double_signed_sync.sync WHERE sync.community = ?"
            pairs = list(conn.execute(psql, args))
        return cls.from_rows([(i, g, m, u, bytes(p), mb, sq) for i, g, m, u, p, mb, _, sq in rows], ctx=ctx,
                             communities={r[6] for r in rows} if rows else ({community} if community is not None else None),
                             pairs=pairs)

    @classmethod
    def attach(cls, ctx, handle, global_time, meta, lengths, member=None, undone=None, pairs=None, rowid=None):
        """A store exported straight into HBM (dsy_store_attach / dsy_store_upload made by the caller): the host keeps
        the small columns only (rows in index order), the packets of these rows stay on the device -- packet() serves
        only rows appended later.  `handle` is the dsy_store* (the caller keeps ownership); `undone` must be the
        column the device index was built from (None: every row live), so host and device agree on the live rows.
        pairs / rowid: as from_rows (the rows' sync ids default to 1..n)."""
        lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
        offsets = np.zeros(len(lengths) + 1, dtype=np.uint64)
        np.cumsum(lengths, out=offsets[1:])
        st = cls(bytearray(), offsets, global_time, meta, ctx=ctx, member=member, undone=undone, rowid=rowid)
        st._blob_base = int(offsets[-1])
        st._handle = handle if isinstance(handle, ctypes.c_void_p) else ctypes.c_void_p(handle)
        st._owns_handle = False
        if pairs is not None:
            st._load_pairs(pairs)
        return st

    def _load_pairs(self, pairs):
        """The exported double_signed_sync rows (sync id, member1, member2) as the pair groups set_pairs keeps."""
        rows, a, b = [], [], []
        for sync_id, m1, m2 in pairs:
            try:
                rows.append(self.row_of_id(sync_id))
            except KeyError:  # a pair row whose sync row is gone (or of another community): the JOIN drops it
                continue
            a.append(int(m1))
            b.append(int(m2))
        self.set_pairs(np.asarray(rows, dtype=np.int64), a, b)
        self._pairs_exported = True

    # --------------------------------------------------------------------------------------- accessors
    def packet(self, i):
        if self._replaced:
            p = self._replaced.get(int(i))
            if p is not None:
                return p
        off = self._buf["offsets"]
        if self._tail and i >= self._tail_row[0]:
            k = bisect.bisect_right(self._tail_row, i) - 1
            t = self._tail[k]
            if isinstance(t, list):
                return t[i - self._tail_row[k]]
            a, b = int(off[i]) - self._tail_at[k], int(off[i + 1]) - self._tail_at[k]
            return t[a:b]
        a, b = int(off[i]), int(off[i + 1])
        a, b = a - self._blob_base, b - self._blob_base
        if a < 0:
            raise KeyError("row %d's packet lives only on the device (SyncStore.attach)" % int(i))
        return bytes(self.blob[a:b])

    def _host_blob(self):
        """Every host-held packet byte in one buffer (the initial blob, then the appended batches)."""
        if self._tail:
            self.blob = bytes(self.blob) + b"".join(t if not isinstance(t, list) else b"".join(t) for t in self._tail)
            self._tail, self._tail_at, self._tail_row = [], [], []
        return self.blob

    def packets(self, rows):
        return [self.packet(int(i)) for i in rows]

    def length(self, i):
        if self._replaced and int(i) in self._replaced:
            return len(self._replaced[int(i)])
        off = self._buf["offsets"]
        return int(off[i + 1] - off[i])

    def row_of_id(self, rowid):
        """The row holding `rowid` (KeyError when there is none, or it was deleted: SELECT ... WHERE id = ? is empty)."""
        if self._row_of_id is None:
            keep = np.flatnonzero(~self.deleted)
            self._row_of_id = dict(zip(self.rowid[keep].tolist(), keep.tolist()))
        return self._row_of_id[int(rowid)]

    def rows_of_keys(self, members, global_times):
        """The row of each (member, global_time) -- the sync table's UNIQUE(community, member, global_time) key
        within one community -- or -1 when no (undeleted) row has it: the WHERE of `UPDATE sync SET undone = ? WHERE
        community = ? AND member = ? AND global_time = ?` (community.py:3479-3480)."""
        if self.member is None:
            raise ValueError("rows_of_keys needs the store's member column")
        if self.communities is not None and len(self.communities) > 1:
            raise ValueError("rows_of_keys: the store spans communities %s; the (member, global_time) key is unique "
                             "only within one community (UNIQUE(community, member, global_time))"
                             % sorted(self.communities))
        if self._keys is None:
            keep = np.flatnonzero(~self.deleted)
            self._keys = dict(zip(zip(self.member[keep].tolist(), self.global_time[keep].tolist()), keep.tolist()))
        return np.asarray([self._keys.get((int(m), int(g)), -1) for m, g in zip(members, global_times)], dtype=np.int64)

    def live_rows(self, meta_id):
        """Store rows of one meta with undone == 0 (not deleted), in (global_time, rowid) order."""
        lv = self._live.get(int(meta_id))
        return self._empty if lv is None else lv.rows(self.global_time)

    def live_count(self, meta_id):
        lv = self._live.get(int(meta_id))
        return 0 if lv is None else lv.n

    def count_live(self, meta_ids):
        return int(sum(self.live_count(m) for m in set(int(x) for x in meta_ids)))

    def meta_ids(self):
        return sorted(m for m, lv in self._live.items() if lv.n or len(lv.base))

    def _live_of(self, m):
        lv = self._live.get(m)
        if lv is None:
            lv = self._live[m] = _LiveRows(self._empty, np.zeros(0, dtype=np.uint64))
        return lv

    def member_rows(self, meta_id, member):
        """Rows of one (meta_message, member) -- undone ones included, deleted ones not -- in global_time order (unique
        within a member): `SELECT ... FROM sync WHERE member = ? AND meta_message = ? ORDER BY global_time`
        (dispersy.py:959, :986, :1582-1586)."""
        if self.member is None:
            raise ValueError("member_rows needs the store's member column")
        if self._groups is None:
            keep = np.flatnonzero(~self.deleted)
            order = keep[np.lexsort((self.global_time[keep], self.member[keep], self.meta[keep]))]
            km, kb = self.meta[order], self.member[order]
            cuts = np.flatnonzero((km[1:] != km[:-1]) | (kb[1:] != kb[:-1])) + 1
            self._groups = {(int(self.meta[g[0]]), int(self.member[g[0]])): g for g in np.split(order, cuts) if len(g)}
            self._gpending = {}
        key = (int(meta_id), int(member))
        rows = self._groups.get(key, self._empty)
        pend = self._gpending.pop(key, None)
        if pend:
            rows = np.concatenate([rows] + pend)
        rows = rows[~self.deleted[rows]]
        if pend:
            rows = rows[np.argsort(self.global_time[rows], kind="stable")]
        self._groups[key] = rows
        return rows

    # ------------------------------------------------------------------------------ double_signed_sync
    def set_pairs(self, rows, member_a, member_b):
        """INSERT INTO double_signed_sync (sync, member1, member2) for the given rows of double-member-signed messages:
        the member pair, smaller id first (dispersy.py:1537-1541)."""
        for r, a, b in zip(np.asarray(rows).tolist(), np.asarray(member_a).tolist(), np.asarray(member_b).tolist()):
            pair = (a, b) if a < b else (b, a)
            self._pair_groups.setdefault((int(self.meta[r]),) + pair, []).append(r)

    def pairs_exported(self, meta_id):
        """Whether pair_rows can see every stored row of this meta: the store's initial rows came with their
        double_signed_sync table, or none of them is of this meta (rows appended later record their pairs)."""
        if self._pairs_exported:
            return True
        known = self.__dict__.setdefault("_pairless_metas", {})
        m = int(meta_id)
        if m not in known:
            known[m] = not bool(np.any(self._buf["meta"][:self._n_sorted] == m))
        return known[m]

    def pair_rows(self, meta_id, member1, member2):
        """Rows of one meta signed by the member pair (member1 < member2), deleted ones not, in the order of
        `SELECT sync.id FROM sync JOIN double_signed_sync ON double_signed_sync.sync = sync.id WHERE
        sync.meta_message = ? AND member1 = ? AND member2 = ? ORDER BY sync.global_time, sync.packet`
        (dispersy.py:1571-1578): global time, then the packet bytes."""
        rows = [r for r in self._pair_groups.get((int(meta_id), int(member1), int(member2)), ()) if not self.deleted[r]]
        self._pair_groups[(int(meta_id), int(member1), int(member2))] = rows
        return np.asarray(sorted(rows, key=lambda r: (int(self.global_time[r]), self.packet(r))), dtype=np.int64)

    # ------------------------------------------------------------------------------------------ ingest
    def append(self, packets, global_time, meta, rowid=None, member=None, sequence=None, _gather=None):
        """INSERT INTO sync of a batch of received packets (dispersy.py:1475-1612), undone = 0.

        packets: list of bytes; global_time / meta (/ member): one per packet; rowid: increasing ids above every
        stored one (default: the next ids, as SQLite assigns them); sequence: the messages' sequence numbers (0 or None:
        NULL).  Returns the new rows' positions.  When the store is on the device already, the batch goes there in one
        dsy_store_append call.  Host work is O(batch).  _gather: (lengths, addresses) of `packets`, all exactly bytes,
        as SyncCommunity.store_messages' C column reader returns them (the gather list, not recomputed)."""
        a = len(packets)
        gts = np.ascontiguousarray(global_time, dtype=np.uint64)
        metas = np.ascontiguousarray(meta, dtype=np.uint32)
        if len(gts) != a or len(metas) != a:
            raise ValueError("append: one global_time and one meta per packet")
        top = self._top_rowid()
        ids = (np.arange(top + 1, top + 1 + a, dtype=np.int64) if rowid is None
               else np.ascontiguousarray(rowid, dtype=np.int64))
        if len(ids) != a or (a and (ids[0] <= top or (a > 1 and (ids[1:] <= ids[:-1]).any()))):
            raise ValueError("append: rowids must increase and exceed every stored rowid")
        if self.n and (self.member is None) != (member is None):
            raise ValueError("append: give members exactly when the store has a member column")
        mem = None if member is None else np.ascontiguousarray(member, dtype=np.uint64)
        n0 = self.n
        rows = np.arange(n0, n0 + a, dtype=np.int64)
        if a == 0:
            return rows
        if _gather is not None:
            lens, addrs = _gather
            if len(lens) != a or len(addrs) != a:
                raise ValueError("append: one (length, address) per packet")
        else:
            lens = np.fromiter(map(len, packets), dtype=np.uint64, count=a)
        new_off = np.zeros(a + 1, dtype=np.uint64)
        np.cumsum(lens, out=new_off[1:])
        if self._handle is not None and (_gather is not None or
                                         (_BYTES_DATA is not None and set(map(type, packets)) == _ONLY_BYTES)):
            # the packet objects' own bytes as a gather list (no joined copy: it cost more than the device call)
            if _gather is None:
                packets = list(packets)
                addrs = np.fromiter(map(id, packets), dtype=np.uint64, count=a) + np.uint64(_BYTES_DATA)
            _native.check(self.ctx.lib.dsy_store_append_gather(
                self.ctx.handle, self._handle, addrs.ctypes.data, lens.ctypes.data, a, gts.ctypes.data,
                metas.ctypes.data, mem.ctypes.data if mem is not None else None))
            data = packets
        else:
            data = b"".join(packets)  # bytes-like items join as they are
            if self._handle is not None:
                _native.check(self.ctx.lib.dsy_store_append(self.ctx.handle, self._handle, data, len(data),
                                                            new_off.ctypes.data, a, gts.ctypes.data, metas.ctypes.data,
                                                            mem.ctypes.data if mem is not None else None))
        # host columns: geometric growth, O(batch) per append
        b = self._buf
        b["offsets"] = _room(b["offsets"], n0 + 1, n0 + a + 1)
        b["offsets"][n0 + 1:n0 + a + 1] = b["offsets"][n0] + new_off[1:]
        if sequence is None:
            seqs = np.zeros(a, dtype=np.int64)
        else:
            try:
                seqs = np.asarray(sequence, dtype=np.int64)  # ints (0: NULL)
            except TypeError:  # None entries
                seqs = np.asarray([x or 0 for x in sequence], dtype=np.int64)
        for name, vals in (("global_time", gts), ("meta", metas), ("undone", np.zeros(a, dtype=np.int64)),
                           ("rowid", ids), ("sequence", seqs), ("deleted", np.zeros(a, dtype=bool))):
            b[name] = _room(b[name], n0, n0 + a)
            b[name][n0:n0 + a] = vals
        if mem is not None:
            b["member"] = np.empty(0, dtype=np.uint64) if b["member"] is None else b["member"]
            b["member"] = _room(b["member"], n0, n0 + a)
            b["member"][n0:n0 + a] = mem
        self._tail_at.append(int(b["offsets"][n0]))
        self._tail_row.append(n0)
        self._tail.append(data)
        self.n = n0 + a
        self._top = int(ids[-1])
        if self._row_of_id is not None:
            self._row_of_id.update(zip(ids.tolist(), rows.tolist()))
        if self._keys is not None and mem is not None:
            self._keys.update(zip(zip(mem.tolist(), gts.tolist()), rows.tolist()))
        if self._groups is not None and mem is not None:
            for r, m, b_ in zip(rows.tolist(), metas.tolist(), mem.tolist()):
                self._gpending.setdefault((m, b_), []).append(np.asarray([r], dtype=np.int64))
        # per-meta live rows: merged lazily (live_rows)
        if a and metas[0] == metas[-1] and (metas == metas[0]).all():  # one meta (the usual batch)
            self._live_of(int(metas[0])).add(rows, self.global_time)
        else:
            order = np.argsort(metas, kind="stable")
            sm = metas[order]
            cuts = np.flatnonzero(sm[1:] != sm[:-1]) + 1
            for part in np.split(order, cuts):
                self._live_of(int(metas[part[0]])).add(rows[part], self.global_time)
        return rows

    def _top_rowid(self):
        if getattr(self, "_top", None) is None:
            self._top = int(self.rowid.max()) if self.n else 0
        return self._top

    # ------------------------------------------------------------------------------------------ DELETEs
    def prune(self, meta_id, max_global_time):
        """DELETE FROM sync WHERE meta_message = ? AND global_time <= ? (community.py:1092-1096, GlobalTimePruning):
        the rows -- live and undone alike, as the SQL DELETE does -- leave the store: the live ones the index (host and
        device), all of them the duplicate table and row_of_id.  Returns the number of rows deleted."""
        m = int(meta_id)
        if max_global_time < 0:
            return 0
        lv = self._live.get(m)
        gt = self.global_time
        # the live rows the DELETE reaches: a prefix of the meta's index order (plus rows added since its last merge)
        k = lv.count_upto(gt, max_global_time) if lv is not None else 0
        und = self._undone_rows.get(m)
        gone = np.asarray(sorted(r for r in und if gt[r] <= max_global_time), dtype=np.int64) if und else self._empty
        # the device first: a refused call (e.g. DSY_EINVAL while responder batches are in flight) leaves the host
        # bookkeeping untouched, so host and device never drift apart
        if k:
            if self._handle is not None:
                out = ctypes.c_uint64()
                _native.check(self.ctx.lib.dsy_store_prune(self.ctx.handle, self._handle, m, int(max_global_time),
                                                           ctypes.byref(out)))
                if out.value != k:
                    raise RuntimeError("device and host stores disagree: the device pruned %d rows, the host %d"
                                       % (out.value, k))
            cut = lv.cut(gt, max_global_time)
            assert len(cut) == k
            self._mark_deleted(cut)
            self._ops.append(("prune", m, int(max_global_time), self.n))
        if len(gone):  # undone rows are outside the index: only their duplicate-table slots go
            if self._handle is not None:
                out = ctypes.c_uint64()
                rws = gone.astype(np.uint64)
                _native.check(self.ctx.lib.dsy_store_delete(self.ctx.handle, self._handle, rws.ctypes.data, len(rws),
                                                            ctypes.byref(out)))
            und.difference_update(gone.tolist())
            self._mark_deleted(gone)
            self._ops.append(("delete", gone, self.n))
        return k + len(gone)

    def delete_rows(self, rows):
        """DELETE FROM sync WHERE id = ? for the given store rows (the sequence-number conflict DELETE,
        dispersy.py:1006-1007, and LastSyncDistribution's history pruning, :1581-1591): they leave the live index, the
        duplicate table and row_of_id.  Returns the number of rows deleted (already deleted ones not counted)."""
        rows = np.unique(np.asarray(rows, dtype=np.int64))
        if not len(rows):
            return 0
        if rows[0] < 0 or rows[-1] >= self.n:
            raise IndexError("delete_rows: row out of range")
        rows = rows[~self.deleted[rows]]
        if not len(rows):
            return 0
        live = rows[self.undone[rows] == 0]
        if self._handle is not None:  # the device first (see prune)
            out = ctypes.c_uint64()
            rws = rows.astype(np.uint64)  # keep the array alive across the call
            _native.check(self.ctx.lib.dsy_store_delete(self.ctx.handle, self._handle, rws.ctypes.data, len(rws),
                                                        ctypes.byref(out)))
            if out.value != len(live):
                raise RuntimeError("device and host stores disagree: the device removed %d index entries, the host "
                                   "counts %d live rows" % (out.value, len(live)))
        lm = self.meta[live]
        for m in np.unique(lm).tolist():
            self._live[m].remove(live[lm == m], self.global_time)
        und = rows[self.undone[rows] != 0]
        for r, m in zip(und.tolist(), self.meta[und].tolist()):
            self._undone_rows[int(m)].discard(r)
        self._mark_deleted(rows)
        self._ops.append(("delete", rows, self.n))
        return len(rows)

    # ------------------------------------------------------------------------------------------ undo / redo
    def set_undone(self, rows, values):
        """UPDATE sync SET undone = ? WHERE id = ? for the given store rows: Community.on_undo (community.py:3457-3481,
        the undo message's packet id) and _update_timerange (:3633-3642, 1 to undo, 0 to redo).  A row given several
        times keeps its last value (executemany order); deleted rows are left alone (the UPDATE finds no row).  Rows
        that become undone leave the responder's index (host and device) but keep their duplicate-table slots (the
        duplicate check still finds them and sends the undo proof, dispersy.py:886-892); rows that become live again
        re-enter it at their (global_time, rowid) place.  Returns the number of rows whose undone-ness changed."""
        rows = np.atleast_1d(np.asarray(rows, dtype=np.int64))
        values = np.broadcast_to(np.asarray(values, dtype=np.int64), rows.shape)
        if not len(rows):
            return 0
        if rows.min() < 0 or rows.max() >= self.n:
            raise IndexError("set_undone: row out of range")
        last = dict(zip(rows.tolist(), values.tolist()))
        rows = np.fromiter(last.keys(), dtype=np.int64, count=len(last))
        vals = np.fromiter(last.values(), dtype=np.int64, count=len(last))
        alive = ~self.deleted[rows]
        rows, vals = rows[alive], vals[alive]
        cur = self.undone[rows]
        undo = np.sort(rows[(cur == 0) & (vals != 0)])
        redo = np.sort(rows[(cur != 0) & (vals == 0)])
        if self._handle is not None:  # the device first (see prune)
            self._set_undone_device(undo, redo)
        self._buf["undone"][rows] = vals
        um = self.meta[undo]
        for m in np.unique(um).tolist():
            part = undo[um == m]
            self._live[m].remove(part, self.global_time)
            self._undone_rows.setdefault(m, set()).update(part.tolist())
        rm = self.meta[redo]
        for m in np.unique(rm).tolist():
            part = redo[rm == m]
            self._undone_rows[m].difference_update(part.tolist())
            self._live_of(m).add(part, self.global_time)
        return len(undo) + len(redo)

    def _set_undone_device(self, undo, redo):
        lib, out = self.ctx.lib, ctypes.c_uint64()
        if len(undo):
            u = undo.astype(np.uint64)
            _native.check(lib.dsy_store_set_undone(self.ctx.handle, self._handle, u.ctypes.data, len(u), None, None, 1,
                                                   ctypes.byref(out)))
            if out.value != len(u):
                raise RuntimeError("device and host stores disagree: %d of %d rows to undo were in the device index"
                                   % (out.value, len(u)))
        if len(redo):
            r = redo.astype(np.uint64)
            mt = np.ascontiguousarray(self.meta[redo])
            gt = np.ascontiguousarray(self.global_time[redo])
            _native.check(lib.dsy_store_set_undone(self.ctx.handle, self._handle, r.ctypes.data, len(r), mt.ctypes.data,
                                                   gt.ctypes.data, 0, ctypes.byref(out)))

    def _mark_deleted(self, rows):
        self._buf["deleted"][rows] = True
        if self._keys is not None:
            for k in zip(self.member[rows].tolist(), self.global_time[rows].tolist()):
                self._keys.pop(k, None)
        if self._row_of_id is not None:
            for rid in self.rowid[rows].tolist():
                self._row_of_id.pop(rid, None)

    # ------------------------------------------------------------------------------- duplicate check
    def dup_check(self, members, global_times, packets, signature_lengths):
        """(verdict, row) per received message against the stored (member, global_time) rows (dsy_dup_check,
        _is_duplicate_sync_message dispersy.py:831-918): verdicts are _native.DSY_DUP_*; row -1 when new."""
        if self.member is None:
            raise ValueError("dup_check needs the store's member column")
        if self.communities is not None and len(self.communities) > 1:
            raise ValueError("dup_check: the store spans communities %s; the (member, global_time) key is unique only "
                             "within one community (UNIQUE(community, member, global_time))" % sorted(self.communities))
        h = self.handle
        lib = self.ctx.lib
        if not self._dup_indexed:
            _native.check(lib.dsy_store_index_members(self.ctx.handle, h, self.member.ctypes.data,
                                                      self.global_time.ctypes.data, self.n))
            self._dup_indexed = True
            gone = np.flatnonzero(self.deleted).astype(np.uint64)
            if len(gone):  # rows deleted before the table existed are not in it
                out = ctypes.c_uint64()
                _native.check(lib.dsy_store_delete(self.ctx.handle, h, gone.ctypes.data, len(gone), ctypes.byref(out)))
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
            blob = self._host_blob()
            blob = blob if isinstance(blob, bytes) else bytes(blob)
            h = ctypes.c_void_p()
            n0 = self._n_sorted
            offsets = np.ascontiguousarray(self.offsets)
            blob0 = blob[:int(offsets[n0])] if n0 < self.n else blob
            undone = (self.undone[:n0] != 0).astype(np.uint8)
            gts0, metas0 = np.ascontiguousarray(self.global_time[:n0]), np.ascontiguousarray(self.meta[:n0])
            _native.check(ctx.lib.dsy_store_upload(ctx.handle, blob0, len(blob0), offsets.ctypes.data, n0,
                                                   gts0.ctypes.data, metas0.ctypes.data, undone.ctypes.data,
                                                   ctypes.byref(h)))
            self._handle = h
            # rows appended and DELETEs made before the first upload, replayed in their order (a DELETE never
            # reaches rows appended after it)
            done = n0
            for op in self._ops + [("end", None, None, self.n)]:
                n_at = op[-1]
                if n_at > done:
                    off = np.ascontiguousarray(offsets[done:n_at + 1] - offsets[done])
                    tail = blob[int(offsets[done]):int(offsets[n_at])]
                    gts1 = np.ascontiguousarray(self.global_time[done:n_at])
                    metas1 = np.ascontiguousarray(self.meta[done:n_at])
                    _native.check(ctx.lib.dsy_store_append(ctx.handle, h, tail, len(tail), off.ctypes.data,
                                                           n_at - done, gts1.ctypes.data, metas1.ctypes.data, None))
                    done = n_at
                out = ctypes.c_uint64()
                if op[0] == "prune":
                    _native.check(ctx.lib.dsy_store_prune(ctx.handle, h, op[1], op[2], ctypes.byref(out)))
                elif op[0] == "delete":
                    rws = op[1].astype(np.uint64)
                    _native.check(ctx.lib.dsy_store_delete(ctx.handle, h, rws.ctypes.data, len(rws), ctypes.byref(out)))
            if self._replaced:  # UPDATEs made before the first upload
                rows = sorted(self._replaced)
                self._replace_device(rows, [self._replaced[r] for r in rows])
            # rows appended before the upload went in live; the ones undone since leave the index (the upload's own
            # rows took their current undone column)
            late = np.arange(n0, self.n, dtype=np.int64)
            late = late[(self.undone[late] != 0) & ~self.deleted[late]]
            if len(late):
                self._set_undone_device(late, np.zeros(0, dtype=np.int64))
        return self._handle

    def close(self):
        if self._handle is not None and self._owns_handle and self._ctx is not None and self._ctx.handle:
            self._ctx.lib.dsy_store_free(self._handle)
        self._handle = None

    __del__ = close

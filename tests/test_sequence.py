"""The sequence-number branch of _check_full_sync_distribution_batch (dispersy.py:954-1037) and LastSyncDistribution's
history pruning in _store (:1558-1591), against the reference's own methods lifted from dispersy.py's AST
(tests/golden/gen_dedup_golden.py: dedup_seq_vectors.json -- 40 batches replayed on one table, with the DELETEs of
conflicting sequence numbers and the py2 generator cut-off --, laststore_vectors.json -- 12 _store batches with
history_size 2).

CPU: the oracle restatement (oracle/sync_ref.check_sequence_batch / store_last_sync over sqlite3) replays them.
GPU: SyncCommunity does -- the (member, global_time) lookups as one dsy_dup_check per batch, the DELETEs through
dsy_store_delete -- and the responder's index and the duplicate table follow the table after every batch."""
import sqlite3

import numpy as np
import pytest

from dispersy_amd.community import DelayMessageBySequence, DropMessage, SyncCommunity
from dispersy_amd.distribution import FullSyncDistribution, GlobalTimePruning, LastSyncDistribution, MetaMessage
from dispersy_amd.store import SyncStore
from golden_util import load
from oracle import sync_ref

SEQ = load("dedup_seq_vectors.json")
LAST = load("laststore_vectors.json")
DOUBLE = load("doublestore_vectors.json")


def sqlite_of(table):
    conn = sqlite3.connect(":memory:")
    conn.executescript(sync_ref.SYNC_SCHEMA)
    conn.executemany("INSERT INTO sync (id, community, member, global_time, meta_message, undone, packet, sequence) "
                     "VALUES (?, 1, ?, ?, ?, ?, ?, ?)",
                     [(i, mem, gt, meta, und, bytes.fromhex(p), sq) for i, mem, gt, meta, und, p, sq in table])
    return conn


def table_of(conn):
    return [list(r) for r in conn.execute("SELECT id, member, global_time, meta_message, undone, hex(packet), sequence "
                                          "FROM sync ORDER BY id")]


def _expect(r):
    return tuple(r) if isinstance(r, list) else r


def test_oracle_sequence_branch_matches_reference():
    conn = sqlite_of(SEQ["table_before"])
    assert sum(b["ended_early"] for b in SEQ["batches"]) > 5
    for b in SEQ["batches"]:
        msgs = [dict(member=m["member"], gt=m["gt"], seq=m["seq"], packet=bytes.fromhex(m["packet"]),
                     signature_length=SEQ["signature_length"], inactive=SEQ["inactive"], index=m["index"])
                for m in b["batch"]]
        out, sends, ended = sync_ref.check_sequence_batch(conn, 1, 2, msgs, SEQ["acceptable_global_time"],
                                                          SEQ["global_time"])
        assert [(i, _expect(r)) for i, r in out] == [(i, _expect(r)) for i, r in b["results"]]
        assert ended == b["ended_early"]
        assert [["c%d" % i, p.hex()] for i, p in sends] == [s[:2] for s in b["sent"]]
        assert table_of(conn) == b["table_after"]


def test_oracle_last_sync_store_matches_reference():
    conn = sqlite_of(LAST["initial_table"])
    for step in LAST["steps"]:
        ids = sync_ref.store_last_sync(conn, 1, LAST["meta"], LAST["history_size"],
                                       [(m["member"], m["gt"], bytes.fromhex(m["packet"])) for m in step["messages"]])
        assert ids == step["packet_ids"]
        assert table_of(conn) == step["table"]


def double_table_of(conn):
    return [list(r) for r in conn.execute("SELECT sync, member1, member2 FROM double_signed_sync ORDER BY sync")]


def test_oracle_double_signed_store_matches_reference():
    """dispersy.py:1537-1541, :1567-1594 (double_signed_sync), replayed by the lifted reference _store."""
    conn = sqlite_of(DOUBLE["initial_table"])
    conn.executemany("INSERT INTO double_signed_sync (sync, member1, member2) VALUES (?, ?, ?)",
                     [tuple(r) for r in DOUBLE["initial_double"]])
    for step in DOUBLE["steps"]:
        ids = sync_ref.store_double_signed(conn, 1, DOUBLE["meta"], DOUBLE["history_size"],
                                           [(m["members"][0], m["members"][1], m["gt"], bytes.fromhex(m["packet"]))
                                            for m in step["messages"]])
        assert ids == step["packet_ids"]
        assert table_of(conn) == step["table"]
        assert double_table_of(conn) == step["double"]


# ------------------------------------------------------------------------------------------------- GPU
class _Member(object):
    def __init__(self, database_id, signature_length):
        self.database_id, self.signature_length = database_id, signature_length


class _Auth(object):
    def __init__(self, member):
        self.member = member


class _Dist(object):
    def __init__(self, gt, seq=0):
        self.global_time, self.sequence_number, self.priority = gt, seq, 128


class _Msg(object):
    def __init__(self, meta, member, gt, packet, index, seq=0, sig=60):
        self.meta, self.database_id = meta, meta.database_id
        self.authentication = _Auth(_Member(member, sig))
        self.distribution = _Dist(gt, seq)
        self.packet, self.index, self.candidate = packet, index, "c%d" % index


def store_of(table, pairs=None):
    return SyncStore.from_rows([(i, gt, meta, und, bytes.fromhex(p), mem, sq or 0)
                                for i, mem, gt, meta, und, p, sq in table], pairs=pairs)


def alive(store):
    keep = np.flatnonzero(~store.deleted)
    return sorted((int(store.rowid[r]), store.packet(int(r)).hex().upper()) for r in keep)


@pytest.mark.gpu
def test_sequence_branch_matches_reference():
    store = store_of(SEQ["table_before"])
    seq_meta = MetaMessage("seq", 2, FullSyncDistribution("ASC", 128, True,
                                                          GlobalTimePruning(SEQ["inactive"], SEQ["inactive"] + 1)))
    plain = MetaMessage("plain", 1, FullSyncDistribution("ASC", 128))
    com = SyncCommunity(store, [plain, seq_meta], global_time=SEQ["global_time"],
                        signature_length=SEQ["signature_length"])
    assert com.acceptable_global_time == SEQ["acceptable_global_time"]
    for b in SEQ["batches"]:
        msgs = [_Msg(seq_meta, m["member"], m["gt"], bytes.fromhex(m["packet"]), m["index"], m["seq"])
                for m in b["batch"]]
        com.sent_packets = []
        got = []
        for out in com._check_full_sync_distribution_batch(msgs):
            if isinstance(out, DropMessage):
                got.append((out.dropped.index, out.reason))
            elif isinstance(out, DelayMessageBySequence):
                got.append((out.delayed.index, ("delay", out.missing_low, out.missing_high)))
            else:
                got.append((out.index, None))
        assert got == [(i, _expect(r)) for i, r in b["results"]]
        assert [[c, p.hex(), why] for c, p, why in com.sent_packets] == b["sent"]
        assert alive(store) == sorted((r[0], r[5]) for r in b["table_after"])
    # the responder's index and the duplicate table after the DELETEs: every remaining (member, gt) is found,
    # every deleted one is not
    gone = np.flatnonzero(store.deleted)
    assert len(gone) > 20
    keep = np.flatnonzero(~store.deleted)
    probe = np.concatenate([gone, keep[:200]])
    verdict, _ = store.dup_check(store.member[probe], store.global_time[probe], [b"?"] * len(probe), [60] * len(probe))
    assert (verdict[:len(gone)] == 0).all() and (verdict[len(gone):] != 0).all()
    for m in (1, 2):
        assert set(store.rowid[store.live_rows(m)].tolist()) == {r[0] for r in SEQ["batches"][-1]["table_after"]
                                                               if r[3] == m and r[4] == 0}


@pytest.mark.gpu
@pytest.mark.parametrize("lazy", [False, True])
def test_last_sync_history_matches_reference(lazy):
    store = store_of(LAST["initial_table"])
    if not lazy:
        store.handle  # noqa: B018 -- the DELETEs then run on the device index
    meta = MetaMessage("last", LAST["meta"], LastSyncDistribution("ASC", 128, LAST["history_size"]))
    com = SyncCommunity(store, [meta], global_time=1)
    for step in LAST["steps"]:
        msgs = [_Msg(meta, m["member"], m["gt"], bytes.fromhex(m["packet"]), m["index"]) for m in step["messages"]]
        rows = com.store_messages(msgs)
        assert store.rowid[rows].tolist() == step["packet_ids"]
        assert alive(store) == sorted((r[0], r[5]) for r in step["table"])
        assert com.global_time == max([1] + [m["gt"] for s in LAST["steps"][:LAST["steps"].index(step) + 1]
                                             for m in s["messages"]])
    want = sorted(r[0] for r in LAST["steps"][-1]["table"])
    assert sorted(store.rowid[store.live_rows(LAST["meta"])].tolist()) == want
    # the device index: a claim over everything with an empty filter returns exactly the kept rows
    from dispersy_amd import BloomFilter
    from dispersy_amd.community import ClaimRequest
    (got,) = com.respond([ClaimRequest(1, 10 ** 6, 1, 0, BloomFilter(1024, 0.01, b"\x00"))], include_inactive=True,
                         byte_limit=1 << 40)
    assert sorted(store.rowid[got].tolist()) == want


def test_store_messages_refuses_what_it_cannot_keep_consistent():
    """store_messages checks a batch before storing any of it: a LastSync meta, or a double-member-signed one, without
    the store's member column is refused with both store copies unchanged (CPU: the store is not on the device)."""
    import pytest as _pytest
    from dispersy_amd.community import SyncCommunity
    from dispersy_amd.distribution import LastSyncDistribution, MetaMessage
    from dispersy_amd.store import SyncStore

    class D(object):
        def __init__(self, gt):
            self.global_time = gt

    class M(object):
        def __init__(self, meta, gt, member):
            self.meta, self.packet, self.distribution, self.member = meta, b"p%d" % gt, D(gt), member
            self.database_id = meta.database_id

    last = MetaMessage("last", 1, LastSyncDistribution("ASC", 128, history_size=2))
    store = SyncStore.from_rows([(1, 5, 1, 0, b"x")], ctx=object())  # no member column
    com = SyncCommunity(store, [last], global_time=10)
    with _pytest.raises(ValueError):
        com.store_messages([M(last, 7, 3)])
    assert store.n == 1
    dbl = MetaMessage("dbl", 2, LastSyncDistribution("ASC", 128, history_size=1), double_signed=True)
    store2 = SyncStore.from_rows([(1, 5, 2, 0, b"x")], ctx=object())  # no member column
    com2 = SyncCommunity(store2, [dbl], global_time=10)
    with _pytest.raises(ValueError):
        com2.store_messages([M(dbl, 7, 4)])
    assert store2.n == 1


class _DoubleAuth(object):
    """DoubleMemberAuthentication.Implementation's surface: .members, and .member = members[0] (authentication.py:276-290)."""

    def __init__(self, a, b):
        self.members = [_Member(a, 60), _Member(b, 60)]
        self.member = self.members[0]


class _DoubleMsg(_Msg):
    def __init__(self, meta, a, b, gt, packet, index):
        super(_DoubleMsg, self).__init__(meta, a, gt, packet, index)
        self.authentication = _DoubleAuth(a, b)


def _double_replay(store, com, meta):
    for step in DOUBLE["steps"]:
        msgs = [_DoubleMsg(meta, m["members"][0], m["members"][1], m["gt"], bytes.fromhex(m["packet"]), m["index"])
                for m in step["messages"]]
        rows = com.store_messages(msgs)
        assert store.rowid[rows].tolist() == step["packet_ids"]
        assert alive(store) == sorted((r[0], r[5]) for r in step["table"])
        # the double_signed_sync rows that join a live sync row: each live row's pair
        pairs = {}
        for (mid, m1, m2), rs in store._pair_groups.items():
            for r in rs:
                if not store.deleted[r]:
                    pairs[int(store.rowid[r])] = [m1, m2]
        assert sorted([k] + v for k, v in pairs.items()) == step["double"]


def _double_meta():
    return MetaMessage("double", DOUBLE["meta"], LastSyncDistribution("ASC", 128, DOUBLE["history_size"]),
                       double_signed=True)


def _double_store():
    return store_of(DOUBLE["initial_table"], pairs=[tuple(r) for r in DOUBLE["initial_double"]]), _double_meta()


def test_double_signed_history_from_a_sqlite_export():
    """A store exported from a Dispersy database (SyncStore.from_sqlite) brings its double_signed_sync rows along, so
    the per-pair LastSync history sees the pairs' older rows (before, the export dropped the table and the
    store silently kept more than history_size rows per pair).  CPU: the host copy."""
    conn = sqlite_of(DOUBLE["initial_table"])
    conn.executemany("INSERT INTO double_signed_sync (sync, member1, member2) VALUES (?, ?, ?)",
                     [tuple(r) for r in DOUBLE["initial_double"]])
    store = SyncStore.from_sqlite(conn)
    store._ctx = object()  # never uploaded
    meta = _double_meta()
    _double_replay(store, SyncCommunity(store, [meta], global_time=1), meta)


def test_double_signed_history_needs_the_pairs_of_stored_rows():
    """A store whose rows of a double-member-signed meta came without their double_signed_sync table cannot apply the
    per-pair history (pair_rows would miss the older rows): store_messages refuses the batch before storing any of
    it.  Rows of other metas do not matter, and an empty store records every pair itself."""
    meta = _double_meta()
    bare = store_of(DOUBLE["initial_table"])
    bare._ctx = object()
    step = DOUBLE["steps"][0]
    msgs = [_DoubleMsg(meta, m["members"][0], m["members"][1], m["gt"], bytes.fromhex(m["packet"]), m["index"])
            for m in step["messages"]]
    n0 = bare.n
    with pytest.raises(ValueError):
        SyncCommunity(bare, [meta], global_time=1).store_messages(msgs)
    assert bare.n == n0
    other = store_of([r[:3] + [r[3] + 1] + r[4:] for r in DOUBLE["initial_table"]])  # the rows under another meta
    other._ctx = object()
    assert other.pairs_exported(DOUBLE["meta"])
    SyncCommunity(other, [meta], global_time=1).store_messages(msgs)


def test_double_signed_history_matches_reference_host():
    """Double-member-signed LastSync messages (dispersy.py:1537-1541, :1567-1594) replayed by SyncCommunity on a store
    not yet on the device (the host copy: rows, DELETEs, double_signed_sync)."""
    store, meta = _double_store()
    store._ctx = object()  # never uploaded
    _double_replay(store, SyncCommunity(store, [meta], global_time=1), meta)


@pytest.mark.gpu
def test_double_signed_history_matches_reference():
    """The same replay with the store in HBM: the DELETEs go through dsy_store_delete, and a claim over everything
    with an empty filter returns exactly the rows the reference keeps."""
    store, meta = _double_store()
    store.handle  # noqa: B018
    com = SyncCommunity(store, [meta], global_time=1)
    _double_replay(store, com, meta)
    from dispersy_amd import BloomFilter
    from dispersy_amd.community import ClaimRequest
    (got,) = com.respond([ClaimRequest(1, 10 ** 6, 1, 0, BloomFilter(1024, 0.01, b"\x00"))], include_inactive=True,
                         byte_limit=1 << 40)
    assert sorted(store.rowid[got].tolist()) == sorted(r[0] for r in DOUBLE["steps"][-1]["table"])


def test_store_messages_meta_ids_by_batch_shape():
    """store_messages reads a message's meta id through its meta when the batch has one meta object (message.py:265-266:
    Message.database_id is its meta's), per message otherwise; each form stores the same columns (CPU, host store)."""
    from dispersy_amd.community import SyncCommunity
    from dispersy_amd.distribution import MetaMessage, SyncDistribution
    from dispersy_amd.store import SyncStore

    class D(object):
        def __init__(self, gt):
            self.global_time, self.priority = gt, 128

    class WithMeta(object):  # the reference's shape: database_id is a property of the meta
        def __init__(self, meta, gt):
            self.meta, self.packet, self.distribution = meta, b"m%d-%d" % (meta.database_id, gt), D(gt)

        @property
        def database_id(self):
            return self.meta.database_id

    class Bare(object):  # no meta: the id on the message itself
        def __init__(self, mid, gt):
            self.database_id, self.packet, self.distribution = mid, b"b%d-%d" % (mid, gt), D(gt)

    import dispersy_amd.community as community

    a = MetaMessage("a", 3, SyncDistribution("ASC", 128))
    b = MetaMessage("b", 5, SyncDistribution("ASC", 128))
    batches = [[WithMeta(a, 10 + i) for i in range(40)],                          # one meta object
               [WithMeta(a if i % 3 else b, 100 + i) for i in range(40)],         # two
               [Bare(5 if i % 2 else 3, 200 + i) for i in range(40)]]             # none
    assert community._dsyhost is not None, "the C column reader (dsy_host.c) is not built"
    reader = community._dsyhost
    try:
        for use_c in (True, False):  # the C column reader and the Python path store the same columns
            community._dsyhost = reader if use_c else None
            store = SyncStore.from_rows([(1, 1, 3, 0, b"x")], ctx=object())
            com = SyncCommunity(store, [a, b], global_time=1)
            for msgs in batches:
                rows = com.store_messages(msgs)
                assert store.meta[rows].tolist() == [m.database_id for m in msgs]
                assert store.global_time[rows].tolist() == [m.distribution.global_time for m in msgs]
                assert [store.packet(int(r)) for r in rows] == [m.packet for m in msgs]
            assert com.global_time == 239
    finally:
        community._dsyhost = reader


def test_message_columns_reader():
    """dsy_host.c message_columns: one pass over a message list -- global times (any integer type), packets, the
    bytes packets' gather list, the one-meta test by identity -- and the errors the Python getters would raise."""
    from dispersy_amd.community import _dsyhost

    assert _dsyhost is not None, "the C column reader (dsy_host.c) is not built"

    class D(object):
        def __init__(self, gt):
            self.global_time = gt

    class M(object):
        def __init__(self, gt, packet, **kw):
            self.distribution, self.packet = D(gt), packet
            self.__dict__.update(kw)

    def run(msgs):
        n = len(msgs)
        gts, lens, addrs = (np.zeros(n, dtype=np.uint64) for _ in range(3))
        out = _dsyhost.message_columns(msgs, gts, lens, addrs)
        return out, gts, lens, addrs

    meta = object()
    msgs = [M(np.uint64(2 ** 63 + 5), b"abc", meta=meta), M(7, b"", meta=meta), M(np.int32(9), b"\x00" * 300, meta=meta)]
    (packets, one, first, all_bytes), gts, lens, addrs = run(msgs)
    assert packets == [m.packet for m in msgs] and packets is not msgs
    assert one and first is meta and all_bytes
    assert gts.tolist() == [2 ** 63 + 5, 7, 9] and lens.tolist() == [3, 0, 300]
    # the addresses are the bytes' own buffers
    import ctypes
    assert ctypes.string_at(int(addrs[0]), 3) == b"abc" and ctypes.string_at(int(addrs[2]), 300) == b"\x00" * 300
    # a second meta object, no meta (None), and a packet that is not exactly bytes
    (_, one, first, all_bytes), _, _, _ = run([M(1, b"a", meta=meta), M(2, bytearray(b"b"), meta=object())])
    assert not one and first is None and not all_bytes
    (_, one, first, _), _, _, _ = run([M(1, b"a"), M(2, b"b")])
    assert one and first is None
    with pytest.raises(OverflowError):
        run([M(-1, b"a")])
    with pytest.raises(TypeError):
        run([M(1.5, b"a")])
    with pytest.raises(AttributeError):
        run([M(1, b"a"), object()])
    with pytest.raises(ValueError):
        _dsyhost.message_columns([M(1, b"a"), M(2, b"b")], np.zeros(1, dtype=np.uint64), np.zeros(2, dtype=np.uint64),
                                 np.zeros(2, dtype=np.uint64))
    with pytest.raises(TypeError):
        run(tuple(msgs))

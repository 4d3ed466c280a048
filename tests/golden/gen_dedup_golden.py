"""Golden vectors for the duplicate check of received sync packets, produced by the reference's own code.

Test infrastructure, run in the build container (where /root/reference exists):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_dedup_golden.py
`Dispersy._is_duplicate_sync_message` (dispersy.py:831-918), `Dispersy._check_full_sync_distribution_batch`
(:921-1065, both the plain branch and the sequence-number branch :954-1037) and `Dispersy._store` (:1475-1612: the
INSERT and LastSyncDistribution's history pruning) are lifted unchanged out of dispersy.py's AST, with the same
mechanical edits as gen_sync_golden.py (`__debug__` -> False, decorators dropped), and run against an sqlite3 `sync`
table built from the reference's schema string.  Only those two methods' text is parsed (the rest of dispersy.py is Python 2).  Bound in their
globals: `str`/`buffer` -> bytes, `cmp`, `Message.Implementation` (the message stand-in class), and a
`sorted` that accepts the py2 positional comparison function.  Only the resulting data is committed
(dedup_vectors.json, dedup_seq_vectors.json, laststore_vectors.json, doublestore_vectors.json).
"""
import ast
import collections
import functools
import json
import os
import sqlite3

import numpy as np

from gen_sync_golden import REF, _NoDebug, reference_schema

LIFT = ("_is_duplicate_sync_message", "_check_full_sync_distribution_batch", "_store")


def method_source(text, name):
    """The text of one method of the Dispersy class (dispersy.py as a whole is Python 2 and does not parse here):
    from its `def` line to the next line at class-body indentation, dedented."""
    lines = text.split("\n")
    start = [i for i, l in enumerate(lines) if l.startswith("    def %s(" % name)][0]
    end = start + 1
    while end < len(lines) and not (lines[end].startswith("    ") and not lines[end].startswith("     ")
                                    and lines[end].strip()):
        end += 1
    # dedent by the class-body indentation only where it is present (the SQL of _store's triple-quoted strings
    # starts at column 0)
    return "\n".join(l[4:] if l.startswith("    ") else l for l in lines[start:end])


def lift():
    text = open(os.path.join(REF, "dispersy.py")).read()
    cls = ast.Module([ast.parse(method_source(text, name)).body[0] for name in LIFT], [])

    def py2_sorted(seq, cmp=None, key=None, reverse=False):
        if cmp is not None:
            return sorted(seq, key=functools.cmp_to_key(cmp), reverse=reverse)
        return sorted(seq, key=key, reverse=reverse)

    g = dict(str=bytes, buffer=bytes, cmp=lambda a, b: (a > b) - (a < b), sorted=py2_sorted,
             DropMessage=DropMessage, DelayMessageBySequence=DelayMessageBySequence,
             Message=_Obj(Implementation=_Obj), defaultdict=collections.defaultdict,
             SyncDistribution=_Obj(Implementation=_Dist), FullSyncDistribution=FullSync, LastSyncDistribution=LastSync,
             MemberAuthentication=_Obj(Implementation=_Auth), DoubleMemberAuthentication=_DoubleAuth)
    funcs = {}
    for node in cls.body:
        if isinstance(node, ast.FunctionDef) and node.name in LIFT:
            node.decorator_list = []
            node = _NoDebug().visit(node)
            exec(compile(ast.fix_missing_locations(ast.Module([node], [])), "dispersy.py", "exec"), g)
            funcs[node.name] = g[node.name]
    assert set(funcs) == set(LIFT)
    return funcs


class DropMessage(object):
    def __init__(self, message, reason):
        self.dropped, self.reason = message, reason


class DelayMessageBySequence(object):
    """message.py:147-166."""

    def __init__(self, delayed, missing_low, missing_high):
        assert 0 < missing_low <= missing_high, (missing_low, missing_high)
        self.delayed, self.missing_low, self.missing_high = delayed, missing_low, missing_high


# stand-ins for the isinstance checks of _store (dispersy.py:1497-1567)
class _Dist(object):
    def __init__(self, **kw):
        self.__dict__.update(kw)


class FullSync(object):
    pass


class LastSync(object):
    def __init__(self, history_size, custom_callback=None):
        self.history_size, self.custom_callback = history_size, custom_callback


class _Auth(object):
    encoding = "bin"
    is_signed = True

    def __init__(self, member):
        self.member = member


class _DoubleAuth(object):
    class Implementation(object):
        pass


class _Cursor(object):
    def __init__(self, cur):
        self.cur = cur

    def __iter__(self):  # list(execute(...)) (dispersy.py:1571-1586)
        return iter(self.cur.fetchall())

    def next(self):  # py2 iterator protocol the reference calls (dispersy.py:868)
        row = self.cur.fetchone()
        if row is None:
            raise StopIteration
        return row


class _DB(object):
    def __init__(self, conn):
        self.conn = conn

    def execute(self, sql, args=(), get_lastrowid=False):
        cur = self.conn.execute(sql, args)
        return cur.lastrowid if get_lastrowid else _Cursor(cur)

    def executemany(self, sql, seq):
        self.conn.executemany(sql, list(seq))


class _Log(object):
    def debug(self, *a, **k):
        pass

    warning = debug


class StubDispersy(object):
    def __init__(self, conn, funcs):
        self._database = _DB(conn)
        self._logger = _Log()
        self.sent = []
        self._is_duplicate_sync_message = funcs["_is_duplicate_sync_message"].__get__(self)
        self.check = funcs["_check_full_sync_distribution_batch"].__get__(self)
        self.store = funcs["_store"].__get__(self)

    def _send_packets(self, candidates, packets, community, reason):
        for c in candidates:
            for p in packets:
                self.sent.append([c, p.hex(), reason])


class _Obj(object):
    def __init__(self, **kw):
        self.__dict__.update(kw)


def main():
    rng = np.random.Generator(np.random.PCG64(4242))
    sig, gt_now, inactive = 60, 5000, 3000
    conn = sqlite3.connect(":memory:")
    conn.executescript(reference_schema())
    rows, seen = [], set()
    while len(rows) < 400:
        member, gt = int(rng.integers(1, 40)), int(rng.integers(1, gt_now))
        if (member, gt) in seen:
            continue
        seen.add((member, gt))
        i = len(rows) + 1
        rows.append(dict(id=i, member=member, gt=gt, undone=0,
                         packet=(i.to_bytes(4, "big") + rng.bytes(int(rng.integers(sig + 8, 300)) - 4))))
    for i in rng.choice(len(rows), size=40, replace=False):
        rows[int(i)]["undone"] = int(rng.integers(1, len(rows) + 1))
    conn.executemany("INSERT INTO sync (id, community, member, global_time, meta_message, undone, packet) "
                     "VALUES (?, 1, ?, ?, 1, ?, ?)",
                     [(r["id"], r["member"], r["gt"], r["undone"], r["packet"]) for r in rows])
    community = _Obj(database_id=1, acceptable_global_time=gt_now + 10000, global_time=gt_now)
    meta = _Obj(distribution=_Obj(enable_sequence_number=False))
    batch = []
    for j in range(600):
        kind = int(rng.integers(0, 8))
        r = rows[int(rng.integers(0, len(rows)))]
        if kind == 0:
            member, gt, packet = int(rng.integers(40, 60)), int(rng.integers(1, gt_now)), rng.bytes(int(rng.integers(80, 200)))
        elif kind == 1:
            member, gt, packet = r["member"], r["gt"], r["packet"]
        elif kind in (2, 3):
            tail = bytearray(r["packet"][sig:])
            p = int(rng.integers(0, len(tail)))
            tail[p] = (tail[p] + (1 if kind == 2 else 255)) % 256
            if kind == 3 and rng.random() < 0.3:
                tail = tail[:len(tail) - 3]
            member, gt, packet = r["member"], r["gt"], r["packet"][:sig] + bytes(tail)
        elif kind == 4:
            member, gt, packet = r["member"], r["gt"], rng.bytes(len(r["packet"]))
        elif kind == 5 and batch:
            prev = batch[int(rng.integers(0, len(batch)))]
            member, gt, packet = prev["member"], prev["gt"], bytes.fromhex(prev["packet"]) + b"y"
        elif kind == 6:
            member, gt, packet = r["member"], gt_now + 10001 + int(rng.integers(0, 5)), r["packet"]
        else:
            member, gt, packet = int(rng.integers(1, 60)), int(rng.integers(1, gt_now - inactive)), rng.bytes(120)
        batch.append(dict(index=j, member=member, gt=gt, packet=packet.hex()))
    messages = []
    for b in batch:
        active = gt_now - b["gt"] < inactive  # GlobalTimePruning.is_active (distribution.py:80-81)
        messages.append(_Obj(index=b["index"], name="full-sync", community=community, meta=meta, database_id=1,
                             packet=bytes.fromhex(b["packet"]), candidate="c%d" % b["index"],
                             authentication=_Obj(member=_Obj(database_id=b["member"], signature_length=sig)),
                             distribution=_Obj(global_time=b["gt"], pruning=_Obj(is_active=lambda a=active: a))))
    d = StubDispersy(conn, lift())
    results = []
    for out in d.check(messages):
        if isinstance(out, DropMessage):
            results.append([out.dropped.index, out.reason])
        else:
            results.append([out.index, None])
    final = {i: bytes(p).hex() for i, p in conn.execute("SELECT id, packet FROM sync")}
    changed = {str(r["id"]): final[r["id"]] for r in rows if final[r["id"]] != r["packet"].hex()}
    out = dict(signature_length=sig, global_time=gt_now, acceptable_global_time=gt_now + 10000, inactive=inactive,
               rows=[dict(r, packet=r["packet"].hex()) for r in rows], batch=batch, results=results, sent=d.sent,
               updated=changed)
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "dedup_vectors.json"), "w") as f:
        json.dump(out, f)
    print("dedup vectors: %d messages, %d accepted, %d sent, %d updated" % (
        len(results), sum(1 for _, r in results if r is None), len(d.sent), len(changed)))


def _table(conn):
    return [list(r) for r in conn.execute("SELECT id, member, global_time, meta_message, undone, hex(packet), sequence "
                                          "FROM sync ORDER BY id")]


def seq_main():
    """The sequence-number branch of _check_full_sync_distribution_batch (dispersy.py:954-1037): per-member highest
    (global_time, sequence), duplicates by binary packet, conflicting sequence numbers (keep ours and send it back, or
    DELETE ours and everything after it), gaps (DelayMessageBySequence), lower global time with a higher sequence
    number, and the duplicate lookup by (member, global_time)."""
    rng = np.random.Generator(np.random.PCG64(777))
    sig, gt_now, inactive = 60, 4000, 3500
    conn = sqlite3.connect(":memory:")
    conn.executescript(reference_schema())
    rows, used = [], set()

    def fresh_gt(member, lo=1, hi=gt_now):
        while True:
            gt = int(rng.integers(lo, hi))
            if (member, gt) not in used:
                used.add((member, gt))
                return gt

    # meta 1: plain rows (sequence NULL); meta 2: sequence-numbered rows 1..c per member in global-time order
    for member in range(1, 31):
        for _ in range(int(rng.integers(0, 4))):
            gt = fresh_gt(member)
            rows.append(dict(member=member, gt=gt, meta=1, seq=None))
        gts = sorted(fresh_gt(member, 1, gt_now - 600) for _ in range(int(rng.integers(0, 9))))
        for j, gt in enumerate(gts):
            rows.append(dict(member=member, gt=gt, meta=2, seq=j + 1))
    for i, r in enumerate(rows):
        r["id"] = i + 1
        r["packet"] = (r["id"].to_bytes(4, "big") + rng.bytes(int(rng.integers(sig + 8, 200)) - 4))
    conn.executemany("INSERT INTO sync (id, community, member, global_time, meta_message, undone, packet, sequence) "
                     "VALUES (?, 1, ?, ?, ?, 0, ?, ?)",
                     [(r["id"], r["member"], r["gt"], r["meta"], r["packet"], r["seq"]) for r in rows])
    community = _Obj(database_id=1, acceptable_global_time=gt_now + 10000, global_time=gt_now)
    meta = _Obj(distribution=_Obj(enable_sequence_number=True))
    d = StubDispersy(conn, lift())
    table0 = _table(conn)
    batches, idx = [], 0
    for bno in range(40):
        seq_rows = {}
        for rid, member, gt, mid, _, phex, seq in _table(conn):
            if mid == 2:
                seq_rows.setdefault(member, []).append(dict(gt=gt, seq=seq, packet=bytes.fromhex(phex)))
        for v in seq_rows.values():
            v.sort(key=lambda r: r["gt"])
        plain = {}
        for rid, member, gt, mid, *_ in _table(conn):
            if mid == 1:
                plain.setdefault(member, []).append(gt)
        batch = []
        for j in range(int(rng.integers(4, 30))):
            member = int(rng.integers(1, 36))  # 31..35: members without stored rows
            mine = seq_rows.get(member, [])
            c = len(mine)
            kind = int(rng.integers(0, 10))
            seq, gt, packet = c + 1, None, rng.bytes(int(rng.integers(80, 160)))
            if kind == 0 and c:                      # binary duplicate of a stored sequence number
                r = mine[int(rng.integers(0, c))]
                seq, gt, packet = r["seq"], r["gt"], r["packet"]
            elif kind == 1 and c:                    # same sequence number, different message: (gt, packet) higher
                r = mine[int(rng.integers(0, c))]
                seq, gt = r["seq"], r["gt"] + int(rng.integers(0, 3))
                if gt == r["gt"]:
                    packet = r["packet"][:sig] + bytes([255]) + rng.bytes(20)
            elif kind == 2 and c:                    # same sequence number, (gt, packet) lower: ours and later go
                r = mine[int(rng.integers(0, c))]
                seq, gt = r["seq"], max(1, r["gt"] - int(rng.integers(1, 40)))
            elif kind == 3:                          # a gap: delayed
                seq = c + int(rng.integers(2, 5))
            elif kind == 4 and c:                    # next sequence number but an older global time
                gt = max(1, mine[-1]["gt"] - int(rng.integers(0, 50)))
            elif kind == 5 and plain.get(member):    # next sequence number at the (member, gt) of a plain row
                gt = plain[member][0]
            elif kind == 6:                          # beyond the acceptable global time
                gt = gt_now + 10001 + int(rng.integers(0, 9))
            elif kind == 7:                          # inactive (pruned)
                gt = int(rng.integers(1, max(2, gt_now - inactive)))
            if gt is None:
                top = mine[-1]["gt"] if c else 0
                gt = int(rng.integers(top + 1, gt_now + 200))
            batch.append(dict(index=idx, member=member, gt=int(gt), seq=int(seq), packet=bytes(packet).hex()))
            idx += 1
        messages = []
        for b in batch:
            active = gt_now - b["gt"] < inactive
            messages.append(_Obj(index=b["index"], name="seq-sync", community=community, meta=meta, database_id=2,
                                 packet=bytes.fromhex(b["packet"]), candidate="c%d" % b["index"],
                                 authentication=_Obj(member=_Obj(database_id=b["member"], signature_length=sig)),
                                 distribution=_Obj(global_time=b["gt"], sequence_number=b["seq"],
                                                   pruning=_Obj(is_active=lambda a=active: a))))
        d.sent = []
        results, ended = [], False
        gen = d.check(messages)
        while True:
            try:
                out = next(gen)
            except StopIteration:
                break
            except RuntimeError as e:
                # py2: a StopIteration inside a generator ends it silently (the `.next()` of a LIMIT 1 OFFSET query
                # that finds no row, dispersy.py:986-987); py3 turns that into this RuntimeError (PEP 479)
                assert isinstance(e.__cause__, StopIteration), e
                ended = True
                break
            if isinstance(out, DropMessage):
                results.append([out.dropped.index, out.reason])
            elif isinstance(out, DelayMessageBySequence):
                results.append([out.delayed.index, ["delay", out.missing_low, out.missing_high]])
            else:
                results.append([out.index, None])
        batches.append(dict(batch=batch, results=results, ended_early=ended, sent=d.sent, table_after=_table(conn)))
    out = dict(signature_length=sig, global_time=gt_now, acceptable_global_time=gt_now + 10000, inactive=inactive,
               table_before=table0, batches=batches)
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "dedup_seq_vectors.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    kinds = collections.Counter(r if r is None or isinstance(r, str) else r[0]
                                for b in batches for _, r in b["results"])
    print("seq vectors: %d batches, %d ended early, %d rows deleted" % (
        len(batches), sum(b["ended_early"] for b in batches), len(table0) - len(batches[-1]["table_after"])),
        dict(kinds))


def laststore_main():
    """_store (dispersy.py:1475-1612) for a LastSyncDistribution meta: INSERT, then DELETE every member's rows
    beyond the newest history_size (by global time, :1581-1591); batches in sequence, the table after each."""
    rng = np.random.Generator(np.random.PCG64(909))
    conn = sqlite3.connect(":memory:")
    conn.executescript(reference_schema())
    used = set()
    n0 = 0
    for member in range(1, 25):
        for gt in sorted(rng.choice(np.arange(1, 500), size=int(rng.integers(0, 3)), replace=False).tolist()):
            n0 += 1
            used.add((member, gt))
            conn.execute("INSERT INTO sync (id, community, member, global_time, meta_message, undone, packet) "
                         "VALUES (?, 1, ?, ?, 3, 0, ?)", (n0, member, gt, rng.bytes(40)))
    stored = []

    class Community(object):
        database_id = 1

        def update_global_time(self, gt):
            stored.append(["update_global_time", gt])

        def dispersy_store(self, messages):
            stored.append(["dispersy_store", [m.index for m in messages]])

    community = Community()
    meta = _Obj(name="last", community=community, database_id=3, authentication=_Obj(),
                distribution=LastSync(history_size=2))
    d = StubDispersy(conn, lift())
    initial = _table(conn)
    steps, idx = [], 0
    for b in range(12):
        msgs, members = [], set()
        for _ in range(int(rng.integers(1, 12))):
            member = int(rng.integers(1, 30))
            gt = int(rng.integers(1, 1000))
            if (member, gt) in used:
                continue
            used.add((member, gt))
            packet = rng.bytes(int(rng.integers(30, 90))) + b"\x01"
            m = _Obj(index=idx, name="last", community=community, meta=meta, database_id=3, packet=packet,
                     authentication=_Auth(_Obj(database_id=member, has_identity=lambda c: True)),
                     distribution=_Dist(global_time=gt))
            idx += 1
            msgs.append(m)
        if not msgs:
            continue
        stored.clear()
        d.store(msgs)
        steps.append(dict(messages=[dict(index=m.index, member=m.authentication.member.database_id,
                                         gt=m.distribution.global_time, packet=m.packet.hex()) for m in msgs],
                          packet_ids=[m.packet_id for m in msgs], calls=list(stored), table=_table(conn)))
    out = dict(history_size=2, meta=3, initial_table=initial, steps=steps)
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "laststore_vectors.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("laststore vectors: %d batches, table %d -> %d rows" % (len(steps), len(initial), len(steps[-1]["table"])))


class _DoubleImpl(_DoubleAuth.Implementation):
    """A DoubleMemberAuthentication.Implementation stand-in: .member is members[0] (authentication.py:276-290)."""
    encoding = "bin"
    is_signed = True

    def __init__(self, members):
        self.members = members
        self.member = members[0]


def _double_table(conn):
    return [list(r) for r in conn.execute("SELECT sync, member1, member2 FROM double_signed_sync ORDER BY sync")]


def doublestore_main():
    """_store (dispersy.py:1475-1612) for a double-member-signed LastSyncDistribution meta: each INSERT into sync
    (member = members[0]) is paired with one into double_signed_sync (the member pair, smaller id first, :1537-1541);
    the history is kept per member pair -- rows joined through double_signed_sync, ordered by (global_time, packet)
    (:1567-1578) -- and what falls out is DELETEd from both tables (:1589-1594).  Batches in sequence; both tables
    after each.  Member ids are few, so pairs recur in both orders and global times tie within a pair."""
    rng = np.random.Generator(np.random.PCG64(4242))
    conn = sqlite3.connect(":memory:")
    conn.executescript(reference_schema())
    used = set()
    n0 = 0
    for _ in range(30):
        a, b = (int(x) for x in rng.choice(np.arange(1, 9), size=2, replace=False))
        gt = int(rng.integers(1, 12))
        if (a, gt) in used:
            continue
        used.add((a, gt))
        n0 += 1
        conn.execute("INSERT INTO sync (id, community, member, global_time, meta_message, undone, packet) "
                     "VALUES (?, 1, ?, ?, 5, 0, ?)", (n0, a, gt, rng.bytes(int(rng.integers(20, 40)))))
        conn.execute("INSERT INTO double_signed_sync (sync, member1, member2) VALUES (?, ?, ?)", (n0, min(a, b), max(a, b)))
    stored = []

    class Community(object):
        database_id = 1

        def update_global_time(self, gt):
            stored.append(["update_global_time", gt])

        def dispersy_store(self, messages):
            stored.append(["dispersy_store", [m.index for m in messages]])

    community = Community()
    meta = _Obj(name="double", community=community, database_id=5, authentication=_DoubleAuth(),
                distribution=LastSync(history_size=2))
    d = StubDispersy(conn, lift())
    initial, initial_double = _table(conn), _double_table(conn)
    steps, idx = [], 0
    for _ in range(16):
        msgs = []
        for _ in range(int(rng.integers(1, 9))):
            a, b = (int(x) for x in rng.choice(np.arange(1, 9), size=2, replace=False))
            gt = int(rng.integers(1, 16))
            if (a, gt) in used:
                continue
            used.add((a, gt))
            packet = rng.bytes(int(rng.integers(20, 60))) + b"\x01"
            m = _Obj(index=idx, name="double", community=community, meta=meta, database_id=5, packet=packet,
                     authentication=_DoubleImpl([_Obj(database_id=a, has_identity=lambda c: True),
                                                 _Obj(database_id=b, has_identity=lambda c: True)]),
                     distribution=_Dist(global_time=gt))
            idx += 1
            msgs.append(m)
        if not msgs:
            continue
        stored.clear()
        d.store(msgs)
        steps.append(dict(messages=[dict(index=m.index, members=[x.database_id for x in m.authentication.members],
                                         gt=m.distribution.global_time, packet=m.packet.hex()) for m in msgs],
                          packet_ids=[m.packet_id for m in msgs], calls=list(stored), table=_table(conn),
                          double=_double_table(conn)))
    out = dict(history_size=2, meta=5, initial_table=initial, initial_double=initial_double, steps=steps)
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "doublestore_vectors.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("doublestore vectors: %d batches, table %d -> %d rows, double_signed_sync %d -> %d" % (
        len(steps), len(initial), len(steps[-1]["table"]), len(initial_double), len(steps[-1]["double"])))


if __name__ == "__main__":
    import sys
    if sys.argv[1:] == ["double"]:
        doublestore_main()
    else:
        main()
        seq_main()
        laststore_main()
        doublestore_main()

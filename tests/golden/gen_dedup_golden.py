"""Golden vectors for the duplicate check of received sync packets, produced by the reference's own code.

Test infrastructure, run in the build container (where /root/reference exists):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_dedup_golden.py
`Dispersy._is_duplicate_sync_message` (dispersy.py:831-918) and `Dispersy._check_full_sync_distribution_batch`
(:921-1065) are lifted unchanged out of dispersy.py's AST, with the same mechanical edits as gen_sync_golden.py
(`__debug__` -> False, decorators dropped), and run against an sqlite3 `sync` table built from the reference's
schema string.  Only those two methods' text is parsed (the rest of dispersy.py is Python 2).  Bound in their
globals: `str`/`buffer` -> bytes, `cmp`, `Message.Implementation` (the message stand-in class), and a
`sorted` that accepts the py2 positional comparison function.  Only the resulting data is committed
(dedup_vectors.json).
"""
import ast
import functools
import json
import os
import sqlite3

import numpy as np

from gen_sync_golden import REF, _NoDebug, reference_schema

LIFT = ("_is_duplicate_sync_message", "_check_full_sync_distribution_batch")


def method_source(text, name):
    """The text of one method of the Dispersy class (dispersy.py as a whole is Python 2 and does not parse here):
    from its `def` line to the next line at class-body indentation, dedented."""
    lines = text.split("\n")
    start = [i for i, l in enumerate(lines) if l.startswith("    def %s(" % name)][0]
    end = start + 1
    while end < len(lines) and not (lines[end].startswith("    ") and not lines[end].startswith("     ")
                                    and lines[end].strip()):
        end += 1
    return "\n".join(l[4:] for l in lines[start:end])


def lift():
    text = open(os.path.join(REF, "dispersy.py")).read()
    cls = ast.Module([ast.parse(method_source(text, name)).body[0] for name in LIFT], [])

    def py2_sorted(seq, cmp=None, key=None, reverse=False):
        if cmp is not None:
            return sorted(seq, key=functools.cmp_to_key(cmp), reverse=reverse)
        return sorted(seq, key=key, reverse=reverse)

    g = dict(str=bytes, buffer=bytes, cmp=lambda a, b: (a > b) - (a < b), sorted=py2_sorted,
             DropMessage=DropMessage, DelayMessageBySequence=None, Message=_Obj(Implementation=_Obj))
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


class _Cursor(object):
    def __init__(self, cur):
        self.cur = cur

    def next(self):  # py2 iterator protocol the reference calls (dispersy.py:868)
        row = self.cur.fetchone()
        if row is None:
            raise StopIteration
        return row


class _DB(object):
    def __init__(self, conn):
        self.conn = conn

    def execute(self, sql, args=()):
        return _Cursor(self.conn.execute(sql, args))


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


if __name__ == "__main__":
    main()

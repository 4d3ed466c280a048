"""Golden vectors for undo / redo of stored packets, produced by the reference's own code.

Test infrastructure, run in the build container (where /root/reference exists):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_undo_golden.py
`Community.on_undo` (community.py:3457-3481) and `Community._update_timerange` (:3606-3642) are lifted out of
community.py's AST (decorators dropped, `__debug__` -> False, as gen_sync_golden.py does), `Dispersy.
_is_duplicate_sync_message` (dispersy.py:831-918) out of dispersy.py (gen_dedup_golden.lift), and the responder
`_get_packets_for_bloomfilters` (community.py:2746-2811) with the byte-limited loop of :2555-2567 as in
gen_sync_golden.py.  They run over one sqlite3 `sync` table built from the reference's schema: a script of undo
batches (undo messages and DispersyDuplicatedUndo pairs) and timeline re-evaluations (the timeline's verdict is this
script's input: a set of packet ids it no longer allows), and after every step the `undone` column, the answers to
16 claims and the duplicate check's undo-proof sends for 12 received copies of stored packets are recorded.  Only
the data is committed (undo_vectors.json).
"""
import ast
import itertools
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from gen_dedup_golden import StubDispersy, _Obj  # noqa: E402
from gen_dedup_golden import lift as lift_dispersy  # noqa: E402
from gen_sync_golden import (REF, META_SETS, DrawLog, StubCommunity, _NoDebug, build_db, lift_methods,  # noqa: E402
                             meta_json, metas_of, reference_schema)


class DispersyDuplicatedUndo(object):  # community.py:74-79
    name = candidate = u"_DUPLICATED_UNDO_"

    def __init__(self, low_message, high_message):
        self.low_message = low_message
        self.high_message = high_message


class _Implementation(object):
    pass


def lift_undo():
    tree = ast.parse(open(os.path.join(REF, "community.py")).read())
    cls = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "Community"][0]
    g = dict(DispersyDuplicatedUndo=DispersyDuplicatedUndo, Message=_Obj(Implementation=_Implementation),
             groupby=itertools.groupby, str=bytes, unicode=str)
    funcs = {}
    for node in cls.body:
        if isinstance(node, ast.FunctionDef) and node.name in ("on_undo", "_update_timerange"):
            node.decorator_list = []
            node = _NoDebug().visit(node)
            exec(compile(ast.fix_missing_locations(ast.Module([node], [])), "community.py", "exec"), g)
            funcs[node.name] = g[node.name]
    assert set(funcs) == {"on_undo", "_update_timerange"}
    return funcs


class _UndoMessage(_Implementation):
    """An undo message as on_undo reads it (community.py:3471-3474)."""
    name = u"dispersy-undo-other"

    def __init__(self, packet_id, member, global_time, meta):
        self.packet_id = packet_id
        self.payload = _Obj(process_undo=True, member=_Obj(database_id=member), global_time=global_time,
                            packet=_Obj(meta=meta))


class _Meta(object):
    def __init__(self, database_id, name):
        self.database_id, self.name = database_id, name
        self.undone, self.redone = [], []

    def undo_callback(self, items):
        self.undone.extend(items)

    def handle_callback(self, messages):
        self.redone.extend(messages)


class _UndoCommunity(object):
    def __init__(self, conn, funcs, revoked):
        self.database_id = 1
        self._dispersy = StubDispersy(conn, lift_dispersy())
        self._dispersy.convert_packet_to_message = self._convert
        self._logger = _Obj(debug=lambda *a, **k: None)
        self.timeline = _Obj(check=lambda message: (message.packet_id not in revoked, []))
        self.on_undo = funcs["on_undo"].__get__(self)
        self._update_timerange = funcs["_update_timerange"].__get__(self)
        self.conn = conn

    def _convert(self, packet, community):
        return _Obj(name="m", distribution=_Obj(global_time=0), authentication=_Obj(member=None))


def main():
    schema = reference_schema()
    spec = META_SETS["random"][:1] + [("desc", 2, "DESC", 200, None)]
    rng = np.random.Generator(np.random.PCG64(5150))
    rows, seen = [], set()
    while len(rows) < 420:
        member, gt = int(rng.integers(1, 25)), int(rng.integers(1, 900))
        if (member, gt) in seen:
            continue
        seen.add((member, gt))
        rid = len(rows) + 1
        packet = rid.to_bytes(4, "big") + rng.bytes(int(rng.integers(64, 320)) - 4)
        rows.append(dict(id=rid, member=member, gt=gt, meta=int(rng.choice([1, 2])), undone=0, packet=packet.hex()))
    for i in rng.choice(len(rows), size=20, replace=False):
        rows[int(i)]["undone"] = int(rng.integers(1, len(rows) + 1))
    conn = build_db(schema, rows)
    packets = {r["id"]: bytes.fromhex(r["packet"]) for r in rows}
    by_packet = {v: k for k, v in packets.items()}

    # the responder's claims (fixed), filters over ~80% of the packets
    B = load_bloom()
    draws = DrawLog(0)
    sync_funcs, _ = lift_methods(B, draws)
    claims = []
    for q in range(16):
        modulo = int(rng.choice([1, 1, 2, 3]))
        lo = int(rng.integers(1, 400))
        hi = int(rng.integers(lo, 950))
        bf = B.BloomFilter(10160 if q % 2 else 4096, 0.01 if q % 2 else 0.001, bytes([q]))
        bf.add_keys([p for p in packets.values() if rng.random() < 0.8])
        claims.append(dict(time_low=lo, time_high=hi, modulo=modulo, offset=int(rng.integers(0, modulo)), m=bf.size,
                           k=bf.functions, prefix=bytes([q]).hex(), filter=bf.bytes.hex(),
                           byte_limit=int(rng.choice([5120, 1 << 40])), _bf=bf))
    metas = metas_of(spec)
    meta_objs = {mid: _Meta(mid, name) for name, mid, _, _, _ in spec}

    def responses():
        out = []
        for c in claims:
            stub = StubCommunity(conn, metas, 1000, 11000, 10160, 0.01, draws)
            reqs = [(c, c["time_low"], c["time_high"], c["offset"], c["modulo"])]
            sent, budget = [], c["byte_limit"]
            for _, gen in sync_funcs["_get_packets_for_bloomfilters"](stub, reqs, include_inactive=True):
                for packet, in c["_bf"].not_filter(gen):
                    sent.append(by_packet[bytes(packet)])
                    budget -= len(packet)
                    if budget <= 0:
                        break
            out.append(sent)
        return out

    revoked = set()
    com = _UndoCommunity(conn, lift_undo(), revoked)
    steps = []
    for step in range(24):
        ev = dict(step=step)
        if step % 3 != 2:  # a batch of undo messages (and duplicated-undo pairs)
            entries, msgs = [], []
            for _ in range(int(rng.integers(1, 7))):
                r = rows[int(rng.integers(0, len(rows)))]
                undo_id = int(rng.integers(1, len(rows) + 1))
                member, gt = r["member"], r["gt"]
                if rng.random() < 0.1:  # no such (member, global_time): the UPDATE changes nothing
                    member, gt = 99, int(rng.integers(1, 900))
                if rng.random() < 0.25:
                    low = _Obj(packet_id=undo_id)
                    high = _Obj(authentication=_Obj(member=_Obj(database_id=member)), distribution=_Obj(global_time=gt))
                    msgs.append(DispersyDuplicatedUndo(low, high))
                else:
                    msgs.append(_UndoMessage(undo_id, member, gt, meta_objs[r["meta"]]))
                entries.append([undo_id, member, gt])
            com.on_undo(msgs)
            ev["on_undo"] = entries
        else:  # the timeline re-evaluates one meta's range: it revokes some packets and allows others again
            mid = int(rng.choice([1, 2]))
            lo = int(rng.integers(1, 600))
            hi = int(rng.integers(lo, 950))
            ids = [r["id"] for r in rows if r["meta"] == mid and lo <= r["gt"] <= hi]
            for i in ids:
                if rng.random() < 0.15:
                    revoked.add(i)
                elif rng.random() < 0.5:
                    revoked.discard(i)
            meta = meta_objs[mid]
            meta.undone, meta.redone = [], []
            com._update_timerange(meta, lo, hi)
            ev["timeline"] = dict(meta=mid, time_low=lo, time_high=hi,
                                  undo=sorted(m.packet_id for _, _, m in meta.undone),
                                  redo=sorted(m.packet_id for m in meta.redone))
        ev["undone"] = [list(x) for x in conn.execute("SELECT id, undone FROM sync ORDER BY id")]
        ev["responses"] = responses()
        # received exact copies of stored packets: an undone one makes the duplicate check send the undo proof
        dsp = com._dispersy
        dsp.sent = []
        picks = [rows[int(i)] for i in rng.integers(0, len(rows), size=12)]
        for j, r in enumerate(picks):
            msg = _Obj(community=_Obj(database_id=1), candidate="c%d" % j, packet=packets[r["id"]], name="m",
                       authentication=_Obj(member=_Obj(database_id=r["member"], signature_length=60)),
                       distribution=_Obj(global_time=r["gt"]))
            dsp._is_duplicate_sync_message(msg)
        ev["dup_checks"] = [[r["member"], r["gt"], r["id"]] for r in picks]
        ev["proofs"] = [[c, p, why] for c, p, why in dsp.sent]
        steps.append(ev)
    for c in claims:
        del c["_bf"]
    out = dict(generator="tests/golden/gen_undo_golden.py",
               source="/root/reference/community.py on_undo, _update_timerange, _get_packets_for_bloomfilters; "
                      "dispersy.py _is_duplicate_sync_message; lifted via ast",
               metas=meta_json(spec), rows=rows, claims=claims, responder_global_time=1000, steps=steps)
    with open(os.path.join(HERE, "undo_vectors.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    n_undone = [sum(1 for _, u in s["undone"] if u) for s in steps]
    print("undo vectors: %d steps, undone rows %d..%d, proofs %d" % (len(steps), min(n_undone), max(n_undone),
                                                                     sum(len(s["proofs"]) for s in steps)))


def load_bloom():
    import gen_golden
    return gen_golden.load_reference_bloomfilter()


if __name__ == "__main__":
    main()

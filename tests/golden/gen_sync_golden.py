"""Golden vectors for the sync-selection half of the hot path, produced by the reference's own code.

Test infrastructure; invoked by gen_golden.py (see that file for how the reference is loaded).  The sync
methods are lifted unchanged out of community.py's AST, with exactly three mechanical edits:
  * `__debug__` -> `False`  (the debug blocks call py2-only `str.encode("HEX")`);
  * decorators dropped  (`runtime_duration_warning` / `attach_runtime_statistics` are Twisted-side
    instrumentation, util.py:62-158);
  * the py2 byte-string literal `prefix='\x00'` (community.py:837, :933) -> `b'\x00'`.
They run against an sqlite3 database built from the reference's schema string (dispersydatabase.py:17-68).
"""
import ast
import json
import math
import os
import random as pyrandom
import sqlite3
import types
from collections import OrderedDict

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

LIFT = ("_get_packets_for_bloomfilters", "_select_and_fix", "_select_bloomfilter_range",
        "_dispersy_claim_sync_bloom_filter_largest", "_dispersy_claim_sync_bloom_filter_modulo",
        "dispersy_claim_sync_bloom_filter", "dispersy_store")


class _NoDebug(ast.NodeTransformer):
    def visit_Name(self, node):
        if node.id == "__debug__":
            return ast.copy_location(ast.Constant(False), node)
        return node

    def visit_keyword(self, node):
        # py2 byte-string literal `prefix='\x00'` (community.py:837, :933) -> bytes, as bloomfilter.py's `""` default
        self.generic_visit(node)
        if node.arg == "prefix" and isinstance(node.value, ast.Constant) and isinstance(node.value.value, str):
            node.value = ast.copy_location(ast.Constant(node.value.value.encode("latin-1")), node.value)
        return node


def reference_schema():
    tree = ast.parse(open(os.path.join(REF, "dispersydatabase.py")).read())
    env = {}
    for node in tree.body:
        if isinstance(node, ast.Assign) and node.targets[0].id in ("LATEST_VERSION", "schema"):
            exec(compile(ast.Module([node], []), "dispersydatabase.py", "exec"), env)
    return env["schema"]


# ---- stand-ins for the objects the lifted methods touch (distribution.py:68-242, message.py meta) ----------
class Pruning(object):
    pass


class NoPruning(Pruning):
    pass


class GlobalTimePruning(Pruning):
    def __init__(self, inactive, pruned):
        self.inactive_threshold = inactive
        self.prune_threshold = pruned


class SyncDistribution(object):
    def __init__(self, direction, priority, pruning=None):
        self.synchronization_direction = direction
        self.priority = priority
        self.pruning = pruning if pruning is not None else NoPruning()


class DirectDistribution(object):
    priority = 0


class Meta(object):
    def __init__(self, name, database_id, distribution):
        self.name, self.database_id, self.distribution = name, database_id, distribution


class _Py2Dict(OrderedDict):
    def itervalues(self):
        return iter(self.values())


class _Cid(bytes):
    def encode(self, codec):  # py2 str.encode("HEX"), used in non-debug log arguments (community.py:724-727)
        return self.hex()


class _Logger(object):
    def debug(self, *a, **k):
        pass
    info = warning = debug


class _Stats(object):
    sync_bloom_new = sync_bloom_reuse = sync_bloom_send = sync_bloom_skip = 0


class _DB(object):
    def __init__(self, conn):
        self.conn = conn

    def execute(self, sql, args=()):
        return self.conn.execute(sql, args)


class _Dispersy(object):
    def __init__(self, db):
        self.database = self._database = db


class DrawLog(object):
    """Records every random draw the reference makes, in call order, so the build's mirror can replay them."""

    def __init__(self, seed):
        self.rng = pyrandom.Random(seed)
        self.log = []

    def random(self):
        v = self.rng.random()
        self.log.append(["random", v])
        return v

    def expovariate(self, lambd):
        v = self.rng.expovariate(lambd)
        self.log.append(["expovariate", v])
        return v

    def randint(self, a, b):
        v = self.rng.randint(a, b)
        self.log.append(["randint", v])
        return v


def lift_methods(B, draws):
    tree = ast.parse(open(os.path.join(REF, "community.py")).read())
    cls = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "Community"][0]
    funcs = {}
    g = dict(BloomFilter=B.BloomFilter, SyncDistribution=SyncDistribution, GlobalTimePruning=GlobalTimePruning,
             unicode=str, str=bytes, long=int, ceil=math.ceil, chr=lambda i: bytes([i]),
             random=draws.random, randint=draws.randint, SyncCache=None)
    # SyncCache (community.py:57-67) is lifted too: dispersy_claim_sync_bloom_filter constructs it.
    sc = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "SyncCache"][0]
    exec(compile(ast.fix_missing_locations(ast.Module([sc], [])), "community.py", "exec"), g)
    for node in cls.body:
        if isinstance(node, ast.FunctionDef) and node.name in LIFT:
            node.decorator_list = []
            node = _NoDebug().visit(node)
            mod = ast.fix_missing_locations(ast.Module([node], []))
            exec(compile(mod, "community.py", "exec"), g)
            funcs[node.name] = g[node.name]
    assert set(funcs) == set(LIFT), set(LIFT) - set(funcs)
    return funcs, g


class StubCommunity(object):
    _SKIP_CURVE_STEPS = [0, 0, 0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9]  # community.py:86
    _SKIP_STEPS = len(_SKIP_CURVE_STEPS)

    def __init__(self, conn, metas, global_time, acceptable_global_time, bits, error_rate, draws):
        self._dispersy = _Dispersy(_DB(conn))
        self._meta_messages = _Py2Dict((m.name, m) for m in metas)
        self.global_time = global_time
        self.acceptable_global_time = acceptable_global_time
        self.dispersy_sync_bloom_filter_bits = bits
        self.dispersy_sync_bloom_filter_error_rate = error_rate
        self.dispersy_sync_skip_enable = True
        self.dispersy_sync_cache_enable = True
        self._random = draws
        self._nrsyncpackets = 0
        self._logger = _Logger()
        self._statistics = _Stats()
        self._sync_cache = None
        self._sync_cache_skip_count = 0
        self._cid = _Cid(b"c" * 20)
        self.cid = self._cid

    def get_meta_messages(self):
        return list(self._meta_messages.values())


# -------------------------------------------------------------------------------------------- scenarios
def build_db(schema, rows):
    conn = sqlite3.connect(":memory:")
    conn.executescript(schema)
    conn.execute("INSERT INTO community(id, master, member, classification) VALUES (1, 1, 1, 'x')")
    for mid in sorted({r["meta"] for r in rows}):
        conn.execute("INSERT INTO meta_message(id, community, name) VALUES (?, 1, ?)", (mid, "m%d" % mid))
    conn.executemany("INSERT INTO sync(id, community, member, global_time, meta_message, undone, packet, sequence) "
                     "VALUES (?, 1, ?, ?, ?, ?, ?, 0)",
                     [(r["id"], r["member"], r["gt"], r["meta"], r["undone"], bytes.fromhex(r["packet"])) for r in rows])
    return conn


def make_rows(seed, n, metas, gt_max, undone_frac, lo=40, hi=260, members=7, skew=False):
    """Unique (member, gt) pairs (schema UNIQUE(community, member, global_time)), random meta, random undone."""
    rng = np.random.Generator(np.random.PCG64(seed))
    seen, rows = set(), []
    rid = 0
    while len(rows) < n:
        member = int(rng.integers(1, members + 1))
        gt = int(min(gt_max, rng.zipf(1.3))) if skew else int(rng.integers(1, gt_max + 1))
        if (member, gt) in seen:
            continue
        seen.add((member, gt))
        rid += 1 + int(rng.integers(0, 3))  # rowids with gaps
        length = int(rng.integers(lo, hi + 1))
        packet = rid.to_bytes(4, "big") + rng.bytes(length - 4)
        rows.append(dict(id=rid, member=member, gt=gt, meta=int(metas[int(rng.integers(0, len(metas)))]),
                         undone=int(rng.random() < undone_frac), packet=packet.hex()))
    return rows


META_SETS = {
    # test_sync / test_pruning shapes (tests/debugcommunity/community.py:100-190); meta 9 is not syncable (priority <= 32)
    "det": [("asc", 1, "ASC", 128, None), ("desc", 2, "DESC", 128, None), ("high", 3, "ASC", 200, None),
            ("medium", 4, "ASC", 150, None), ("low", 5, "DESC", 100, None), ("prune", 6, "ASC", 128, (10, 20)),
            ("nosync", 9, "ASC", 16, None)],
    "random": [("asc", 1, "ASC", 128, None), ("rand", 7, "RANDOM", 128, None), ("desc", 2, "DESC", 140, None)],
    "single": [("full", 1, "ASC", 128, None)],
}


def metas_of(spec):
    return [Meta(name, mid, SyncDistribution(d, prio, GlobalTimePruning(*pr) if pr else None))
            for name, mid, d, prio, pr in spec]


def meta_json(spec):
    return [dict(name=n, id=mid, direction=d, priority=p, pruning=pr) for n, mid, d, p, pr in spec]


def respond_scenarios(B, funcs, schema):
    out = []
    configs = [
        dict(name="det_small", metas="det", seed=101, n=260, gt_max=120, undone=0.1),
        dict(name="det_skew", metas="det", seed=102, n=300, gt_max=400, undone=0.05, skew=True),
        dict(name="single_big", metas="single", seed=103, n=600, gt_max=5000, undone=0.0),
        dict(name="random_meta", metas="random", seed=104, n=240, gt_max=100, undone=0.1),
    ]
    bloom_shapes = [(10160, 0.01), (4096, 0.001), (1 << 15, 0.01), (8, 0.1)]
    for cfg in configs:
        spec = META_SETS[cfg["metas"]]
        rows = make_rows(cfg["seed"], cfg["n"], [m[1] for m in spec], cfg["gt_max"], cfg["undone"],
                         skew=cfg.get("skew", False))
        conn = build_db(schema, rows)
        by_packet = {bytes.fromhex(r["packet"]): r["id"] for r in rows}
        rng = np.random.Generator(np.random.PCG64(cfg["seed"] + 1))
        requests = []
        gmax = max(r["gt"] for r in rows)
        for q in range(40):
            modulo = int(rng.choice([1, 1, 2, 3, 5, 7, 16]))
            offset = int(rng.integers(0, modulo))
            lo = int(rng.integers(1, max(2, gmax // 2)))
            hi = int(rng.integers(lo, gmax + 3)) if q % 5 else 0  # time_high 0 => responder's global_time
            m, f = bloom_shapes[q % len(bloom_shapes)]
            prefix = bytes([int(rng.integers(0, 256))])
            bf = B.BloomFilter(m, f, prefix)
            # the requester knows a random ~70% of the store
            known = [bytes.fromhex(r["packet"]) for r in rows if rng.random() < 0.7]
            bf.add_keys(iter(known))
            include_inactive = bool(q % 3 == 0)
            byte_limit = int(rng.choice([5120, 5120, 1000, 300, 1 << 40]))
            responder_gt = int(gmax + rng.integers(0, 30))
            requests.append(dict(time_low=lo, time_high=hi, modulo=modulo, offset=offset, m=bf.size, k=bf.functions,
                                 prefix=prefix.hex(), filter=bf.bytes.hex(), include_inactive=include_inactive,
                                 byte_limit=byte_limit, responder_global_time=responder_gt, _bf=bf))
        results = []
        for req in requests:
            stub = StubCommunity(conn, metas_of(spec), req["responder_global_time"], req["responder_global_time"] + 10000,
                                 10160, 0.01, DrawLog(0))
            # on_introduction_request (community.py:2545-2553): time_high 0 => own global_time; clamp 2^63-1
            time_low = min(req["time_low"], 2 ** 63 - 1)
            time_high = min(req["time_high"] if req["time_high"] else stub.global_time, 2 ** 63 - 1)
            reqs = [(req, time_low, time_high, req["offset"], req["modulo"])]
            for _, gen in funcs["_get_packets_for_bloomfilters"](stub, reqs, include_inactive=req["include_inactive"]):
                all_rows = [by_packet[p] for p, in gen]
            # the responder's byte-limited loop, community.py:2555-2567
            byte_limit = req["byte_limit"]
            packets = []
            stub2 = StubCommunity(conn, metas_of(spec), req["responder_global_time"], 0, 10160, 0.01, DrawLog(0))
            for _, gen in funcs["_get_packets_for_bloomfilters"](stub2, reqs, include_inactive=req["include_inactive"]):
                for packet, in req["_bf"].not_filter(gen):
                    packets.append(packet)
                    byte_limit -= len(packet)
                    if byte_limit <= 0:
                        break
            missing_all = [i for i in all_rows
                           if bytes(conn.execute("SELECT packet FROM sync WHERE id=?", (i,)).fetchone()[0]) not in req["_bf"]]
            results.append(dict(selected=all_rows, missing_all=missing_all, response=[by_packet[p] for p in packets]))
        for req in requests:
            del req["_bf"]
        out.append(dict(name=cfg["name"], metas=meta_json(spec), rows=rows, requests=requests, results=results,
                        random_directions=[m[1] for m in spec if m[2] == "RANDOM"]))
    return out


def claim_scenarios(B, funcs, schema):
    """_dispersy_claim_sync_bloom_filter_largest / _modulo with every random draw recorded (community.py:763-933)."""
    out = []
    cfgs = [
        dict(name="few_rows", metas="det", seed=201, n=120, gt_max=300, bits=10160),   # < capacity: 'first capacity rows'
        dict(name="tiny_filter", metas="det", seed=202, n=400, gt_max=2000, bits=1024),  # capacity 106 -> pivot ranges
        dict(name="dup_gt", metas="single", seed=203, n=500, gt_max=90, bits=1024),     # many equal gts: drop trailing group
        dict(name="skew", metas="det", seed=204, n=500, gt_max=3000, bits=2048, skew=True),
        dict(name="empty", metas="single", seed=205, n=0, gt_max=10, bits=10160),
    ]
    for cfg in cfgs:
        spec = META_SETS[cfg["metas"]]
        rows = make_rows(cfg["seed"], cfg["n"], [m[1] for m in spec], cfg["gt_max"], 0.1,
                         skew=cfg.get("skew", False)) if cfg["n"] else []
        conn = build_db(schema, rows)
        gmax = max([r["gt"] for r in rows] or [1])
        calls = []
        for trial in range(16):
            strategy = "largest" if trial % 4 != 3 else "modulo"
            draws = DrawLog(cfg["seed"] * 100 + trial)
            funcs_g = funcs["_g"]
            funcs_g["random"], funcs_g["randint"] = draws.random, draws.randint
            nrsync = [0, 10 ** 9, -1][trial % 3]
            if nrsync == -1:
                nrsync = conn.execute("SELECT count(*) FROM sync WHERE undone = 0").fetchone()[0]
            stub = StubCommunity(conn, metas_of(spec), gmax + trial, gmax + trial + 10000, cfg["bits"], 0.01, draws)
            stub._nrsyncpackets = nrsync
            fn = funcs["_dispersy_claim_sync_bloom_filter_%s" % strategy]
            call = dict(strategy=strategy, global_time=stub.global_time, acceptable_global_time=stub.acceptable_global_time,
                        nrsyncpackets_in=nrsync)
            try:
                lo, hi, modulo, offset, bf = fn(stub, None)
                call["result"] = dict(time_low=lo, time_high=hi, modulo=modulo, offset=offset, m=bf.size, k=bf.functions,
                                      prefix=bf.prefix.hex(), filter=bf.bytes.hex())
            except Exception as e:  # noqa: BLE001 - e.g. IndexError at community.py:857 on a stale _nrsyncpackets
                call["error"] = type(e).__name__
            call.update(nrsyncpackets_out=stub._nrsyncpackets, draws=draws.log)
            calls.append(call)
        out.append(dict(name=cfg["name"], metas=meta_json(spec), rows=rows, bits=cfg["bits"], error_rate=0.01, calls=calls))
    return out


def claim_state_machine(B, funcs, schema):
    """dispersy_claim_sync_bloom_filter (community.py:709-758) + dispersy_store (:680-707): reuse / skip / stats."""
    spec = META_SETS["single"]
    rows = make_rows(301, 200, [1], 800, 0.0)
    conn = build_db(schema, rows)
    draws = DrawLog(3030)
    g = funcs["_g"]
    g["random"], g["randint"] = draws.random, draws.randint
    stub = StubCommunity(conn, metas_of(spec), 800, 10800, 10160, 0.01, draws)
    stub.dispersy_sync_bloom_filter_strategy = lambda rc: funcs["_dispersy_claim_sync_bloom_filter_largest"](stub, rc)

    class RC(object):
        helper_candidate = None

    class Dist(object):
        def __init__(self, gt):
            self.priority, self.global_time = 128, gt

    class Msg(object):
        def __init__(self, gt, packet):
            self.distribution, self.packet, self.candidate = Dist(gt), packet, None

    script = []
    for step in range(40):
        n_before = len(draws.log)
        res = funcs["dispersy_claim_sync_bloom_filter"](stub, RC())
        ev = dict(step=step, draws=draws.log[n_before:], result=None)
        if res is not None:
            lo, hi, modulo, offset, bf = res
            ev["result"] = dict(time_low=lo, time_high=hi, modulo=modulo, offset=offset, prefix=bf.prefix.hex(),
                                filter=bf.bytes.hex())
        # feed "responses" on some steps: store new packets and mark a response received
        if step % 3 == 1 and stub._sync_cache is not None:
            newp = [(int(stub._sync_cache.time_low) + j, os.urandom(0) + bytes([step, j]) * 30) for j in range(3)]
            funcs["dispersy_store"](stub, [Msg(gt, p) for gt, p in newp])
            stub._sync_cache.responses_received += 1
            ev["stored"] = [[gt, p.hex()] for gt, p in newp]
        ev["stats"] = [stub._statistics.sync_bloom_new, stub._statistics.sync_bloom_reuse,
                       stub._statistics.sync_bloom_send, stub._statistics.sync_bloom_skip]
        ev["skip_count"] = stub._sync_cache_skip_count
        script.append(ev)
    return dict(metas=meta_json(spec), rows=rows, global_time=800, acceptable_global_time=10800, script=script)


class _Candidate(object):
    def __init__(self, global_time):
        self.global_time = global_time


class _Clock(object):
    def __init__(self):
        self.now = 1000.0

    def __call__(self):
        return self.now


def acceptable_global_time_vectors():
    """Community.acceptable_global_time (community.py:1015-1058) lifted from the AST (the @property decorator dropped;
    `time` bound to a test clock; py2 `/` -> `//` at :1041): the median of > 5 candidate opinions (py2 floor index), the own global time
    otherwise, the + range, the 2^63-1 ceiling, the 5-second cache and the bloom-sync-disabled branch."""
    tree = ast.parse(open(os.path.join(REF, "community.py")).read())
    cls = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "Community"][0]
    node = [n for n in cls.body if isinstance(n, ast.FunctionDef) and n.name == "acceptable_global_time"][0]
    node.decorator_list = []
    # the one py2-ism: `options[len(options) / 2]` (:1041) is integer division in py2
    divs = [n for n in ast.walk(node) if isinstance(n, ast.BinOp) and isinstance(n.op, ast.Div)]
    assert len(divs) == 1
    divs[0].op = ast.FloorDiv()
    clock = _Clock()
    g = dict(time=clock)
    exec(compile(ast.fix_missing_locations(ast.Module([node], [])), "community.py", "exec"), g)
    fn = g["acceptable_global_time"]

    class Stub(object):
        pass

    rng = np.random.Generator(np.random.PCG64(404))
    scripts = []
    for trial in range(40):
        stub = Stub()
        pick = lambda vals: vals[int(rng.integers(0, len(vals)))]  # noqa: E731
        stub._global_time = pick([0, 1, 50, 9000, 12000, 2 ** 63 - 5000, 2 ** 63 - 1])
        stub.dispersy_acceptable_global_time_range = pick([10000, 1, 0, 123456])
        stub.dispersy_enable_bloom_filter_sync = bool(trial % 9 != 4)
        stub._acceptable_global_time_deadline = 0.0
        stub._acceptable_global_time_cache = stub._global_time
        clock.now = 1000.0
        steps = []
        for step in range(8):
            n = int(rng.integers(0, 12))
            gts = [int(x) for x in rng.integers(0, 20000, size=n)]
            if step % 3 == 2:
                gts = [0] * int(rng.integers(0, 4)) + gts  # global_time 0 opinions are ignored
            cands = [_Candidate(x) for x in gts]
            stub.dispersy_yield_verified_candidates = lambda c=cands: iter(c)
            if step % 4 == 3:
                stub._global_time += int(rng.integers(0, 5000))
            clock.now += pick([0.0, 1.5, 4.99, 5.01, 20.0])
            steps.append(dict(now=clock.now, own_global_time=stub._global_time, candidates=gts, result=fn(stub)))
        scripts.append(dict(enable=stub.dispersy_enable_bloom_filter_sync,
                            range=stub.dispersy_acceptable_global_time_range, steps=steps))
    with open(os.path.join(HERE, "acceptable_vectors.json"), "w") as f:
        json.dump(dict(generator="tests/golden/gen_sync_golden.py acceptable_global_time_vectors",
                       source="/root/reference/community.py:1015-1058 lifted via ast", scripts=scripts), f,
                  separators=(",", ":"))
    return len(scripts)


def main(B):
    acceptable_global_time_vectors()
    schema = reference_schema()
    draws = DrawLog(0)
    funcs, g = lift_methods(B, draws)
    for name in LIFT:  # the strategies call self._select_and_fix / self._select_bloomfilter_range
        setattr(StubCommunity, name, funcs[name])
    funcs["_g"] = g
    resp = respond_scenarios(B, funcs, schema)
    claim = claim_scenarios(B, funcs, schema)
    sm = claim_state_machine(B, funcs, schema)
    with open(os.path.join(HERE, "sync_vectors.json"), "w") as f:
        json.dump(dict(generator="tests/golden/gen_sync_golden.py",
                       source="/root/reference/community.py methods lifted via ast (see module docstring)",
                       schema_tables=["sync", "meta_message"], respond=resp, claim=claim, state_machine=sm),
                  f, separators=(",", ":"))
    print("respond scenarios:", len(resp), "claim scenarios:", len(claim))

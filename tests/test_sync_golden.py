"""Sync surface parity against the reference's own outputs (tests/golden/sync_vectors.json).

CPU tests: the host-side selection of _get_packets_for_bloomfilters (SQL order restated over the store index).
GPU tests: the batched HIP responder (selection + digest + probe + byte-limited compaction), the claim
strategies (filters built on the GPU from store rows) and the claim state machine.
"""
import numpy as np
import pytest

from dispersy_amd import BloomFilter
from dispersy_amd.community import ClaimRequest, SyncCommunity
from dispersy_amd.distribution import GlobalTimePruning, MetaMessage, SyncDistribution
from dispersy_amd.store import SyncStore
from golden_util import Replay, load

SYNC = load("sync_vectors.json")


def metas_of(spec):
    return [MetaMessage(m["name"], m["id"], SyncDistribution(m["direction"], m["priority"],
                                                             GlobalTimePruning(*m["pruning"]) if m["pruning"] else None))
            for m in spec]


def store_of(rows):
    return SyncStore.from_rows([(r["id"], r["gt"], r["meta"], r["undone"], bytes.fromhex(r["packet"])) for r in rows])


def claim_of(req):
    return BloomFilter(bytes.fromhex(req["filter"]), req["k"], bytes.fromhex(req["prefix"]))


def resolved(req, gt):
    return ClaimRequest(min(req["time_low"], 2 ** 63 - 1), min(req["time_high"] or gt, 2 ** 63 - 1), req["modulo"],
                        req["offset"], claim_of(req))


@pytest.mark.parametrize("sc", SYNC["respond"], ids=[s["name"] for s in SYNC["respond"]])
def test_host_selection_order(sc):
    """_get_packets_for_bloomfilters yields exactly the reference's rows in the reference's order."""
    store = store_of(sc["rows"])
    random_metas = set(sc["random_directions"])
    meta_of = {r["id"]: r["meta"] for r in sc["rows"]}
    id_of_packet = {bytes.fromhex(r["packet"]): r["id"] for r in sc["rows"]}
    for req, res in zip(sc["requests"], sc["results"]):
        gt = req["responder_global_time"]
        com = SyncCommunity(store, metas_of(sc["metas"]), global_time=gt)
        q = resolved(req, gt)
        [(msg, gen)] = list(com._get_packets_for_bloomfilters([("m", q.time_low, q.time_high, q.offset, q.modulo)],
                                                               include_inactive=req["include_inactive"]))
        got = [id_of_packet[p] for p, in gen]
        if random_metas:
            det = lambda ids: [i for i in ids if meta_of[i] not in random_metas]  # noqa: E731
            assert det(got) == det(res["selected"]) and sorted(got) == sorted(res["selected"])
        else:
            assert got == res["selected"]


def _check_random_response(got, res, req, sc, store):
    random_metas = set(sc["random_directions"])
    meta_of = {r["id"]: r["meta"] for r in sc["rows"]}
    ref = res["response"]
    n_det = 0
    while n_det < len(ref) and meta_of[ref[n_det]] not in random_metas:
        n_det += 1
    assert got[:n_det] == ref[:n_det]
    missing = set(res["missing_all"])
    assert set(got) <= missing and len(set(got)) == len(got)
    lengths = [store.length(store.row_of_id(i)) for i in got]
    limit = req["byte_limit"]
    assert all(sum(lengths[:i]) < limit for i in range(1, len(lengths)))  # every packet but the first had budget
    total_missing = sum(store.length(store.row_of_id(i)) for i in missing)
    if len(got) < len(missing):
        assert sum(lengths) >= limit  # stopped only after crossing the limit
    else:
        assert sum(lengths) == total_missing


@pytest.mark.gpu
@pytest.mark.parametrize("sc", SYNC["respond"], ids=[s["name"] for s in SYNC["respond"]])
def test_respond_matches_reference(sc):
    """The batched HIP responder returns the reference's response for every claim."""
    store = store_of(sc["rows"])
    for req, res in zip(sc["requests"], sc["results"]):
        gt = req["responder_global_time"]
        com = SyncCommunity(store, metas_of(sc["metas"]), global_time=gt)
        [rows] = com.respond([resolved(req, gt)], include_inactive=req["include_inactive"], byte_limit=req["byte_limit"])
        got = store.rowid[rows].tolist()
        if sc["random_directions"]:
            _check_random_response(got, res, req, sc, store)
        else:
            assert got == res["response"], (req, got, res["response"])


@pytest.mark.gpu
def test_respond_batched_equals_single():
    """All claims of a scenario in ONE call (shared responder parameters) == one call per claim."""
    sc = [s for s in SYNC["respond"] if s["name"] == "det_small"][0]
    store = store_of(sc["rows"])
    gt = max(r["gt"] for r in sc["rows"]) + 7
    com = SyncCommunity(store, metas_of(sc["metas"]), global_time=gt)
    reqs = [resolved(r, gt) for r in sc["requests"]]
    batched = com.respond(reqs, include_inactive=False, byte_limit=1000)
    single = [com.respond([q], include_inactive=False, byte_limit=1000)[0] for q in reqs]
    assert [b.tolist() for b in batched] == [s.tolist() for s in single]


@pytest.mark.gpu
@pytest.mark.parametrize("sc", SYNC["claim"], ids=[s["name"] for s in SYNC["claim"]])
def test_claim_strategies_match_reference(sc):
    store = store_of(sc["rows"])
    for call in sc["calls"]:
        draws = Replay(call["draws"])

        class Com(SyncCommunity):
            @property
            def dispersy_sync_bloom_filter_bits(self):
                return sc["bits"]

        com = Com(store, metas_of(sc["metas"]), global_time=call["global_time"], rng=draws, random_source=draws)
        com._nrsyncpackets = call["nrsyncpackets_in"]
        fn = (com._dispersy_claim_sync_bloom_filter_largest if call["strategy"] == "largest"
              else com._dispersy_claim_sync_bloom_filter_modulo)
        if "error" in call:
            with pytest.raises(Exception) as ei:
                fn(None)
            assert type(ei.value).__name__ == call["error"]
            continue
        lo, hi, modulo, offset, bf = fn(None)
        exp = call["result"]
        assert com.acceptable_global_time == call["acceptable_global_time"]
        assert (lo, hi, modulo, offset) == (exp["time_low"], exp["time_high"], exp["modulo"], exp["offset"])
        assert (bf.size, bf.functions, bf.prefix.hex()) == (exp["m"], exp["k"], exp["prefix"])
        assert bf.bytes.hex() == exp["filter"]
        assert com._nrsyncpackets == call["nrsyncpackets_out"]
        assert not draws.log


@pytest.mark.gpu
def test_claim_state_machine_matches_reference():
    """dispersy_claim_sync_bloom_filter reuse / skip / statistics + dispersy_store cache updates."""
    sm = SYNC["state_machine"]
    store = store_of(sm["rows"])
    draws = Replay([d for ev in sm["script"] for d in ev["draws"]])
    com = SyncCommunity(store, metas_of(sm["metas"]), global_time=sm["global_time"], rng=draws, random_source=draws)

    class RC(object):
        helper_candidate = None

    class Dist(object):
        def __init__(self, gt):
            self.priority, self.global_time = 128, gt

    class Msg(object):
        def __init__(self, gt, packet):
            self.distribution, self.packet, self.candidate = Dist(gt), packet, None

    for ev in sm["script"]:
        res = com.dispersy_claim_sync_bloom_filter(RC())
        if ev["result"] is None:
            assert res is None
        else:
            lo, hi, modulo, offset, bf = res
            exp = ev["result"]
            assert (lo, hi, modulo, offset, bf.prefix.hex()) == (exp["time_low"], exp["time_high"], exp["modulo"],
                                                                  exp["offset"], exp["prefix"])
            assert bf.bytes.hex() == exp["filter"]
        if "stored" in ev:
            com.dispersy_store([Msg(gt, bytes.fromhex(p)) for gt, p in ev["stored"]])
            com._sync_cache.responses_received += 1
        st = com._statistics
        assert [st.sync_bloom_new, st.sync_bloom_reuse, st.sync_bloom_send, st.sync_bloom_skip] == ev["stats"]
        assert com._sync_cache_skip_count == ev["skip_count"]
    assert not draws.log


@pytest.mark.gpu
@pytest.mark.parametrize("sc", [s for s in SYNC["respond"] if not s["random_directions"]],
                         ids=[s["name"] for s in SYNC["respond"] if not s["random_directions"]])
def test_respond_wire_matches_reference(sc):
    """Claims that fit the wire (1-byte prefix, m < 2^16, k < 256) encoded as introduction-request sync blocks
    (conversion.py:712-730), decoded and answered in one call (respond_wire): the reference's response; a corrupt
    block in the same batch is dropped with the decoder's reason and does not disturb the others."""
    from dispersy_amd.conversion import DropPacket, encode_sync_blocks
    store = store_of(sc["rows"])
    n = 0
    for req, res in zip(sc["requests"], sc["results"]):
        bf = claim_of(req)
        if len(bf.prefix) != 1 or bf.size >= 1 << 16 or req["time_low"] >= 1 << 63 or req["time_high"] >= 1 << 63:
            continue
        gt = req["responder_global_time"]
        com = SyncCommunity(store, metas_of(sc["metas"]), global_time=gt)
        if com.global_time != gt:
            continue
        [blk] = encode_sync_blocks([(req["time_low"], req["time_high"], req["modulo"], req["offset"], bf)])
        bad = blk[:-1]
        out = com.respond_wire([bad, blk, bad], include_inactive=req["include_inactive"], byte_limit=req["byte_limit"])
        assert isinstance(out[0], DropPacket) and str(out[0]) == "Invalid number of bytes available"
        assert isinstance(out[2], DropPacket)
        assert store.rowid[out[1]].tolist() == res["response"], req
        n += 1
    assert n > 0


def test_respond_wire_batch_dies_on_a_bloom_constructor_assert():
    """A sync block whose (k, m) the reference's BloomFilter constructor rejects makes _decode_introduction_request
    raise AssertionError, which the batch loop does not catch (community.py:2078-2090): no claim of the batch is
    answered.  respond_wire raises before any responder work (host-side decode only, no GPU call)."""
    import struct as _struct
    from dispersy_amd.conversion import encode_sync_blocks
    sc = SYNC["respond"][0]
    store = store_of(sc["rows"])
    com = SyncCommunity(store, metas_of(sc["metas"]), global_time=500)
    [good] = encode_sync_blocks([(1, 0, 1, 0, BloomFilter(4096, 0.001, b"x"))])
    asserting = _struct.pack(">QQHHBH", 1, 0, 1, 0, 40, 4096) + b"x" + bytes(512)  # k=40 needs 640 digest bits
    with pytest.raises(AssertionError):
        com.respond_wire([good, asserting, good])

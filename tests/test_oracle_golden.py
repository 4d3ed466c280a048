"""Pin the CPU oracle (oracle/) against the golden vectors the reference itself produced.  CPU only."""
import hashlib

import pytest

from golden_util import Replay, expected_bytes, keys_for, load, sqlite_from_rows
from oracle import bloom_ref, sync_ref
from oracle.bloom_ref import OracleBloom

BLOOM = load("bloom_vectors.json")
SYNC = load("sync_vectors.json")


def oracle_filter(case):
    ctor, prefix = case["ctor"], bytes.fromhex(case["prefix"])
    if ctor[0] == "m_f":
        return OracleBloom.from_m_f(ctor[1], float(ctor[2]), prefix)
    return OracleBloom.from_f_n(float(ctor[1]), ctor[2], prefix)


@pytest.mark.parametrize("case", BLOOM["cases"], ids=[c["name"] for c in BLOOM["cases"]])
def test_oracle_bloom_case(case):
    e = case["expect"]
    keys, probes = keys_for(case["keys"]), keys_for(case["probes"])
    bf = oracle_filter(case)
    assert (bf.m, bf.k, bf.hash_name, bf.chunk) == (e["m"], e["k"], e["hash"], e["chunk"])
    assert [bf.indices(k) for k in keys[:64]] == e["indices"]
    assert [bf.indices(p) for p in probes[:16]] == e["probe_indices"]
    bf.add_keys(keys)
    raw = bf.to_bytes()
    assert hashlib.sha256(raw).hexdigest() == e["bytes_sha256"]
    assert raw == expected_bytes(e)
    assert bf.bits_checked == e["bits_checked"]
    assert [1 if p in bf else 0 for p in probes] == e["present"]
    assert [i for _, i in bf.not_filter((p, i) for i, p in enumerate(probes))] == e["missing"]
    clone = OracleBloom.from_bytes(raw, bf.k, bf.prefix)
    assert clone.to_bytes() == raw


def test_oracle_chunk_q():
    for row in BLOOM["chunk_q"]:
        bf = OracleBloom(row["m"], row["k"], bytes.fromhex(row["prefix"]))
        assert (bf.hash_name, bf.chunk) == (row["hash"], row["chunk"])
        assert [bf.indices(k) for k in keys_for(row["keys"])] == row["indices"]


def test_oracle_ctor_sizing():
    for row in BLOOM["ctor"]:
        if row["ctor"] == "bad":
            continue
        if row["ctor"] == "m_f":
            make = lambda: OracleBloom.from_m_f(row["a"], row["b"])  # noqa: E731
        else:
            make = lambda: OracleBloom.from_f_n(row["a"], row["b"])  # noqa: E731
        if "error" in row:
            with pytest.raises(Exception) as ei:
                make()
            assert type(ei.value).__name__ == row["error"]
            continue
        bf = make()
        assert (bf.m, bf.k, bf.hash_name, bf.chunk) == (row["m"], row["k"], row["hash"], row["chunk"])
        for f, cap in row.get("capacity", {}).items():
            assert bloom_ref.capacity_for(bf.m, float(f)) == cap


def _ref_bloom(req):
    return OracleBloom.from_bytes(bytes.fromhex(req["filter"]), req["k"], bytes.fromhex(req["prefix"]))


@pytest.mark.parametrize("sc", SYNC["respond"], ids=[s["name"] for s in SYNC["respond"]])
def test_oracle_respond(sc):
    conn = sqlite_from_rows(sc["rows"])
    random_metas = set(sc["random_directions"])
    meta_of = {r["id"]: r["meta"] for r in sc["rows"]}
    for req, res in zip(sc["requests"], sc["results"]):
        gt = req["responder_global_time"]
        hi = min(req["time_high"] or gt, 2 ** 63 - 1)
        args = (min(req["time_low"], 2 ** 63 - 1), hi, req["offset"], req["modulo"])
        rows = sync_ref.selected_rows(conn, sc["metas"], args[0], hi, args[2], args[3], gt, req["include_inactive"])
        got = sync_ref.respond_lists(conn, sc["metas"], args, _ref_bloom(req), gt, req["byte_limit"],
                                     req["include_inactive"])
        if not random_metas:
            assert [i for i, _ in rows] == res["selected"]
            assert got == res["response"]
        else:
            det = lambda ids: [i for i in ids if meta_of[i] not in random_metas]  # noqa: E731
            assert sorted(i for i, _ in rows) == sorted(res["selected"])
            assert det([i for i, _ in rows]) == det(res["selected"])
            if req["byte_limit"] >= 1 << 40:
                assert sorted(got) == sorted(res["response"])


@pytest.mark.parametrize("sc", SYNC["claim"], ids=[s["name"] for s in SYNC["claim"]])
def test_oracle_claim(sc):
    conn = sqlite_from_rows(sc["rows"])
    for call in sc["calls"]:
        draws = Replay(call["draws"])
        try:
            if call["strategy"] == "largest":
                res, nrsync = sync_ref.claim_largest(conn, sc["metas"], sc["bits"], sc["error_rate"], call["global_time"],
                                                     call["acceptable_global_time"], call["nrsyncpackets_in"], draws,
                                                     OracleBloom)
            else:
                res, nrsync = sync_ref.claim_modulo(conn, sc["metas"], sc["bits"], sc["error_rate"],
                                                    call["acceptable_global_time"], draws, OracleBloom)
        except IndexError:
            assert call.get("error") == "IndexError"
            continue
        assert "error" not in call
        lo, hi, modulo, offset, bf = res
        exp = call["result"]
        assert (lo, hi, modulo, offset) == (exp["time_low"], exp["time_high"], exp["modulo"], exp["offset"])
        assert (bf.m, bf.k, bf.prefix.hex()) == (exp["m"], exp["k"], exp["prefix"])
        assert bf.to_bytes().hex() == exp["filter"]
        assert nrsync == call["nrsyncpackets_out"]
        assert not draws.log

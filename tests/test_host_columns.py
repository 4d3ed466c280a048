"""dsy_host.c claim_columns: SyncCommunity.respond's per-claim columns -- the four range fields and the BloomFilter's
16-byte (record, filter) address pair -- read in one C pass, against the Python getters respond() falls back to
(community.py:2531-2572 in the reference; time bounds clamp to 2^63-1 as :2545-2548 do).  CPU only."""
import itertools
import operator

import numpy as np
import pytest

from dispersy_amd import BloomFilter
from dispersy_amd.community import MAX_GT, ClaimRequest, _dsyhost

pytestmark = pytest.mark.skipif(_dsyhost is None, reason="the C column reader (dsy_host.c) is not built")


def c_columns(reqs):
    ranges, words = np.zeros(4 * len(reqs), dtype=np.uint64), np.zeros(2 * len(reqs), dtype=np.uint64)
    _dsyhost.claim_columns(reqs, ranges, words)
    return ranges.tolist(), words.tobytes()


def py_columns(reqs):
    def bound(t):  # past 2^64: 2^63 - 1; otherwise as given (the library clamps above 2^63 - 1)
        return MAX_GT if t >= 2 ** 64 else int(t)
    out = []
    for q in reqs:
        out += [bound(q.time_low), bound(q.time_high), int(q.modulo), int(q.offset)]
    return out, b"".join(map(operator.attrgetter("_refs"), map(operator.itemgetter(4), reqs)))


def test_claim_columns_match_the_python_getters():
    bfs = [BloomFilter(m, 0.01, b"\x01") for m in (1024, 10160, 4096)]
    reqs = [ClaimRequest(i + 1, i + 1000, 1 + i % 3, i % 2, bfs[i % 3]) for i in range(300)]
    reqs += [ClaimRequest(np.uint64(5), np.int64(2 ** 62), np.uint32(7), np.uint8(3), bfs[0]),  # numpy integers
             ClaimRequest(2 ** 63 + 1, 2 ** 64 - 1, 1, 0, bfs[1]),   # above 2^63: passed on, the library clamps
             ClaimRequest(1, 2 ** 70, 1, 0, bfs[2]),                 # past 2^64: stored as 2^63 - 1
             ClaimRequest(2 ** 80, 2 ** 80, 2, 1, bfs[0])]
    assert c_columns(reqs) == py_columns(reqs)
    assert c_columns(tuple(reqs)) == py_columns(reqs)
    assert c_columns([]) == ([], b"")


def test_claim_columns_errors():
    bf = BloomFilter(1024, 0.01, b"\x01")
    with pytest.raises(OverflowError):
        c_columns([ClaimRequest(-1, 5, 1, 0, bf)])
    with pytest.raises(OverflowError):
        c_columns([ClaimRequest(1, 5, 2 ** 64, 0, bf)])
    with pytest.raises(TypeError):
        c_columns([ClaimRequest(1.5, 5, 1, 0, bf)])
    with pytest.raises(TypeError):
        c_columns([(1, 5, 1, 0)])              # not a ClaimRequest (four fields)
    with pytest.raises(AttributeError):
        c_columns([ClaimRequest(1, 5, 1, 0, object())])
    with pytest.raises(TypeError):
        _dsyhost.claim_columns(iter([]), np.zeros(0, dtype=np.uint64), np.zeros(0, dtype=np.uint64))
    with pytest.raises(ValueError):
        _dsyhost.claim_columns([ClaimRequest(1, 5, 1, 0, bf)], np.zeros(3, dtype=np.uint64),
                               np.zeros(2, dtype=np.uint64))


def test_respond_python_and_c_paths_build_the_same_call(monkeypatch):
    """respond() hands the library the same (ranges, refs) with and without the C reader (the library call itself is
    replaced: CPU)."""
    import dispersy_amd.community as community
    from dispersy_amd.community import SyncCommunity

    seen = []

    def fake(self, reqs, R, blob, include_inactive, byte_limit, random_seed, refs=None):
        seen.append((np.asarray(refs[0]).tolist(), bytes(refs[1])))
        return []

    monkeypatch.setattr(SyncCommunity, "_respond_requests", fake)
    bfs = [BloomFilter(10160, 0.01, bytes([i % 256])) for i in range(64)]
    reqs = [ClaimRequest(i, i + 2 ** 70 * (i % 2), 1 + i % 5, i % 3, bfs[i]) for i in range(64)]
    com = SyncCommunity.__new__(SyncCommunity)
    reader = community._dsyhost
    com.respond(reqs)
    monkeypatch.setattr(community, "_dsyhost", None)
    com.respond(reqs)
    monkeypatch.setattr(community, "_dsyhost", reader)
    com.respond(list(itertools.islice(reqs, 10)))
    assert seen[0] == seen[1] and seen[2][1] == seen[0][1][:160]


def test_claim_columns_getter_that_mutates_the_list():
    """A `_refs` getter that pops and re-appends the caller's list (same length, possibly a reallocated item array)
    while claim_columns reads it: the reader works from its own snapshot of the requests (dsy_host.c)."""
    real = BloomFilter(1024, 0.01, b"\x01")
    reqs = []

    class Mutating:
        @property
        def _refs(self):
            for _ in range(64):          # grow and shrink: a list reallocates its item array as it goes
                reqs.extend([None] * 1000)
                del reqs[-1000:]
            reqs.append(reqs.pop(0))     # pop-then-append keeps the length
            return real._refs

    reqs[:] = [ClaimRequest(i + 1, i + 10, 1, 0, Mutating()) for i in range(50)]
    want = [[i + 1, i + 10, 1, 0] for i in range(50)]
    ranges, words = c_columns(reqs)
    assert [ranges[4 * i:4 * i + 4] for i in range(50)] == want
    assert words == real._refs * 50

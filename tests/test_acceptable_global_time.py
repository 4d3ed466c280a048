"""SyncCommunity.acceptable_global_time against the reference's own property (community.py:1015-1058), lifted from
the AST by tests/golden/gen_sync_golden.py:acceptable_global_time_vectors and replayed step by step: candidate
opinions (global_time 0 ignored; median = the lower middle opinion when more than 5), the own global time otherwise,
the range, the 2^63-1 ceiling, the 5-second cache and the bloom-sync-disabled branch.  Host logic only."""
from dispersy_amd.community import SyncCommunity
from golden_util import load


class _Cand(object):
    def __init__(self, gt):
        self.global_time = gt


class _Clock(object):
    now = 0.0

    def __call__(self):
        return self.now


class _NoSync(SyncCommunity):
    @property
    def dispersy_enable_bloom_filter_sync(self):
        return False


def test_acceptable_global_time_replays_reference():
    scripts = load("acceptable_vectors.json")["scripts"]
    assert len(scripts) == 40
    for si, sc in enumerate(scripts):
        clock = _Clock()
        first = sc["steps"][0]["own_global_time"]
        cls = SyncCommunity if sc["enable"] else _NoSync
        com = cls(store=None, meta_messages=[], global_time=first, clock=clock)
        com.dispersy_acceptable_global_time_range = sc["range"]
        for st in sc["steps"]:
            com._global_time = st["own_global_time"]
            com.set_verified_candidates(_Cand(g) for g in st["candidates"])
            clock.now = st["now"]
            assert com.acceptable_global_time == st["result"], (si, st)

"""The parts of Dispersy's message model the sync hot path reads (distribution.py:68-242 of the reference):
per meta-message priority, synchronisation direction and GlobalTimePruning thresholds."""


class Pruning(object):
    pass


class NoPruning(Pruning):
    """distribution.py:29-66 -- never inactive, never pruned."""


class GlobalTimePruning(Pruning):
    """distribution.py:68-114: active while community_gt - gt < inactive, pruned from community_gt - gt >= pruned."""

    def __init__(self, inactive, pruned):
        assert isinstance(inactive, int), type(inactive)
        assert isinstance(pruned, int), type(pruned)
        assert 0 < inactive < pruned, [inactive, pruned]
        self.inactive_threshold = inactive
        self.prune_threshold = pruned


class SyncDistribution(object):
    """distribution.py:142-242 (the Full/Last variants differ only in storage policy, not in sync selection)."""

    def __init__(self, synchronization_direction="ASC", priority=127, pruning=None):
        assert synchronization_direction in ("ASC", "DESC", "RANDOM"), synchronization_direction
        assert isinstance(priority, int) and 0 <= priority <= 255, priority
        self.synchronization_direction = synchronization_direction
        self.priority = priority
        self.pruning = pruning if pruning is not None else NoPruning()

    @property
    def synchronization_direction_value(self):
        return {"ASC": 1, "DESC": -1, "RANDOM": 0}[self.synchronization_direction]


class FullSyncDistribution(SyncDistribution):
    """distribution.py:245-288: optionally sequence-numbered per member (enable_sequence_number): received messages are
    then checked against each member's highest stored sequence number (dispersy.py:954-1037)."""

    def __init__(self, synchronization_direction="ASC", priority=127, enable_sequence_number=False, pruning=None):
        assert isinstance(enable_sequence_number, bool)
        super(FullSyncDistribution, self).__init__(synchronization_direction, priority, pruning)
        self.enable_sequence_number = enable_sequence_number


class LastSyncDistribution(SyncDistribution):
    """distribution.py:291-313: only the newest history_size messages per member are kept; Dispersy._store deletes
    the older ones after every INSERT (dispersy.py:1558-1591).  custom_callback: (check, delete) pair; delete(messages)
    returns the (id, global_time) items to DELETE instead."""

    def __init__(self, synchronization_direction="ASC", priority=127, history_size=1, pruning=None, custom_callback=None):
        assert isinstance(history_size, int) and history_size > 0
        assert not custom_callback or isinstance(custom_callback, tuple)
        super(LastSyncDistribution, self).__init__(synchronization_direction, priority, pruning)
        self.history_size = history_size
        self.custom_callback = custom_callback


class DirectDistribution(object):
    """Messages that are never synced by bloom filters (distribution.py:316-325)."""
    priority = 0


class MetaMessage(object):
    """The subset of a Message meta the sync path needs: name, database id (sync.meta_message) and distribution;
    double_signed: the meta uses DoubleMemberAuthentication (authentication.py), whose messages the reference also
    records in the double_signed_sync table (dispersy.py:1537-1541)."""

    def __init__(self, name, database_id, distribution, double_signed=False):
        self.name, self.database_id, self.distribution = name, database_id, distribution
        self.double_signed = bool(double_signed)

    @property
    def syncable(self):
        # community.py:767, :2790-2794: SyncDistribution with priority > 32
        return isinstance(self.distribution, SyncDistribution) and self.distribution.priority > 32

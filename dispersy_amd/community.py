"""The sync surface of Dispersy's `Community` (community.py of the reference), over a `SyncStore` in HBM.

Kept (same names, argument meaning, return values and statistics):
  dispersy_claim_sync_bloom_filter(request_cache)      community.py:709-758   (reuse / adaptive skip / new claim)
  _dispersy_claim_sync_bloom_filter_largest(rc)         community.py:763-837   (default strategy)
  _select_bloomfilter_range / _select_and_fix           community.py:839-903
  _dispersy_claim_sync_bloom_filter_modulo(rc)          community.py:908-933
  dispersy_store(messages)                              community.py:680-707   (cached-claim update)
  _get_packets_for_bloomfilters(requests, include_inactive)  community.py:2746-2811
  the byte-limited responder loop                       community.py:2531-2572
and the overridable properties of community.py:599-678, :935-941 (the reference's plugin hooks).

The responder runs as ONE batched call into the HIP library (`respond`): selection, prefix-salted digest, probe
and byte-limited compaction for every claim of a receive batch.  Both claim strategies select and hash on the device in
one call each, over the store's live index in HBM: dsy_claim_largest (the pivot ranges of _select_bloomfilter_range /
_select_and_fix) and dsy_claim_modulo (the residue class).
"""
import ctypes
import itertools
import operator
import random as _random_module
import time as _time
from collections import OrderedDict, namedtuple
from math import ceil

import numpy as np

from . import _native
from .bloomfilter import BloomFilter
from .distribution import FullSyncDistribution, GlobalTimePruning, LastSyncDistribution, SyncDistribution

try:  # store_messages' / respond's column reads in C (csrc/dsy_host.c, built beside libdsybloom.so; = the Python path)
    from . import _dsyhost
except ImportError:  # an unbuilt tree
    _dsyhost = None

MAX_GT = 2 ** 63 - 1  # sqlite's signed 64-bit ceiling (community.py:2545-2548)
_REQUEST_DTYPE = np.dtype(_native.Request)  # the dsy_request layout, as a numpy record
_RANGE_DTYPE = np.dtype([("time_low", np.uint64), ("time_high", np.uint64), ("modulo", np.uint64),
                         ("offset", np.uint64)])
_RANGE_OF = operator.itemgetter(0, 1, 2, 3)  # a ClaimRequest's (time_low, time_high, modulo, offset)
_BLOOM_OF = operator.itemgetter(4)
_RECORD_OF = operator.attrgetter("request_record")
_RAW_OF = operator.attrgetter("_raw")
_REFS_OF = operator.attrgetter("_refs")  # a BloomFilter's (record, filter bytes) addresses, 16 B
_DIST_OF = operator.attrgetter("distribution")
_MSG_GT_OF = operator.attrgetter("distribution.global_time")
_PACKET_OF = operator.attrgetter("packet")

# the sync part of an introduction-request payload (payload.py:31-153): time_high == 0 means "up to the
# responder's global time"
ClaimRequest = namedtuple("ClaimRequest", "time_low time_high modulo offset bloom_filter")


class RowLists(object):
    """The responder's answer for a batch of claims: claim i's store rows, in send order, are rows[offsets[i]:
    offsets[i + 1]].  A sequence of per-claim int64 arrays (len, indexing, iteration) built on access, so a caller
    that reads the packed form (rows, offsets) pays for no per-claim objects."""

    __slots__ = ("rows", "offsets")

    def __init__(self, rows, offsets):
        self.rows, self.offsets = rows, offsets

    def __len__(self):
        return len(self.offsets) - 1

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        n = len(self)
        if i < 0:
            i += n
        if not 0 <= i < n:
            raise IndexError(i)
        return self.rows[self.offsets[i]:self.offsets[i + 1]]

    def __iter__(self):
        rows, off = self.rows, self.offsets.tolist()
        return (rows[off[i]:off[i + 1]] for i in range(len(off) - 1))


class DropMessage(object):
    """A received message the checks refuse, with the reference's reason text (message.py DropMessage)."""

    def __init__(self, dropped, reason):
        self.dropped = dropped
        self.reason = reason


class DelayMessageBySequence(object):
    """message.py:147-166: the message waits until its member's sequence numbers missing_low..missing_high arrive."""

    def __init__(self, delayed, missing_low, missing_high):
        assert 0 < missing_low <= missing_high, (missing_low, missing_high)
        self.delayed = delayed
        self.missing_low = missing_low
        self.missing_high = missing_high


def _member_id(message):
    auth = getattr(message, "authentication", None)
    return int(auth.member.database_id) if auth is not None else int(message.member)


def _meta_id(message):
    return message.database_id if hasattr(message, "database_id") else message.meta.database_id


def _signature_length(message, default):
    auth = getattr(message, "authentication", None)
    return int(getattr(auth.member, "signature_length", default)) if auth is not None else default


class SyncCache(object):
    """community.py:57-67."""

    def __init__(self, time_low, time_high, modulo, offset, bloom_filter):
        self.time_low = time_low
        self.time_high = time_high
        self.modulo = modulo
        self.offset = offset
        self.bloom_filter = bloom_filter
        self.times_used = 0
        self.responses_received = 0
        self.candidate = None


class SyncStatistics(object):
    """The four bloom counters of CommunityStatistics (statistics.py:305-308)."""

    def __init__(self):
        self.sync_bloom_new = 0
        self.sync_bloom_reuse = 0
        self.sync_bloom_send = 0
        self.sync_bloom_skip = 0


class SyncCommunity(object):
    """Bloom-filter synchronisation of one community over a SyncStore."""

    # probability steps to get a sync skipped if the previous one was empty (community.py:86-87)
    _SKIP_CURVE_STEPS = [0, 0, 0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9]
    _SKIP_STEPS = len(_SKIP_CURVE_STEPS)

    def __init__(self, store, meta_messages, global_time=0, signature_length=60, rng=None, random_source=None,
                 clock=None):
        """rng: the community's private Random (expovariate pivot, community.py:778-780); random_source: provider of
        the module-level random()/randint() draws (prefix, skip, modulo offset).  Both default to `random`.
        clock: the time() acceptable_global_time's 5-second cache reads (default time.time)."""
        self._store = store
        self._respond_out = None  # _respond_requests' reusable output buffer
        self._meta_messages = OrderedDict((m.name, m) for m in meta_messages)
        self._global_time = global_time
        self._signature_length = signature_length
        self._random = rng if rng is not None else _random_module.Random()
        self._rand = random_source if random_source is not None else _random_module
        self._statistics = SyncStatistics()
        self._sync_cache = None
        self._sync_cache_skip_count = 0
        self._nrsyncpackets = 0
        self.dispersy_acceptable_global_time_range = 10000  # community.py:952-953
        self._clock = clock if clock is not None else _time.time
        self._verified_candidates = []
        self._acceptable_global_time_deadline = 0.0  # community.py:294, :392
        self._acceptable_global_time_cache = global_time
        self.sent_packets = []  # (candidate, packet, reason) the checks answer with (Dispersy._send_packets)
        # community.py:430-431
        self._do_pruning = any(isinstance(m.distribution, SyncDistribution) and
                               isinstance(m.distribution.pruning, GlobalTimePruning) for m in meta_messages)

    # ------------------------------------------------------------------------ plugin hooks (properties)
    @property
    def dispersy_enable_bloom_filter_sync(self):
        return True

    @property
    def dispersy_sync_bloom_filter_error_rate(self):
        return 0.01

    @property
    def dispersy_sync_bloom_filter_bits(self):
        # one MTU: 1500 - IP 60 - UDP 8 - header 51 - signature - payload 21 - sync 30 bytes (community.py:637-666)
        return (1500 - 60 - 8 - 51 - self._signature_length - 21 - 30) * 8

    @property
    def dispersy_sync_bloom_filter_strategy(self):
        return self._dispersy_claim_sync_bloom_filter_largest

    @property
    def dispersy_sync_skip_enable(self):
        return True

    @property
    def dispersy_sync_cache_enable(self):
        return True

    @property
    def dispersy_sync_response_limit(self):
        return 5 * 1024

    # ------------------------------------------------------------------------------------- community state
    @property
    def store(self):
        return self._store

    @property
    def global_time(self):
        return max(1, self._global_time)

    def dispersy_yield_verified_candidates(self):
        """The candidates whose global-time opinion counts (community.py:1036).  The walker that keeps them is out of
        scope, so the caller supplies them with set_verified_candidates (objects with a .global_time)."""
        return iter(self._verified_candidates)

    def set_verified_candidates(self, candidates):
        self._verified_candidates = list(candidates)

    @property
    def acceptable_global_time(self):
        """community.py:1015-1058: the highest global time accepted for incoming messages -- the median of the
        candidates' opinions when there are more than 5 (the lower middle one, a py2 floor index), else our own
        global time, plus dispersy_acceptable_global_time_range, at most 2^63-1; recomputed at most every 5 s."""
        if not self.dispersy_enable_bloom_filter_sync:
            return MAX_GT
        now = self._clock()
        if self._acceptable_global_time_deadline < now:
            options = sorted(g for g in (c.global_time for c in self.dispersy_yield_verified_candidates()) if g > 0)
            median_global_time = options[len(options) // 2] if len(options) > 5 else 0
            self._acceptable_global_time_cache = min(max(self._global_time, median_global_time) +
                                                     self.dispersy_acceptable_global_time_range, MAX_GT)
            self._acceptable_global_time_deadline = now + 5.0
        return self._acceptable_global_time_cache

    def update_global_time(self, global_time):
        """community.py:1082-1096: raise the global time; with GlobalTimePruning metas, DELETE their packets that
        reached the prune threshold (SyncStore.prune -> dsy_store_prune)."""
        if global_time > self._global_time:
            self._global_time = global_time
            if self._do_pruning:
                for meta in self._meta_messages.values():
                    if (isinstance(meta.distribution, SyncDistribution) and
                            isinstance(meta.distribution.pruning, GlobalTimePruning)):
                        self._store.prune(meta.database_id,
                                          self._global_time - meta.distribution.pruning.prune_threshold)

    def get_meta_messages(self):
        return list(self._meta_messages.values())

    def _syncable_meta_ids(self):
        return [m.database_id for m in self._meta_messages.values() if m.syncable]

    def _served_metas(self):
        """Syncable metas, priority DESC, stable (community.py:2790-2794)."""
        return sorted((m for m in self._meta_messages.values() if m.syncable),
                      key=lambda m: m.distribution.priority, reverse=True)

    # ----------------------------------------------------------------------------------- requester side
    def dispersy_store(self, messages):
        """community.py:680-707: packets just stored that fall in the cached claim are added to its filter, and
        responses from the claim's candidate are counted.  All qualifying packets go to the GPU in one launch."""
        cache = self._sync_cache
        if not cache:
            return
        packets = []
        for message in messages:
            gt = message.distribution.global_time
            if (message.distribution.priority > 32 and cache.time_low <= gt <= cache.time_high and
                    (gt + cache.offset) % cache.modulo == 0):
                packets.append(message.packet)
                if (cache.candidate and getattr(message, "candidate", None) and
                        cache.candidate.sock_addr == message.candidate.sock_addr):
                    cache.responses_received += 1
        if packets:
            cache.bloom_filter.add_keys(packets)

    def _check_full_sync_distribution_batch(self, messages):
        """dispersy.py:921-1065: every message, in (global_time, packet) order, either as itself (accept),
        DropMessage(message, reason) or -- sequence-numbered metas only -- DelayMessageBySequence.
        The per-message `_is_duplicate_sync_message` lookups (:831-918) run as ONE hash join on the GPU
        (SyncStore.dup_check); their side effects follow in order: the undo proof of an exact duplicate of an undone
        packet is sent (recorded in self.sent_packets as (candidate, packet, reason)), and a stored packet that
        differs only after the first signature_length bytes and compares lower is replaced (UPDATE, :903).
        A message carries .packet, .distribution.global_time, .candidate, its member's database id
        (.authentication.member.database_id, or .member) and signature length
        (.authentication.member.signature_length, else the community's), and optionally .meta (its pruning; a
        FullSyncDistribution with enable_sequence_number selects the sequence-number branch :954-1037, whose messages
        also carry .distribution.sequence_number and their meta's database id)."""
        messages = sorted(messages, key=lambda m: (m.distribution.global_time, m.packet))
        meta = getattr(messages[0], "meta", None) if messages else None
        if meta is not None and getattr(meta.distribution, "enable_sequence_number", False):
            return self._check_sequence_number_batch(messages)
        acceptable = self.acceptable_global_time
        out, todo, unique = [], [], set()
        for message in messages:
            gt = message.distribution.global_time
            if gt > acceptable:
                out.append(DropMessage(message, "global time is not within acceptable range"))
                continue
            if self._is_pruned(message):
                out.append(DropMessage(message, "message has been pruned"))  # distribution.py:80-81
                continue
            key = (_member_id(message), gt)
            if key in unique:
                out.append(DropMessage(message, "duplicate message by member^global_time (2)"))
                continue
            unique.add(key)
            out.append(message)
            todo.append(len(out) - 1)
        if todo:
            checked = [out[i] for i in todo]
            verdict, rows = self._dup_lookup(checked)
            replaces = []
            for i, message, v, row in zip(todo, checked, verdict.tolist(), rows.tolist()):
                if self._duplicate_side_effects(message, v, row, replaces):
                    out[i] = DropMessage(message, "duplicate message by global_time (2)")
            self._flush_replaces(replaces)
        return out

    def _is_pruned(self, message):
        meta = getattr(message, "meta", None)
        pruning = meta.distribution.pruning if meta is not None else None
        return isinstance(pruning, GlobalTimePruning) and not (self.global_time - message.distribution.global_time <
                                                               pruning.inactive_threshold)

    def _dup_lookup(self, messages):
        return self._store.dup_check([_member_id(m) for m in messages],
                                     [m.distribution.global_time for m in messages], [m.packet for m in messages],
                                     [_signature_length(m, self._signature_length) for m in messages])

    def _duplicate_side_effects(self, message, verdict, row, replaces):
        """_is_duplicate_sync_message (dispersy.py:868-918) given the GPU lookup's verdict: True when a row with the
        message's (member, global_time) exists; sends the undo proof / records the UPDATE like the reference."""
        if verdict == _native.DSY_DUP_NEW:
            return False
        if verdict == _native.DSY_DUP_EXACT:
            undone = int(self._store.undone[row])
            if undone:
                try:
                    proof = self._store.packet(self._store.row_of_id(undone))
                except KeyError:
                    proof = None
                if proof is not None:
                    self.sent_packets.append((message.candidate, proof, "-caused by duplicate-undo-"))
        elif verdict == _native.DSY_DUP_REPLACE:
            # the host copy changes now (a later proof send in this batch reads it), HBM once the batch is done
            self._store.replace_packet([row], [message.packet], device=False)
            replaces.append((row, message.packet))
        return True

    def _flush_replaces(self, replaces):
        if replaces:
            self._store.replace_packet([r for r, _ in replaces], [p for _, p in replaces])

    # ---------------------------------------------------------------------------------------- undo / redo
    def on_undo(self, entries):
        """The UPDATE of Community.on_undo (community.py:3457-3481) for a batch of undo messages: entries are
        (undo packet id, member, global_time) -- for an undo message its own packet id and the payload's member and
        global time; for a DispersyDuplicatedUndo the lower undo's packet id and the higher one's member and global
        time -- as `UPDATE sync SET undone = ? WHERE community = ? AND member = ? AND global_time = ?`, executed in
        order.  The undone packets leave the responder's index; their rows stay for the duplicate check's undo proof.
        (The meta's undo_callback is the application's.)  Returns the number of rows whose undone-ness changed."""
        entries = list(entries)
        if not entries:
            return 0
        rows = self._store.rows_of_keys([e[1] for e in entries], [e[2] for e in entries])
        hit = rows >= 0
        return self._store.set_undone(rows[hit], np.asarray([e[0] for e in entries], dtype=np.int64)[hit])

    def update_undone(self, packet_ids, undone):
        """_update_timerange's UPDATEs (community.py:3633-3642): `UPDATE sync SET undone = 1 WHERE id = ?` for the
        messages the timeline no longer allows (undone=1) and `... undone = 0 WHERE id = ?` for the ones it allows
        again (undone=0).  Which messages those are is the timeline's decision (permissions, out of this path).
        Returns the number of rows whose undone-ness changed."""
        rows = []
        for pid in packet_ids:
            try:
                rows.append(self._store.row_of_id(int(pid)))
            except KeyError:
                pass
        return self._store.set_undone(np.asarray(rows, dtype=np.int64), int(undone))

    def _highest(self, meta_id, member):
        """SELECT MAX(global_time), MAX(sequence), COUNT(*) FROM sync WHERE member = ? AND meta_message = ?
        (dispersy.py:959-961, :1010-1012) -> (last_global_time or 0, last_sequence or 0)."""
        rows = self._store.member_rows(meta_id, member)
        if not len(rows):
            return 0, 0
        return int(self._store.global_time[rows].max()), int(self._store.sequence[rows].max())

    def _check_sequence_number_batch(self, messages):
        """dispersy.py:954-1037, messages already in (global_time, packet) order.  The (member, global_time) lookups
        of every message run up front as one GPU hash join; a row that a DELETE of this batch removed before the
        message's turn counts as absent (nothing is INSERTed during the check, so this is exactly the sequential
        lookup).  The reference's generator ends -- silently, the rest of the batch is neither yielded nor dropped --
        when its `LIMIT 1 OFFSET ?` query finds no row (py2: the StopIteration of `.next()` inside the generator,
        :986-987): that happens when an earlier message of the batch raised the member's in-memory highest sequence
        number past the stored rows; the same cut-off is kept here."""
        st = self._store
        meta_id = _meta_id(messages[0])
        acceptable = self.acceptable_global_time
        highest = {}
        for message in messages:
            member = _member_id(message)
            if member not in highest:
                highest[member] = self._highest(meta_id, member)
        verdict, found = self._dup_lookup(messages)
        out, unique, replaces = [], set(), []
        for message, v, row in zip(messages, verdict.tolist(), found.tolist()):
            gt, seq_no = message.distribution.global_time, message.distribution.sequence_number
            member = _member_id(message)
            if gt > acceptable:
                out.append(DropMessage(message, "global time is not within acceptable range (%d, we accept %d)"
                                       % (gt, acceptable)))
                continue
            if self._is_pruned(message):
                out.append(DropMessage(message, "message has been pruned"))
                continue
            key = (member, gt)
            if key in unique:
                out.append(DropMessage(message, "duplicate message by member^global_time (1)"))
                continue
            unique.add(key)
            last_global_time, seq = highest[member]
            if seq >= seq_no:
                rows = st.member_rows(meta_id, member)
                if seq_no - 1 >= len(rows):
                    break  # the OFFSET query's StopIteration ends the reference's generator (see above)
                have = int(rows[seq_no - 1])
                have_gt, have_packet = int(st.global_time[have]), st.packet(have)
                if message.packet == have_packet:
                    out.append(DropMessage(message, "duplicate message by binary packet"))
                    continue
                if (have_gt, have_packet) < (gt, message.packet):
                    # keep ours and send it back (:996-1002)
                    self.sent_packets.append((message.candidate, have_packet, "-caused by check_full_sync-"))
                    out.append(DropMessage(message, "duplicate message by sequence number (1)"))
                    continue
                # DELETE FROM sync WHERE member = ? AND meta_message = ? AND global_time >= ? (:1006-1007), then the
                # highest cache is refreshed (:1010-1012 also rebind last_global_time; the local `seq` keeps its
                # value, as in the reference)
                st.delete_rows(rows[st.global_time[rows] >= np.uint64(have_gt)])
                highest[member] = self._highest(meta_id, member)
                last_global_time = highest[member][0]
            elif seq + 1 != seq_no:
                out.append(DelayMessageBySequence(message, seq + 1, seq_no - 1))
                continue
            if row >= 0 and st.deleted[row]:
                v = _native.DSY_DUP_NEW  # deleted earlier in this batch: the SELECT finds nothing
            if self._duplicate_side_effects(message, v, row, replaces):
                out.append(DropMessage(message, "duplicate message by global_time (1)"))
                continue
            if last_global_time and gt <= last_global_time:
                out.append(DropMessage(message, "higher sequence number with lower global time than most recent "
                                                "message"))
                continue
            highest[member] = (gt, seq + 1)
            out.append(message)
        self._flush_replaces(replaces)
        return out

    def store_messages(self, messages):
        """Dispersy._store (dispersy.py:1475-1612) for the sync table: INSERT the messages' packets (one batched
        SyncStore.append -> dsy_store_append into HBM; sequence-numbered FullSync messages store their sequence
        number, :1529-1531), DELETE what LastSyncDistribution no longer keeps -- each member's rows beyond the newest
        history_size, or the items its custom_callback names (:1558-1591; one dsy_store_delete) --, raise the
        community's global time to the highest stored one, then dispersy_store(messages) updates the cached claim
        filter.  A message carries .packet, .distribution.global_time and its meta's database id (.database_id, or
        .meta.database_id); .meta.distribution selects the sequence/history handling.  As in the reference, the
        caller has already dropped duplicates (dispersy.py:1496-1498).  Messages of a double-member-signed meta
        (meta.double_signed; .authentication.members, .member = members[0]) also record their member pair
        (double_signed_sync, :1537-1541), and their LastSync history is kept per pair.  Returns the new store rows."""
        if not messages:
            return np.zeros(0, dtype=np.int64)
        # column by column (C-level getters over the list, no Python frame per message); what a meta needs (history,
        # sequence numbers, its checks) is worked out once per meta object, and everything is checked before anything
        # is stored, so a refused batch changes neither copy
        n = len(messages)
        has_member = self._store.member is not None
        cols = None
        if _dsyhost is not None and type(messages) is list:
            # one C pass (dsy_host.c): global times, packets, their gather list, whether one meta object serves all
            gts, lens, addrs = (np.empty(n, dtype=np.uint64) for _ in range(3))
            packets, one_meta, first, all_bytes = _dsyhost.message_columns(messages, gts, lens, addrs)
            meta_objs = [first] * n if one_meta else list(map(getattr, messages, itertools.repeat("meta", n),
                                                                     itertools.repeat(None, n)))
            cols = (lens, addrs) if all_bytes else None
        else:
            meta_objs = list(map(getattr, messages, itertools.repeat("meta", n), itertools.repeat(None, n)))
            first = meta_objs[0]
            # one meta object for the whole batch (the usual case): an identity scan instead of a dict over 10 k ids
            one_meta = all(map(operator.is_, meta_objs, itertools.repeat(first, n)))
            gts = np.fromiter(map(_MSG_GT_OF, messages), dtype=np.uint64, count=n)
            packets = list(map(_PACKET_OF, messages))
        uniq = [first] if one_meta else dict(zip(map(id, meta_objs), meta_objs)).values()
        per_meta = {}
        for meta in uniq:
            per_meta[id(meta)] = self._meta_store_info(meta)
        meta_id = getattr(first, "database_id", None) if one_meta else None
        if meta_id is not None:
            # a message's database_id is its meta's (message.py:265-266): one value for the batch
            metas = np.full(n, meta_id, dtype=np.uint32)
        else:
            try:
                metas = np.fromiter(map(getattr, messages, itertools.repeat("database_id", n),
                                        itertools.repeat(None, n)), dtype=np.uint32, count=n)
            except TypeError:  # messages that carry their meta's id on .meta only
                metas = [getattr(m, "database_id", None) for m in messages]
                metas = np.array([d if d is not None else meta.database_id for d, meta in zip(metas, meta_objs)],
                                 dtype=np.uint32)
        seqs = None
        if any(info[0] for info in per_meta.values()):
            seqs = [d.sequence_number if per_meta[id(meta)][0] else 0
                    for d, meta in zip(map(_DIST_OF, messages), meta_objs)]
        members = list(map(_member_id, messages)) if has_member else None
        double = ([i for i, meta in enumerate(meta_objs) if per_meta[id(meta)][2]]
                  if any(info[2] for info in per_meta.values()) else [])
        # members[0] and members[1] (dispersy.py:1537-1538)
        pairs = [(int(ms[0].database_id), int(ms[1].database_id))
                 for ms in (messages[i].authentication.members for i in double)]
        rows = self._store.append(packets, gts, metas, member=members, sequence=seqs, _gather=cols)
        if double:  # INSERT INTO double_signed_sync (dispersy.py:1537-1541)
            p = np.asarray(pairs, dtype=np.int64).reshape(-1, 2)
            self._store.set_pairs(rows[double], p[:, 0], p[:, 1])
        if any(info[1] for info in per_meta.values()):
            self._last_sync_history(messages)
        self.update_global_time(int(gts.max()))
        self.dispersy_store(messages)
        return rows

    def _meta_store_info(self, meta):
        """(sequence, history, double): whether messages of `meta` store a sequence number (a sequence-numbered
        FullSyncDistribution, dispersy.py:1529-1531), keep a LastSyncDistribution history, and are double-member
        signed (their member pair goes to double_signed_sync, :1537-1541; the history is then kept per pair,
        :1567-1578).  Raises for per-member history or sequence numbers in a store without its member column."""
        dist = getattr(meta, "distribution", None)
        history = isinstance(dist, LastSyncDistribution)
        seq = isinstance(dist, FullSyncDistribution) and bool(dist.enable_sequence_number)
        double = bool(getattr(meta, "double_signed", False))
        if self._store.member is None and (history or seq or double):
            raise ValueError("store_messages: meta %s keeps per-member history; the store needs its member column"
                             % getattr(meta, "name", "?"))
        if history and double and not dist.custom_callback and not self._store.pairs_exported(meta.database_id):
            # the per-pair history (:1567-1578) joins double_signed_sync: rows stored without it would be missed
            raise ValueError("store_messages: meta %s keeps its history per member pair, but the store's rows of it "
                             "were exported without their double_signed_sync table (SyncStore.from_rows / attach: "
                             "pass pairs=)" % getattr(meta, "name", "?"))
        return seq, history, double

    def _last_sync_history(self, messages):
        st = self._store
        by_meta = OrderedDict()
        for m in messages:
            meta = getattr(m, "meta", None)
            if meta is not None and isinstance(meta.distribution, LastSyncDistribution):
                by_meta.setdefault(id(meta), (meta, []))[1].append(m)
        drop = []
        for meta, msgs in by_meta.values():
            dist = meta.distribution
            if dist.custom_callback:
                for syncid, _ in dist.custom_callback[1](msgs):
                    try:
                        drop.append(st.row_of_id(syncid))
                    except KeyError:
                        pass
                continue
            if getattr(meta, "double_signed", False):  # per member pair, through double_signed_sync (:1567-1578)
                for pair in OrderedDict.fromkeys(
                        tuple(sorted((int(m.authentication.members[0].database_id),
                                      int(m.authentication.members[1].database_id)))) for m in msgs):
                    rows = st.pair_rows(meta.database_id, *pair)
                    if len(rows) > dist.history_size:
                        drop.extend(rows[:len(rows) - dist.history_size].tolist())
                continue
            for member in OrderedDict.fromkeys(_member_id(m) for m in msgs):
                rows = st.member_rows(meta.database_id, member)
                if len(rows) > dist.history_size:
                    drop.extend(rows[:len(rows) - dist.history_size].tolist())
        if drop:
            st.delete_rows(drop)

    def dispersy_claim_sync_bloom_filter(self, request_cache):
        """community.py:709-758.  Returns (time_low, time_high, modulo, offset, bloom_filter) or None."""
        if self._sync_cache:
            if self._sync_cache.responses_received > 0:
                if self.dispersy_sync_skip_enable:
                    self._sync_cache_skip_count = 0
                if self.dispersy_sync_cache_enable and self._sync_cache.times_used < 100:
                    self._statistics.sync_bloom_reuse += 1
                    self._statistics.sync_bloom_send += 1
                    cache = self._sync_cache
                    cache.times_used += 1
                    cache.responses_received = 0
                    cache.candidate = getattr(request_cache, "helper_candidate", None)
                    return cache.time_low, cache.time_high, cache.modulo, cache.offset, cache.bloom_filter
            elif self._sync_cache.times_used == 0:
                self._sync_cache_skip_count = min(self._sync_cache_skip_count + 1, self._SKIP_STEPS)

        if (self.dispersy_sync_skip_enable and self._sync_cache_skip_count and
                self._rand.random() < self._SKIP_CURVE_STEPS[self._sync_cache_skip_count - 1]):
            self._statistics.sync_bloom_skip += 1
            self._sync_cache = None
            return None

        sync = self.dispersy_sync_bloom_filter_strategy(request_cache)
        if sync:
            self._sync_cache = SyncCache(*sync)
            self._sync_cache.candidate = getattr(request_cache, "helper_candidate", None)
            self._statistics.sync_bloom_new += 1
            self._statistics.sync_bloom_send += 1
        return sync

    def _new_claim_filter(self):
        return BloomFilter(self.dispersy_sync_bloom_filter_bits, self.dispersy_sync_bloom_filter_error_rate,
                           prefix=bytes([int(self._rand.random() * 256)]))

    def _empty_claim(self, acceptable):
        return (1, acceptable, 1, 0, BloomFilter(8, 0.1, prefix=b"\x00"))

    def _dispersy_claim_sync_bloom_filter_largest(self, request_cache):
        """community.py:763-837: a filter over <= capacity packets around an exponentially distributed pivot."""
        syncable = self._syncable_meta_ids()
        acceptable_global_time = self.acceptable_global_time
        if not syncable:
            return self._empty_claim(acceptable_global_time)
        bloom = self._new_claim_filter()
        capacity = bloom.get_capacity(self.dispersy_sync_bloom_filter_error_rate)
        desired_mean = self.global_time / 2.0
        from_gbtime = self.global_time - int(self._random.expovariate(1.0 / desired_mean))
        if from_gbtime < 1:
            from_gbtime = int(self._random.random() * self.global_time)

        # the range selection (_select_bloomfilter_range / _select_and_fix, :783-815) and add_keys (:821) run on the
        # device over the store's live index, in one call
        time_low, time_high, added, self._nrsyncpackets = bloom.claim_largest(
            self._store, syncable, from_gbtime, capacity, self._nrsyncpackets, acceptable_global_time)
        if added:
            return (time_low, time_high, 1, 0, bloom)
        return self._empty_claim(acceptable_global_time)

    def _select_bloomfilter_range(self, request_cache, syncable, global_time, to_select, higher=True):
        """community.py:839-879 over the host index columns (the strategy itself uses the device form,
        dsy_claim_largest; this mirror keeps the reference's method for callers and tests)."""
        data, fixed = self._select_and_fix(request_cache, syncable, global_time, to_select, higher)
        lowerfixed = higherfixed = True
        if len(data) < to_select:
            to_select = to_select - len(data)
            if to_select > 25:
                if higher:
                    lowerdata, lowerfixed = self._select_and_fix(request_cache, syncable, global_time + 1, to_select, False)
                    data = lowerdata + data
                else:
                    higherdata, higherfixed = self._select_and_fix(request_cache, syncable, global_time - 1, to_select, True)
                    data = data + higherdata

        bloomfilter_range = [data[0][0], data[-1][0], len(data)]
        if higher:
            bloomfilter_range[0] = min(bloomfilter_range[0], global_time + 1)
            if not fixed:
                bloomfilter_range[1] = self.acceptable_global_time
            if not lowerfixed:
                bloomfilter_range[0] = 1
        else:
            bloomfilter_range[1] = max(bloomfilter_range[1], global_time - 1)
            if not fixed:
                bloomfilter_range[0] = 1
            if not higherfixed:
                bloomfilter_range[1] = self.acceptable_global_time
        return bloomfilter_range, data

    def _select_and_fix(self, request_cache, syncable, global_time, to_select, higher=True):
        """community.py:881-903 over the store's index: up to to_select+1 live packets strictly above (below) the
        pivot in global-time order; when over-full, the trailing global-time group is dropped.  Returns
        ([(global_time, store_row)], fixed)."""
        st, limit = self._store, to_select + 1
        gts, rows = [], []
        for meta_id in syncable:
            seg = st.live_rows(meta_id)
            g = st.global_time[seg]
            if higher:
                i = int(np.searchsorted(g, global_time, side="right"))
                part = seg[i:i + limit]
            else:
                i = int(np.searchsorted(g, max(global_time, 0), side="left")) if global_time > 0 else 0
                part = seg[max(0, i - limit):i][::-1]
            rows.append(part)
            gts.append(st.global_time[part])
        rows = np.concatenate(rows) if rows else np.zeros(0, dtype=np.int64)
        gts = np.concatenate(gts) if gts else np.zeros(0, dtype=np.uint64)
        order = np.argsort(gts, kind="stable")
        if not higher:
            order = order[::-1]
        rows, gts = rows[order][:limit], gts[order][:limit]
        data = [(int(g), int(r)) for g, r in zip(gts, rows)]
        fixed = False
        if len(data) > to_select:
            fixed = True
            cut = data[-1][0]
            del data[-1]
            while data and data[-1][0] == cut:
                del data[-1]
        if not higher:
            data.reverse()
        return data, fixed

    def _dispersy_claim_sync_bloom_filter_modulo(self, request_cache):
        """community.py:908-933: a filter over the residue class (global_time + offset) % modulo == 0."""
        syncable = self._syncable_meta_ids()
        if not syncable:
            return self._empty_claim(self.acceptable_global_time)
        bloom = self._new_claim_filter()
        capacity = bloom.get_capacity(self.dispersy_sync_bloom_filter_error_rate)
        st = self._store
        self._nrsyncpackets = st.count_live(syncable)
        modulo = int(ceil(self._nrsyncpackets / float(capacity)))
        if modulo > 1:
            offset = self._rand.randint(0, modulo - 1)
        else:
            offset, modulo = 0, 1
        # the SELECTs (:918, :922) and add_keys (:924) run on the device over the store's live index
        bloom.add_store_modulo(st, syncable, offset, modulo)
        return (1, self.acceptable_global_time, modulo, offset, bloom)

    # ----------------------------------------------------------------------------------- responder side
    def _meta_time_low(self, meta, time_low, include_inactive):
        # community.py:2800-2808
        if include_inactive or not isinstance(meta.distribution.pruning, GlobalTimePruning):
            return time_low
        return min(max(time_low, self.global_time - meta.distribution.pruning.inactive_threshold + 1), MAX_GT)

    def _select_rows(self, time_low, time_high, offset, modulo, include_inactive, shuffle):
        """Store rows one request selects, in send order (the UNION ALL query of community.py:2764-2797)."""
        st = self._store
        out = []
        for meta in self._served_metas():
            seg = st.live_rows(meta.database_id)
            g = st.global_time[seg]
            lo = self._meta_time_low(meta, time_low, include_inactive)
            a = int(np.searchsorted(g, lo, side="left")) if lo <= MAX_GT else len(seg)
            b = int(np.searchsorted(g, time_high, side="right"))
            part = seg[a:b] if a < b else seg[:0]
            if modulo > 1 and len(part):
                part = part[(st.global_time[part] + np.uint64(offset)) % np.uint64(modulo) == 0]
            direction = meta.distribution.synchronization_direction
            if direction == "DESC":
                part = part[::-1]
            elif direction == "RANDOM":
                part = shuffle(part)
            out.append(part)
        return np.concatenate(out) if out else np.zeros(0, dtype=np.int64)

    def _get_packets_for_bloomfilters(self, requests, include_inactive=True):
        """community.py:2746-2811: yields (message, generator of (packet,)) per request
        (message, time_low, time_high, offset, modulo), in the reference's send order."""
        assert isinstance(requests, list)
        assert all(len(request) == 5 for request in requests)
        perm = lambda rows: rows[np.random.Generator(np.random.PCG64(self._random.getrandbits(64))).permutation(len(rows))]  # noqa: E731
        for message, time_low, time_high, offset, modulo in requests:
            rows = self._select_rows(time_low, time_high, offset, modulo, include_inactive, perm)
            yield message, ((self._store.packet(int(r)),) for r in rows)

    def respond(self, requests, include_inactive=False, byte_limit=None, random_seed=None):
        """Batched responder (community.py:2531-2572): for each ClaimRequest (time_high already resolved), the store
        rows the reference would send, in send order.  One call into the HIP library for the whole batch
        (dsy_sync_respond_refs): per claim its four range fields and its BloomFilter's two addresses -- the library
        reads the filter's shape and bytes where the BloomFilter keeps them."""
        R = len(requests)
        if not R:
            return self._respond_requests(np.zeros(1, dtype=_REQUEST_DTYPE), 0, b"", include_inactive, byte_limit,
                                          random_seed)
        ranges, refs = self._claim_columns(requests)
        return self._respond_requests(None, R, None, include_inactive, byte_limit, random_seed, (ranges, refs))

    @staticmethod
    def _claim_columns(requests):
        """respond()'s per-claim columns: the four range fields (uint64 x 4R) and the BloomFilters' (record, filter)
        address pairs (16 B each)."""
        R = len(requests)
        if _dsyhost is not None and type(requests) in (list, tuple):
            # one C pass (dsy_host.c claim_columns): the ranges (time bounds past 2^64 stored as 2^63-1) and addresses
            ranges, ref_words = np.empty(4 * R, dtype=np.uint64), np.empty(2 * R, dtype=np.uint64)
            _dsyhost.claim_columns(requests, ranges, ref_words)
            refs = ref_words.tobytes()
        else:
            try:
                ranges = np.fromiter(itertools.chain.from_iterable(map(_RANGE_OF, requests)), dtype=np.uint64,
                                     count=4 * R)
            except OverflowError:  # a bound past 2^64: clamp in Python first (the library clamps to 2^63-1)
                ranges = np.fromiter(itertools.chain.from_iterable((min(q.time_low, MAX_GT), min(q.time_high, MAX_GT),
                                                                    q.modulo, q.offset) for q in requests),
                                     dtype=np.uint64, count=4 * R)
            refs = b"".join(map(_REFS_OF, map(_BLOOM_OF, requests)))
        return ranges, refs

    @staticmethod
    def _request_table(requests):
        """(dsy_request records with filter_offset unset, R, the claims' BloomFilters): the filters' static record
        parts (BloomFilter.request_record) joined into the record array in one pass, the claims' (time_low, time_high,
        modulo, offset) filled as columns, time bounds clamped to 2^63-1 (community.py:2545-2548)."""
        R = len(requests)
        if not R:
            return np.zeros(1, dtype=_REQUEST_DTYPE), 0, []
        bfs = list(map(_BLOOM_OF, requests))
        reqs = np.frombuffer(bytearray(b"".join(map(_RECORD_OF, bfs))), dtype=_REQUEST_DTYPE)
        try:  # a flat uint64 fromiter: the structured-dtype one builds a tuple per claim
            t = np.fromiter(itertools.chain.from_iterable(map(_RANGE_OF, requests)), dtype=np.uint64,
                            count=4 * R).view(_RANGE_DTYPE)
        except OverflowError:  # a bound past 2^64: clamp in Python first
            t = np.fromiter(((min(q.time_low, MAX_GT), min(q.time_high, MAX_GT), q.modulo, q.offset) for q in requests),
                            dtype=_RANGE_DTYPE, count=R)
        reqs["time_low"] = np.minimum(t["time_low"], np.uint64(MAX_GT))
        reqs["time_high"] = np.minimum(t["time_high"], np.uint64(MAX_GT))
        reqs["modulo"] = t["modulo"]
        reqs["offset"] = t["offset"]
        return reqs, R, bfs

    @staticmethod
    def request_records(requests):
        """(dsy_request records, R, packed filters) of a list of ClaimRequests, as dsy_sync_respond takes them
        (_request_table's records); each filter sits 4-byte aligned in the blob at its record's filter_offset."""
        reqs, R, bfs = SyncCommunity._request_table(requests)
        if not R:
            return reqs, 0, b""
        raws = list(map(_RAW_OF, bfs))
        if len(set(map(len, raws))) == 1:
            # one filter size (the MTU claim): the padding is the join's separator (an empty last item adds the
            # last filter's)
            first = len(raws[0])
            step = (first + 3) & ~3
            reqs["filter_offset"] = np.arange(R, dtype=np.uint64) * np.uint64(step)
            raws.append(b"")
            blob = (b"\x00" * (step - first)).join(raws)
        else:
            sizes = np.fromiter(((len(r) + 3) & ~3 for r in raws), dtype=np.uint64, count=R)
            reqs["filter_offset"] = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
            blob = b"".join(bytes(r) + b"\x00" * ((-len(r)) % 4) for r in raws)
        return reqs, R, blob

    def meta_records(self):
        """The served metas as dsy_meta records, in serving order (priority DESC, community.py:2790-2794)."""
        metas = self._served_metas()
        mt = (_native.Meta * max(len(metas), 1))()
        for j, m in enumerate(metas):
            mt[j].meta_id = m.database_id
            mt[j].direction = _native.DIRECTIONS[m.distribution.synchronization_direction]
            pr = m.distribution.pruning
            mt[j].has_pruning = 1 if isinstance(pr, GlobalTimePruning) else 0
            mt[j].inactive_threshold = pr.inactive_threshold if isinstance(pr, GlobalTimePruning) else 0
        return mt, len(metas)

    def respond_wire(self, blocks, include_inactive=False, byte_limit=None, random_seed=None):
        """on_introduction_request's sync half for a receive batch of raw sync blocks: decode (conversion.py:732-799,
        time_high 0 resolved to this community's global time, community.py:2545-2553) and answer every good claim
        in one responder call.  Returns, per block, a DropPacket (the decoder's verdict) or the store rows to send.
        A block whose filter the BloomFilter constructor rejects raises AssertionError for the whole batch, as the
        reference's decode loop does."""
        from .conversion import DECODE_ASSERT, DROP_REASONS, DropPacket, decode_sync_blocks, raise_for_status
        batch = decode_sync_blocks(blocks, responder_global_time=self.global_time)
        asserting = np.flatnonzero(batch.status == DECODE_ASSERT)
        if len(asserting):
            # the reference's decode loop dies on this block's AssertionError (community.py:2078-2090 catches only
            # DropPacket/DelayPacket): no claim of the batch is answered
            raise_for_status(DECODE_ASSERT, int(asserting[0]))
        good = np.flatnonzero(batch.status == 0)
        sub = np.zeros(max(len(good), 1), dtype=_REQUEST_DTYPE)
        if len(good):
            sub[:len(good)] = np.ctypeslib.as_array(batch.requests)[good]
        rows = self._respond_requests(sub, len(good), batch.filters, include_inactive, byte_limit, random_seed)
        out = [DropPacket(DROP_REASONS.get(int(st), "Invalid sync block")) for st in batch.status]
        for i, r in zip(good, rows):
            out[int(i)] = r
        return out

    def _respond_requests(self, reqs, R, blob, include_inactive, byte_limit, random_seed, refs=None):
        """One dsy_sync_respond call for R dsy_request records whose filters sit in `blob` -- or, with `refs` (the
        claims' ranges and (record, filter) addresses, SyncCommunity.respond), one dsy_sync_respond_refs call."""
        byte_limit = self.dispersy_sync_response_limit if byte_limit is None else byte_limit
        seed = self._random.getrandbits(64) if random_seed is None else random_seed
        st = self._store
        ctx = st.ctx
        mt, n_metas = self.meta_records()
        out_off = np.zeros(R + 1, dtype=np.uint64)
        # one output buffer per community, grown on demand and reused by every call (the answer is copied out of it:
        # RowLists handed to callers never alias the next call's output)
        out = self._respond_out
        if out is None:
            out = self._respond_out = np.empty(1 << 16, dtype=np.uint64)
        while True:
            cap = len(out)
            if refs is None:
                rc = ctx.lib.dsy_sync_respond(ctx.handle, st.handle,
                                              reqs.ctypes.data_as(ctypes.POINTER(_native.Request)), R, blob, len(blob),
                                              mt, n_metas, self.global_time, 1 if include_inactive else 0,
                                              int(byte_limit), seed, out.ctypes.data, cap, out_off.ctypes.data)
            else:
                rc = ctx.lib.dsy_sync_respond_refs(ctx.handle, st.handle, refs[0].ctypes.data, refs[1], R, mt, n_metas,
                                                   self.global_time, 1 if include_inactive else 0, int(byte_limit),
                                                   seed, out.ctypes.data, cap, out_off.ctypes.data)
            if rc == _native.DSY_ECAPACITY and int(out_off[R]) > cap:
                out = self._respond_out = np.empty(int(out_off[R]), dtype=np.uint64)
                continue
            _native.check(rc)
            break
        return RowLists(out[:int(out_off[R])].view(np.int64).copy(), out_off.view(np.int64))

    def on_introduction_request_sync(self, messages, include_inactive=False):
        """The sync half of on_introduction_request (community.py:2531-2572) for a receive batch.

        messages: list of (message, ClaimRequest).  Returns [(message, [packet bytes])] for the messages that get a
        non-empty response, in input order."""
        reqs = []
        for _, q in messages:
            time_high = q.time_high if q.time_high else self.global_time
            reqs.append(q._replace(time_low=min(q.time_low, MAX_GT), time_high=min(time_high, MAX_GT)))
        rows = self.respond(reqs, include_inactive=include_inactive)
        out = []
        for (message, _), rs in zip(messages, rows):
            if len(rs):
                out.append((message, self._store.packets(rs)))
        return out

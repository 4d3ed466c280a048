"""ORACLE -- test infrastructure only.

CPU restatement of the sync-selection half of the hot path, over an sqlite3 `sync` table with the reference's
columns (dispersydatabase.py:53-64).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import it.  Pinned against tests/golden/sync_vectors.json (outputs of the reference's own methods, lifted from
community.py by tests/golden/gen_sync_golden.py).

Restated functions (reference file:line):
  respond_lists        community.py:2746-2811 (_get_packets_for_bloomfilters) + :2555-2567 (byte-limited loop)
  select_and_fix       community.py:881-903
  select_range         community.py:839-879
  claim_largest        community.py:763-837
  claim_modulo         community.py:908-933
  insert_packets       dispersy.py:1523-1533 (Dispersy._store's INSERT INTO sync, one execute per message)
  check_full_sync_batch  dispersy.py:921-1065 (no sequence numbers) + is_duplicate_sync_message :831-918
  check_sequence_batch   dispersy.py:954-1037 (the sequence-number branch)
  store_last_sync        dispersy.py:1475-1612 (_store's INSERT + LastSyncDistribution history DELETE :1558-1591)
  SYNC_SCHEMA          dispersydatabase.py:53-64 (the sync table and its (meta_message, undone, global_time) index)
"""
import math

MAX_GT = 2 ** 63 - 1

SYNC_SCHEMA = """
CREATE TABLE sync(id INTEGER PRIMARY KEY AUTOINCREMENT, community INTEGER, member INTEGER, global_time INTEGER,
                  meta_message INTEGER, undone INTEGER DEFAULT 0, packet BLOB, sequence INTEGER,
                  UNIQUE(community, member, global_time));
CREATE INDEX sync_mug ON sync(meta_message, undone, global_time);
CREATE TABLE double_signed_sync(sync INTEGER REFERENCES sync(id), member1 INTEGER, member2 INTEGER);
CREATE INDEX double_signed_sync_index_0 ON double_signed_sync(member1, member2);
"""


def is_duplicate_sync_message(conn, community, message, sends):
    """dispersy.py:831-918 (_is_duplicate_sync_message).  message: dict(member, gt, packet, signature_length, index).
    Side effects as the reference: the undo proof is 'sent' (appended to sends as (index, packet)) and the stored
    packet is replaced by UPDATE when only the signature differs and ours is smaller."""
    row = conn.execute("SELECT packet, undone FROM sync WHERE community = ? AND member = ? AND global_time = ?",
                       (community, message["member"], message["gt"])).fetchone()
    if row is None:
        return False
    have, undone = bytes(row[0]), row[1]
    packet = message["packet"]
    if have == packet:
        if undone:
            proof = conn.execute("SELECT packet FROM sync WHERE id = ?", (undone,)).fetchone()
            if proof is not None:
                sends.append((message["index"], bytes(proof[0])))
    else:
        sl = message["signature_length"]
        if have[:sl] == packet[:sl]:
            if have < packet:
                conn.execute("UPDATE sync SET packet = ? WHERE community = ? AND member = ? AND global_time = ?",
                             (packet, community, message["member"], message["gt"]))
    return True


def check_full_sync_batch(conn, community, messages, acceptable_global_time, global_time):
    """dispersy.py:921-1065 (_check_full_sync_distribution_batch), the branch without sequence numbers (:1043-1063).
    messages: dicts (member, gt, packet, signature_length, inactive or None, index).  Returns ([(index, reason or
    None)] in the order the reference yields them -- sorted by (global_time, packet) --, sends)."""
    out, sends, unique = [], [], set()
    for message in sorted(messages, key=lambda m: (m["gt"], m["packet"])):
        if message["gt"] > acceptable_global_time:
            out.append((message["index"], "global time is not within acceptable range"))
            continue
        inactive = message.get("inactive")
        if inactive is not None and not (global_time - message["gt"] < inactive):  # distribution.py:80-81
            out.append((message["index"], "message has been pruned"))
            continue
        key = (message["member"], message["gt"])
        if key in unique:
            out.append((message["index"], "duplicate message by member^global_time (2)"))
            continue
        unique.add(key)
        if is_duplicate_sync_message(conn, community, message, sends):
            out.append((message["index"], "duplicate message by global_time (2)"))
            continue
        out.append((message["index"], None))
    return out, sends


def check_sequence_batch(conn, community, meta_id, messages, acceptable_global_time, global_time):
    """dispersy.py:954-1037.  messages: dicts (member, gt, seq, packet, signature_length, inactive or None, index).
    Returns (results, sends, ended_early): results [(index, reason | None | ("delay", low, high))] in the reference's
    order; ended_early when the LIMIT 1 OFFSET query finds no row -- the py2 StopIteration that silently ends the
    reference's generator (:986-987)."""
    def highest_of(member):
        g, s_, c = conn.execute("SELECT MAX(global_time), MAX(sequence), COUNT(*) FROM sync WHERE member = ? AND "
                                "meta_message = ?", (member, meta_id)).fetchone()
        return (g or 0, s_ or 0)

    messages = sorted(messages, key=lambda m: (m["gt"], m["packet"]))
    highest = {}
    for m in messages:
        if m["member"] not in highest:
            highest[m["member"]] = highest_of(m["member"])
    out, sends, unique = [], [], set()
    for m in messages:
        if m["gt"] > acceptable_global_time:
            out.append((m["index"], "global time is not within acceptable range (%d, we accept %d)"
                        % (m["gt"], acceptable_global_time)))
            continue
        if m.get("inactive") is not None and not (global_time - m["gt"] < m["inactive"]):
            out.append((m["index"], "message has been pruned"))
            continue
        key = (m["member"], m["gt"])
        if key in unique:
            out.append((m["index"], "duplicate message by member^global_time (1)"))
            continue
        unique.add(key)
        last_gt, seq = highest[m["member"]]
        if seq >= m["seq"]:
            row = conn.execute("SELECT global_time, packet FROM sync WHERE member = ? AND meta_message = ? "
                               "ORDER BY global_time, packet LIMIT 1 OFFSET ?", (m["member"], meta_id, m["seq"] - 1)).fetchone()
            if row is None:
                return out, sends, True
            have_gt, have = row[0], bytes(row[1])
            if m["packet"] == have:
                out.append((m["index"], "duplicate message by binary packet"))
                continue
            if (have_gt, have) < (m["gt"], m["packet"]):
                sends.append((m["index"], have))
                out.append((m["index"], "duplicate message by sequence number (1)"))
                continue
            conn.execute("DELETE FROM sync WHERE member = ? AND meta_message = ? AND global_time >= ?",
                         (m["member"], meta_id, have_gt))
            highest[m["member"]] = highest_of(m["member"])
            last_gt = highest[m["member"]][0]  # :1010 rebinds last_global_time; `seq` keeps its old value
        elif seq + 1 != m["seq"]:
            out.append((m["index"], ("delay", seq + 1, m["seq"] - 1)))
            continue
        if is_duplicate_sync_message(conn, community, m, sends):
            out.append((m["index"], "duplicate message by global_time (1)"))
            continue
        if last_gt and m["gt"] <= last_gt:
            out.append((m["index"], "higher sequence number with lower global time than most recent message"))
            continue
        highest[m["member"]] = (m["gt"], seq + 1)
        out.append((m["index"], None))
    return out, sends, False


def store_last_sync(conn, community, meta_id, history_size, messages):
    """_store for a LastSyncDistribution meta (dispersy.py:1521-1591): INSERT every message, then for every member of
    the batch DELETE its rows beyond the newest history_size by global time.  messages: (member, gt, packet).
    Returns the new row ids."""
    ids = []
    for member, gt, packet in messages:
        cur = conn.execute("INSERT INTO sync (community, member, global_time, meta_message, packet, sequence) "
                           "VALUES (?, ?, ?, ?, ?, ?)", (community, member, gt, meta_id, packet, None))
        ids.append(cur.lastrowid)
    items = []
    for member in set(m for m, _, _ in messages):
        all_items = conn.execute("SELECT id, global_time FROM sync WHERE meta_message = ? AND member = ? "
                                 "ORDER BY global_time", (meta_id, member)).fetchall()
        if len(all_items) > history_size:
            items.extend(all_items[:len(all_items) - history_size])
    conn.executemany("DELETE FROM sync WHERE id = ?", [(i,) for i, _ in items])
    return ids


def store_double_signed(conn, community, meta_id, history_size, messages):
    """_store for a double-member-signed LastSyncDistribution meta (dispersy.py:1521-1594): INSERT every message into
    sync (member = members[0]) and its member pair, smaller id first, into double_signed_sync (:1537-1541); then per
    member pair of the batch, the pair's rows joined through double_signed_sync in (global_time, packet) order, and the
    ones beyond the newest history_size DELETEd from both tables (:1567-1578, :1589-1594).
    messages: (member_a, member_b, gt, packet).  Returns the new row ids."""
    ids = []
    for a, b, gt, packet in messages:
        cur = conn.execute("INSERT INTO sync (community, member, global_time, meta_message, packet, sequence) "
                           "VALUES (?, ?, ?, ?, ?, ?)", (community, a, gt, meta_id, packet, None))
        ids.append(cur.lastrowid)
        conn.execute("INSERT INTO double_signed_sync (sync, member1, member2) VALUES (?, ?, ?)",
                     (cur.lastrowid, min(a, b), max(a, b)))
    items = set()
    for m1, m2 in set((min(a, b), max(a, b)) for a, b, _, _ in messages):
        all_items = conn.execute("SELECT sync.id, sync.global_time FROM sync JOIN double_signed_sync ON "
                                 "double_signed_sync.sync = sync.id WHERE sync.meta_message = ? AND "
                                 "double_signed_sync.member1 = ? AND double_signed_sync.member2 = ? "
                                 "ORDER BY sync.global_time, sync.packet", (meta_id, m1, m2)).fetchall()
        if len(all_items) > history_size:
            items.update(all_items[:len(all_items) - history_size])
    if items:
        conn.executemany("DELETE FROM sync WHERE id = ?", [(i,) for i, _ in items])
        conn.executemany("DELETE FROM double_signed_sync WHERE sync = ?", [(i,) for i, _ in items])
    return ids


def insert_packets(conn, community, rows):
    """Dispersy._store's INSERT (dispersy.py:1523-1533): one statement per message, in message order.
    rows: iterable of (member, global_time, meta_message, packet).  Returns the new row ids (lastrowid)."""
    ids = []
    for member, gt, meta, packet in rows:
        cur = conn.execute("INSERT INTO sync (community, member, global_time, meta_message, packet, sequence) "
                           "VALUES (?, ?, ?, ?, ?, ?)", (community, member, gt, meta, packet, None))
        ids.append(cur.lastrowid)
    return ids


def syncable(metas):
    """Metas synced by bloom filters: SyncDistribution with priority > 32 (community.py:767, :2790-2794)."""
    return [m for m in metas if m["priority"] > 32]


def ordered_metas(metas):
    """Priority DESC, stable over declaration order (community.py:2790-2794)."""
    return sorted(syncable(metas), key=lambda m: m["priority"], reverse=True)


def meta_time_low(meta, time_low, global_time, include_inactive):
    """community.py:2800-2808: with include_inactive=False, GlobalTimePruning metas only offer active packets."""
    if include_inactive or not meta.get("pruning"):
        return time_low
    inactive = meta["pruning"][0]
    return min(max(time_low, global_time - inactive + 1), MAX_GT)


_ORDER = {"ASC": "global_time ASC", "DESC": "global_time DESC", "RANDOM": "RANDOM()"}


def selected_rows(conn, metas, time_low, time_high, offset, modulo, global_time, include_inactive):
    """[(id, packet)] in the order the reference's UNION ALL query yields them."""
    out = []
    for meta in ordered_metas(metas):
        lo = meta_time_low(meta, time_low, global_time, include_inactive)
        sql = ("SELECT id, packet FROM sync WHERE meta_message = ? AND undone = 0 AND global_time BETWEEN ? AND ? "
               "AND (global_time + ?) % ? = 0 ORDER BY " + _ORDER[meta["direction"]])
        out.extend((i, bytes(p)) for i, p in conn.execute(sql, (meta["id"], lo, time_high, offset, modulo)))
    return out


def respond_lists(conn, metas, request, bloom, global_time, byte_limit, include_inactive=False):
    """Row ids the responder sends for one claim, in send order.

    request: (time_low, time_high, offset, modulo) with time_high already resolved (0 -> global_time) and clamped.
    bloom: an object with not_filter(iterator of tuples) (OracleBloom).
    """
    time_low, time_high, offset, modulo = request
    rows = selected_rows(conn, metas, time_low, time_high, offset, modulo, global_time, include_inactive)
    sent = []
    budget = byte_limit
    for packet, rid in bloom.not_filter((p, i) for i, p in rows):
        sent.append(rid)
        budget -= len(packet)
        if budget <= 0:
            break
    return sent


# ---------------------------------------------------------------------------------------------- claim side
def _ids(metas):
    return ", ".join(str(m["id"]) for m in syncable(metas))


def select_and_fix(conn, metas, global_time, to_select, higher=True):
    cmp, order = (">", "ASC") if higher else ("<", "DESC")
    data = [(g, bytes(p)) for g, p in conn.execute(
        "SELECT global_time, packet FROM sync WHERE meta_message IN (%s) AND undone = 0 AND global_time %s ? "
        "ORDER BY global_time %s LIMIT ?" % (_ids(metas), cmp, order), (global_time, to_select + 1))]
    fixed = len(data) > to_select
    if fixed:
        # the last global time may be only partially selected: drop that whole group
        cut = data[-1][0]
        data.pop()
        while data and data[-1][0] == cut:
            data.pop()
    if not higher:
        data.reverse()
    return data, fixed


def select_range(conn, metas, global_time, to_select, higher, own_global_time, acceptable):
    data, fixed = select_and_fix(conn, metas, global_time, to_select, higher)
    lowerfixed = higherfixed = True
    if len(data) < to_select:
        remain = to_select - len(data)
        if remain > 25:
            if higher:
                more, lowerfixed = select_and_fix(conn, metas, global_time + 1, remain, False)
                data = more + data
            else:
                more, higherfixed = select_and_fix(conn, metas, global_time - 1, remain, True)
                data = data + more
    rng = [data[0][0], data[-1][0], len(data)]  # IndexError on empty data, as community.py:857
    if higher:
        rng[0] = min(rng[0], global_time + 1)
        if not fixed:
            rng[1] = acceptable
        if not lowerfixed:
            rng[0] = 1
    else:
        rng[1] = max(rng[1], global_time - 1)
        if not fixed:
            rng[0] = 1
        if not higherfixed:
            rng[1] = acceptable
    return rng, data


def claim_largest(conn, metas, bits, error_rate, global_time, acceptable, nrsync, draws, bloom_cls):
    """Returns ((time_low, time_high, modulo, offset, bloom), nrsync_after)."""
    if not syncable(metas):
        return (1, acceptable, 1, 0, bloom_cls.from_m_f(8, 0.1, b"\x00")), nrsync
    bloom = bloom_cls.from_m_f(bits, error_rate, bytes([int(draws.random() * 256)]))
    from oracle.bloom_ref import capacity_for
    capacity = capacity_for(bloom.m, error_rate)
    gt = max(1, global_time)
    pivot = gt - int(draws.expovariate(1.0 / (gt / 2.0)))
    if pivot < 1:
        pivot = int(draws.random() * gt)
    if pivot > 1 and nrsync >= capacity:
        right, rdata = select_range(conn, metas, pivot - 1, capacity, True, gt, acceptable)
        if right[2] == capacity:
            left, ldata = select_range(conn, metas, pivot + 1, capacity, False, gt, acceptable)
            if (left[1] or gt) - left[0] > (right[1] or gt) - right[0]:
                rng, data = left, ldata
            else:
                rng, data = right, rdata
        else:
            rng, data = right, rdata
    else:
        rng = [1, acceptable]
        data, fixed = select_and_fix(conn, metas, 0, capacity, True)
        if data and fixed:
            rng[1] = data[-1][0]
            nrsync = capacity + 1
    if data:
        bloom.add_keys(p for _, p in data)
        return (min(rng[0], acceptable), min(rng[1], acceptable), 1, 0, bloom), nrsync
    return (1, acceptable, 1, 0, bloom_cls.from_m_f(8, 0.1, b"\x00")), nrsync


def claim_modulo(conn, metas, bits, error_rate, acceptable, draws, bloom_cls):
    """Returns ((1, acceptable, modulo, offset, bloom), nrsync_after)."""
    if not syncable(metas):
        return (1, acceptable, 1, 0, bloom_cls.from_m_f(8, 0.1, b"\x00")), 0
    bloom = bloom_cls.from_m_f(bits, error_rate, bytes([int(draws.random() * 256)]))
    from oracle.bloom_ref import capacity_for
    capacity = capacity_for(bloom.m, error_rate)
    ids = _ids(metas)
    nrsync = conn.execute("SELECT count(*) FROM sync WHERE meta_message IN (%s) AND undone = 0" % ids).fetchone()[0]
    modulo = int(math.ceil(nrsync / float(capacity)))
    if modulo > 1:
        offset = draws.randint(0, modulo - 1)
        packets = [bytes(p) for p, in conn.execute(
            "SELECT packet FROM sync WHERE meta_message IN (%s) AND undone = 0 AND (global_time + ?) %% ? = 0" % ids,
            (offset, modulo))]
    else:
        offset, modulo = 0, 1
        packets = [bytes(p) for p, in conn.execute(
            "SELECT packet FROM sync WHERE meta_message IN (%s) AND undone = 0" % ids)]
    bloom.add_keys(packets)
    return (1, acceptable, modulo, offset, bloom), nrsync


# ------------------------------------------------------------------------ array form (bench cpu_baseline)
def respond_arrays(packet_of, gt_by_meta, metas, request, bloom, global_time, byte_limit, include_inactive=False,
                   counter=None):
    """The responder over in-memory index columns instead of sqlite (used as the timed CPU baseline, where a
    10-million-row sqlite table cannot be built in seconds).  Selection walks the same index range as
    selected_rows() but evaluates the modulo predicate with numpy (faster than sqlite's per-row VM, so the baseline
    is generous to the CPU); the not_filter/byte-limit loop is the reference's, lazily hashing only until the
    budget is spent.

    packet_of(row) -> bytes-like; gt_by_meta[meta_id] = (rows, gts) numpy arrays sorted by (global_time, row),
    undone == 0 only.  counter: optional one-element list incremented per packet hashed."""
    import numpy as np
    time_low, time_high, offset, modulo = request

    def gen():
        for meta in ordered_metas(metas):
            rows, gts = gt_by_meta.get(meta["id"], (np.zeros(0, np.int64), np.zeros(0, np.uint64)))
            lo = meta_time_low(meta, time_low, global_time, include_inactive)
            a = int(np.searchsorted(gts, lo, side="left"))
            b = int(np.searchsorted(gts, time_high, side="right"))
            sel = np.arange(a, b)
            if modulo > 1 and len(sel):
                sel = sel[(gts[a:b] + np.uint64(offset)) % np.uint64(modulo) == 0]
            if meta["direction"] == "DESC":
                sel = sel[::-1]
            for i in sel.tolist():
                if counter is not None:
                    counter[0] += 1
                r = int(rows[i])
                yield (packet_of(r), r)

    sent, budget = [], byte_limit
    for packet, row in bloom.not_filter(gen()):
        sent.append(row)
        budget -= len(packet)
        if budget <= 0:
            break
    return sent

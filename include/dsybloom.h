/*
 * dsybloom.h -- C-ABI of the MI355X (gfx950) Bloom-filter synchronisation hot path.
 *
 * This is the drop-in boundary between Dispersy's Python host code and the hand-written HIP kernels in
 * dispersy_amd/csrc/.  Everything here is `extern "C"`, plain pointers and sizes; no C++ or torch types cross
 * it.  The Python side binds it with ctypes (dispersy_amd/_native.py); INTEGRATION.md shows the binding a
 * reference maintainer would add.
 *
 * Conventions
 *  - Every function returns an int status: DSY_OK (0) or a negative DSY_E* code.  dsy_last_error() returns a
 *    thread-local message for the last failure on the calling thread.
 *  - "host" entry points take caller-owned host buffers; they stage through the ctx's device workspace and
 *    block until the result is back on the host.  "_dev" entry points take device pointers (HBM) and enqueue on
 *    the ctx's stream without synchronising; call dsy_ctx_synchronize() before reading results.
 *  - Filters cross the boundary serialised exactly like BloomFilter.bytes (bloomfilter.py:288-298): m/8 bytes,
 *    bit i of the filter is bit (i & 7) of byte (i >> 3).  Device filter buffers must be allocated with
 *    dsy_filter_words(m) 32-bit words (zero tail padding), i.e. a multiple of 4 bytes.
 *  - Keys/packets are packed: a byte blob plus uint64 offsets[n+1]; key i is blob[offsets[i] .. offsets[i+1]).
 *  - A ctx is not reentrant (internal mutex); separate ctx objects may be used concurrently from different
 *    threads.
 */
#ifndef DSYBLOOM_H
#define DSYBLOOM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DSY_ABI_VERSION 1

/* status codes */
#define DSY_OK 0
#define DSY_EINVAL -1    /* invalid argument: mirrors the reference's asserts (bloomfilter.py:125-145) */
#define DSY_EHIP -2      /* a HIP runtime call failed */
#define DSY_ENOMEM -3    /* device allocation failed */
#define DSY_ECAPACITY -4 /* output capacity too small; the required size is returned through the count pointer */
#define DSY_EUNSORTED -5 /* store rows are not in (meta, global_time) order */
#define DSY_EEMPTY -6    /* the reference raises IndexError: a claim range over no rows (community.py:857) */
#define DSY_EINTERNAL -7 /* a device-side bounds check tripped (an internal invariant broke): the call's results are void */

/* hash families, selected exactly as bloomfilter.py:134-156 does from (m, k) */
#define DSY_MD5 0
#define DSY_SHA1 1
#define DSY_SHA256 2
#define DSY_SHA384 3
#define DSY_SHA512 4

/* synchronisation directions of a SyncDistribution (distribution.py:180-184) */
#define DSY_ASC 0
#define DSY_DESC 1
#define DSY_RANDOM 2

typedef struct dsy_ctx dsy_ctx;
typedef struct dsy_store dsy_store;

/* One Bloom filter's hashing parameters.  The host computes them with the reference's formulas
 * (bloomfilter.py:69-160); the library validates that hash_kind/chunk_bytes agree with (m_bits, k) and
 * returns DSY_EINVAL otherwise.  prefix_len < 256 (bloomfilter.py:131). */
typedef struct dsy_bloom_params {
    uint64_t m_bits;     /* filter size in bits, > 0, multiple of 8 */
    uint32_t k;          /* number of index chunks per key, 0 < k <= m_bits */
    int32_t hash_kind;   /* DSY_MD5 .. DSY_SHA512 */
    uint32_t chunk_bytes; /* 2 ('H'), 4 ('L') or 8 ('Q') */
    uint32_t prefix_len; /* 0..255 */
    uint8_t prefix[256]; /* the salt prefix: the digest input is prefix || key (bloomfilter.py:161,168-169) */
} dsy_bloom_params;

/* One incoming claim (an introduction-request's sync block, conversion.py:732-799, as resolved by
 * on_introduction_request, community.py:2545-2553). */
typedef struct dsy_request {
    uint64_t time_low;      /* inclusive, already min(., 2^63-1) */
    uint64_t time_high;     /* inclusive, already resolved (0 on the wire -> responder global_time) and clamped */
    uint32_t modulo;        /* >= 1 */
    uint32_t offset;        /* < modulo */
    uint64_t filter_offset; /* byte offset of this claim's filter inside the `filters` buffer (multiple of 4) */
    uint64_t m_bits;
    uint32_t k;
    int32_t hash_kind;
    uint32_t chunk_bytes;
    uint32_t prefix_len;
    uint8_t prefix[256];
} dsy_request;

/* One syncable meta-message, in the order the responder serves them: priority DESC, stable
 * (community.py:2790-2794).  Metas with priority <= 32 must not be passed. */
typedef struct dsy_meta {
    uint32_t meta_id;            /* value stored in the store's meta column (sync.meta_message) */
    int32_t direction;           /* DSY_ASC / DSY_DESC / DSY_RANDOM */
    uint32_t has_pruning;        /* 1 if the meta uses GlobalTimePruning (distribution.py:68-114) */
    uint32_t _pad;
    uint64_t inactive_threshold; /* GlobalTimePruning.inactive_threshold */
} dsy_meta;

/* ---------------------------------------------------------------------------------------------- library */
int dsy_abi_version(void);
const char* dsy_last_error(void);
/* Number of 32-bit words a device filter buffer for an m-bit filter occupies. */
uint64_t dsy_filter_words(uint64_t m_bits);
/* Validate (m, k, hash_kind, chunk) against bloomfilter.py:134-156 and return the hash family it implies in
 * *out_kind and chunk width in *out_chunk. */
int dsy_hash_family(uint64_t m_bits, uint32_t k, int32_t* out_kind, uint32_t* out_chunk);

int dsy_ctx_create(int device, dsy_ctx** out);
int dsy_ctx_destroy(dsy_ctx* ctx);
int dsy_ctx_synchronize(dsy_ctx* ctx);
/* The HIP stream (hipStream_t) the ctx enqueues on. */
void* dsy_ctx_stream(dsy_ctx* ctx);
/* Cross-stream ordering without a host wait (one event each): dsy_ctx_wait_stream makes the ctx stream wait for the
 * work enqueued so far on `stream` (e.g. torch's current stream, which an RCCL collective's completion is ordered
 * on); dsy_ctx_signal_stream makes `stream` wait for the work enqueued so far on the ctx stream.  stream may be
 * NULL (the null stream). */
int dsy_ctx_wait_stream(dsy_ctx* ctx, void* stream);
int dsy_ctx_signal_stream(dsy_ctx* ctx, void* stream);
/* The ctx stream waits (on the device) for a HIP event recorded elsewhere (hipEvent_t, e.g. a torch.cuda.Event
 * recorded behind one collective on a communication stream that has more queued since). */
int dsy_ctx_wait_event(dsy_ctx* ctx, void* event);
/* Kernel timing: when enabled, HIP events bracket every launch of the hash kernels on the ctx stream.
 * dsy_ctx_kernel_time returns the accumulated milliseconds and launch count of kernel class `which`
 * (0 = hash/test of the responder, 1 = single-filter bloom kernels, 2 = selection, 3 = compaction, 4 = the
 * simulator's claim build, 5 = the simulator's respond) and, for classes 0, 4 and 5, the algorithmic work those
 * launches did: compression blocks and packet bytes hashed.
 * enable: 0 off, 1 every class, or DSY_TIME_ONLY(mask) to bracket only the classes whose bit is set in mask (each
 * event pair is a marker packet on the stream: timing just the dominant kernel keeps the others' dispatch tight). */
#define DSY_TIME_ONLY(mask) (0x100 | ((mask)&0xff))
int dsy_ctx_set_timing(dsy_ctx* ctx, int enable);
int dsy_ctx_kernel_time(dsy_ctx* ctx, int which, double* out_ms, uint64_t* out_launches, uint64_t* out_blocks,
                        uint64_t* out_bytes);
int dsy_ctx_reset_timing(dsy_ctx* ctx);
/* Algorithmic work of timer class `which` since the last reset (accumulated whether or not timing is on):
 * out4[0] compression blocks, out4[1] key bytes hashed, out4[2] (class 0) pairs the reference would have hashed --
 * its lazy not_filter stops at the packet that spends the byte limit (community.py:2559-2567), the GPU hashes whole
 * windows --, out4[3] lane-block slots of the hashing waves (64 x the longest lane per wave-task): out4[0] / out4[3]
 * is the active-lane fraction. */
int dsy_ctx_work(dsy_ctx* ctx, int which, uint64_t* out4);
/* Cap the responder's window at max_pairs (a multiple of 64; 0 restores the default, which grows from 4096 to 2^18
 * pairs per claim as claims finish).  Results do not depend on it; tests use small windows to exercise the
 * resumable cursor. */
int dsy_ctx_set_window(dsy_ctx* ctx, uint64_t max_pairs);

/* ---------------------------------------------------------------------------------- BloomFilter kernels */
/* Replaces BloomFilter.add / add_keys (bloomfilter.py:163-194): ORs the k bits of every key into filter_inout
 * (m/8 bytes, serialised as BloomFilter.bytes). */
int dsy_bloom_add(dsy_ctx* ctx, const dsy_bloom_params* p, const uint8_t* blob, uint64_t blob_len,
                  const uint64_t* offsets, uint64_t n, uint8_t* filter_inout);
/* Replaces the digest + probe of BloomFilter.__contains__ (bloomfilter.py:202-212) and not_filter
 * (:214-237): out_present[i] = 1 iff every probe bit of key i is set. */
int dsy_bloom_test(dsy_ctx* ctx, const dsy_bloom_params* p, const uint8_t* blob, uint64_t blob_len,
                   const uint64_t* offsets, uint64_t n, const uint8_t* filter, uint8_t* out_present);
/* The k bit positions of every key (digest slicing of bloomfilter.py:158-171): out_idx[i*k + j]. */
int dsy_bloom_indices(dsy_ctx* ctx, const dsy_bloom_params* p, const uint8_t* blob, uint64_t blob_len,
                      const uint64_t* offsets, uint64_t n, uint64_t* out_idx);

/* Device-pointer forms.  d_blob must stay readable for DSY_BLOB_GUARD bytes before offsets[0] and past
 * offsets[n] (the kernels read whole 64/128-byte blocks and mask, and fetch block 0 from key - prefix_len);
 * d_filter holds dsy_filter_words(m) words. */
#define DSY_BLOB_GUARD 256
int dsy_bloom_add_dev(dsy_ctx* ctx, const dsy_bloom_params* p, const uint8_t* d_blob, const uint64_t* d_offsets,
                      uint64_t n, uint32_t* d_filter);
int dsy_bloom_test_dev(dsy_ctx* ctx, const dsy_bloom_params* p, const uint8_t* d_blob, const uint64_t* d_offsets,
                       uint64_t n, const uint32_t* d_filter, uint8_t* d_present);

/* ------------------------------------------------------------------------------------------ packet store */
/* The packed HBM export of the `sync` table (dispersydatabase.py:53-64): rows sorted by
 * (meta_message, global_time, rowid) -- the order of the sync_meta_message_undone_global_time_index.
 * undone may be NULL (all rows live).  Rows with undone != 0 never take part in selection. */
int dsy_store_upload(dsy_ctx* ctx, const uint8_t* blob, uint64_t blob_len, const uint64_t* offsets, uint64_t n,
                     const uint64_t* global_time, const uint32_t* meta, const uint8_t* undone, dsy_store** out);
/* Same, over device buffers the caller keeps alive (the index arrays are not copied).  d_blob needs
 * DSY_BLOB_GUARD readable bytes before offsets[0] and past offsets[n].
 * Both forms also build the responder's line copy of the packets on the device: every packet starts one byte
 * into a 128-byte line (<= 128 bytes of padding per row), so the hashing kernel's loads are whole cache lines and a
 * message with a 1-byte prefix starts on a line. */
int dsy_store_attach(dsy_ctx* ctx, const uint8_t* d_blob, uint64_t blob_len, const uint64_t* d_offsets, uint64_t n,
                     const uint64_t* d_global_time, const uint32_t* d_meta, const uint8_t* d_undone, dsy_store** out);
int dsy_store_free(dsy_store* store);
uint64_t dsy_store_rows(const dsy_store* store);
/* Requester-side ingest: replaces `INSERT INTO sync (...)` of Dispersy._store (dispersy.py:1475-1612) for a batch
 * of a received packets (host buffers, any order; undone = 0).  The new rows take row positions n .. n+a-1 in
 * argument order (so they keep the rowid order of the inserts) and enter the responder's index by
 * (meta_message, global_time, rowid): a new row follows every stored row with the same meta and global time.
 * The device buffers grow by >= 1.25x when full (copied once); an attached store's caller buffers are left as they
 * were and are no longer read.  The call is O(a): the rows' index entries are queued on the device and join the index
 * when something next reads it (one merge for every append since): each meta's tail from its first new entry on is
 * merged in place into the slack its index region keeps, or -- when a meta's slack is spent -- the whole index is
 * merged once and laid out with fresh slack (a quarter of each region, at least 16384 entries). */
int dsy_store_append(dsy_ctx* ctx, dsy_store* store, const uint8_t* blob, uint64_t blob_len, const uint64_t* offsets,
                     uint64_t a, const uint64_t* global_time, const uint32_t* meta, const uint64_t* member);
/* The same with the packets given as a gather list: packet j is lengths[j] bytes at host address addrs[j] (the
 * caller's own packet objects -- no joined copy); they are copied into the library's pinned staging and uploaded
 * with the columns in one transfer. */
int dsy_store_append_gather(dsy_ctx* ctx, dsy_store* store, const uint64_t* addrs, const uint64_t* lengths, uint64_t a,
                            const uint64_t* global_time, const uint32_t* meta, const uint64_t* member);
/* The responder index's bookkeeping: out[0] live entries, out[1] entries of the index arrays (live + slack),
 * out[2] in-place tail merges, out[3] whole-index merges, out[4] index bytes moved by them (reads + writes),
 * out[5] queued entries not merged yet. */
int dsy_store_index_stats(const dsy_store* store, uint64_t* out6);

/* GlobalTimePruning's DELETE FROM sync WHERE meta_message = ? AND global_time <= ? (community.py:1092-1096, run by
 * update_global_time): the meta's rows up to max_global_time leave the responder's index and, when the store has a
 * (member, global_time) table, that table.  *out_deleted = their number. */
int dsy_store_prune(dsy_ctx* ctx, dsy_store* store, uint32_t meta, uint64_t max_global_time, uint64_t* out_deleted);

/* DELETE FROM sync WHERE id = ? for k arbitrary store rows (0-based positions): the conflict DELETE of the
 * sequence-number check (dispersy.py:1006-1007) and LastSyncDistribution's history pruning (dispersy.py:1581-1591).
 * The rows leave the responder's live index (a stable compaction on the device) and, when the store has a
 * (member, global_time) table, that table too (their slots become tombstones).  Rows may repeat, be undone or be
 * deleted already.  *out_deleted = live index entries removed. */
int dsy_store_delete(dsy_ctx* ctx, dsy_store* store, const uint64_t* rows, uint64_t k, uint64_t* out_deleted);

/* UPDATE sync SET undone = ? for k store rows (0-based positions): Community.on_undo's UPDATE ... WHERE community = ?
 * AND member = ? AND global_time = ? (community.py:3479-3480) and _update_timerange's UPDATE ... WHERE id = ?
 * (:3635, :3642), as the device index sees them.  undone != 0: the rows leave the responder's live index (it serves
 * undone = 0 only, community.py:2764-2787; rows out of the index already are ignored) but keep their
 * (member, global_time) slots, so the duplicate check still finds them and the caller sends the undo proof
 * (dispersy.py:886-892); *out_changed = index entries removed.  undone == 0 (redo): the rows -- undone, not deleted,
 * each once, meta[k] / global_time[k] their columns -- re-enter the index at their (meta_message, global_time, row)
 * place; a row in the index already gives DSY_EINVAL (nothing changes); *out_changed = k.  Which undo packet undid a
 * row (the value of the column) is the caller's: only "undone or not" reaches the device. */
int dsy_store_set_undone(dsy_ctx* ctx, dsy_store* store, const uint64_t* rows, uint64_t k, const uint32_t* meta,
                         const uint64_t* global_time, int undone, uint64_t* out_changed);

/* ------------------------------------------------------------------------------------ duplicate check */
/* Received sync packets are checked against the store by (member, global_time) before they are stored
 * (_is_duplicate_sync_message, dispersy.py:831-918; the sync table is UNIQUE(community, member, global_time)).
 * dsy_store_index_members builds the store's (member, global_time) -> row table from the member and global time
 * of every row (host arrays, n == dsy_store_rows); afterwards dsy_store_append must be given the appended rows'
 * members (member may be NULL only while a store has no table). */
#define DSY_DUP_NEW 0      /* no stored row with this (member, global_time): process the message */
#define DSY_DUP_EXACT 1    /* binary identical packet stored (dispersy.py:872) */
#define DSY_DUP_KEEP 2     /* same first signature_length bytes, stored packet >= received: keep ours (:893) */
#define DSY_DUP_REPLACE 3  /* same first signature_length bytes, stored packet < received: UPDATE it (:901-905) */
#define DSY_DUP_TRIPLET 4  /* same (member, global_time), different message (:910) */
int dsy_store_index_members(dsy_ctx* ctx, dsy_store* store, const uint64_t* member, const uint64_t* global_time,
                            uint64_t n);
/* m received messages (host buffers): verdict[j] one of DSY_DUP_*, row[j] the stored row (~0 for DSY_DUP_NEW). */
int dsy_dup_check(dsy_ctx* ctx, const dsy_store* store, const uint64_t* member, const uint64_t* global_time,
                  const uint8_t* blob, uint64_t blob_len, const uint64_t* offsets, uint64_t m,
                  const uint32_t* signature_length, uint8_t* out_verdict, uint64_t* out_row);
/* UPDATE sync SET packet = ? for k rows (dispersy.py:903): the rows keep their place in the index; their new
 * packets go to the end of the line copy. */
int dsy_store_replace(dsy_ctx* ctx, dsy_store* store, const uint64_t* rows, const uint8_t* blob, uint64_t blob_len,
                      const uint64_t* offsets, uint64_t k);

/* Claim side (community.py:821, :924 and dispersy_store :698): OR the packets of the given store rows into a
 * filter.  rows are store row positions (0-based, export order). */
int dsy_bloom_add_rows(dsy_ctx* ctx, const dsy_bloom_params* p, const dsy_store* store, const uint64_t* rows,
                       uint64_t n, uint8_t* filter_inout);
/* Claim side, modulo strategy: replaces the SELECT of _dispersy_claim_sync_bloom_filter_modulo
 * (community.py:918, :922) and its add_keys (:924).  Selects, on the device, the live rows (undone == 0) of the given
 * metas with (global_time + offset) % modulo == 0 and ORs their packets into the filter; *out_count = rows added.
 * 0 <= offset < modulo, else DSY_EINVAL. */
int dsy_claim_modulo(dsy_ctx* ctx, const dsy_bloom_params* p, const dsy_store* store, const uint32_t* meta_ids,
                     uint32_t nmeta, uint64_t offset, uint64_t modulo, uint8_t* filter_inout, uint64_t* out_count);

/* Claim side, largest strategy (the default, community.py:763-837): everything after the random draws -- the pivot
 * from_gbtime (:776-780) is the caller's, like the filter's random prefix.  Selects the rows of the given syncable
 * metas around the pivot exactly as _select_bloomfilter_range / _select_and_fix do (:839-903: up to capacity rows
 * above and below it in global-time order, the trailing equal-global-time group dropped when over-full, the side
 * with the wider range kept; or, when nrsyncpackets < capacity or the pivot is <= 1, the first capacity rows), on
 * the device over the live index, and ORs their packets into filter_inout (:821).
 * out_claim[0..3] = time_low, time_high (both already min(., acceptable_global_time)), rows added (0: the caller
 * returns the empty claim of :837), and the new _nrsyncpackets (capacity + 1 when the first-rows branch was
 * over-full, :810-815, else nrsyncpackets).  DSY_EEMPTY where the reference raises IndexError (a stale
 * nrsyncpackets over a store with no rows on the pivot's side, :857). */
int dsy_claim_largest(dsy_ctx* ctx, const dsy_bloom_params* p, const dsy_store* store, const uint32_t* meta_ids,
                      uint32_t nmeta, uint64_t from_gbtime, uint64_t capacity, uint64_t nrsyncpackets,
                      uint64_t acceptable_global_time, uint8_t* filter_inout, uint64_t* out_claim);

/* ------------------------------------------------------------------------------------------- responder */
/* Batched responder: replaces _get_packets_for_bloomfilters (community.py:2746-2811) plus the byte-limited
 * not_filter loop of on_introduction_request (:2555-2567) for R claims at once.
 *
 * For claim r the response is the ordered list of store rows the reference would send: metas in the given
 * order; within a meta rows with undone == 0, time_low' <= global_time <= time_high and
 * (global_time + offset) % modulo == 0, in global_time ASC / DESC (ties by row) or a seeded random order for
 * DSY_RANDOM; keep rows whose packet is NOT in the claim's filter; stop after the packet whose length makes the
 * running byte total reach byte_limit (that packet is included).  time_low' = max(time_low,
 * responder_global_time - inactive_threshold + 1) for GlobalTimePruning metas when include_inactive == 0.
 *
 * Output: out_idx[out_req_offsets[r] .. out_req_offsets[r+1]) are claim r's rows in send order.  If out_cap
 * is too small DSY_ECAPACITY is returned and out_req_offsets[R] holds the required size. */
int dsy_sync_respond(dsy_ctx* ctx, const dsy_store* store, const dsy_request* reqs, uint32_t R,
                     const uint8_t* filters, uint64_t filters_len, const dsy_meta* metas, uint32_t nmeta,
                     uint64_t responder_global_time, int include_inactive, int64_t byte_limit, uint64_t random_seed,
                     uint64_t* out_idx, uint64_t out_cap, uint64_t* out_req_offsets);

/* Object form of dsy_sync_respond, for a caller whose claims are separate objects (one BloomFilter per claim,
 * community.py:2531-2553): claim r is ranges[4r .. 4r+3] = time_low, time_high, modulo, offset (the bounds clamped to
 * 2^63-1 here) and refs[2r] = the address of a dsy_request that carries its filter's shape and prefix (m_bits, k,
 * hash_kind, chunk_bytes, prefix_len, prefix; its range and filter_offset fields are ignored), refs[2r+1] = the
 * address of its m_bits/8 filter bytes.  The library lays the filters out and gathers them into pinned staging while
 * the GPU runs the first window's selection; the caller builds no record array and no packed buffer.  Output and
 * errors as dsy_sync_respond.  Replaces community.py:2531-2572's per-request loop for SyncCommunity.respond. */
int dsy_sync_respond_refs(dsy_ctx* ctx, const dsy_store* store, const uint64_t* ranges, const uint64_t* refs, uint32_t R,
                          const dsy_meta* metas, uint32_t nmeta, uint64_t responder_global_time, int include_inactive,
                          int64_t byte_limit, uint64_t random_seed, uint64_t* out_idx, uint64_t out_cap,
                          uint64_t* out_req_offsets);

/* Device form: reqs/metas stay host structs (uploaded into the ctx workspace), filters are device memory
 * (d_filters), results stay in device memory owned by the ctx until the next call:
 *   *d_out_idx   -> uint64 rows, claim r at [d_out_offsets[r], d_out_offsets[r+1])
 *   *d_out_offsets -> uint64[R+1]
 * *out_total_pairs receives the number of (claim, packet) pairs hashed and tested (the bench metric's unit). */
int dsy_sync_respond_dev(dsy_ctx* ctx, const dsy_store* store, const dsy_request* reqs, uint32_t R,
                         const uint8_t* d_filters, const dsy_meta* metas, uint32_t nmeta,
                         uint64_t responder_global_time, int include_inactive, int64_t byte_limit,
                         uint64_t random_seed, const uint64_t** d_out_idx, const uint64_t** d_out_offsets,
                         uint64_t* out_total_pairs);

/* Pipelined form of dsy_sync_respond_dev for a stream of batches (a responder serving receive batch after receive
 * batch): submit validates and stages the claims and enqueues the batch's first window without waiting; wait finishes
 * it (the further windows its unfinished claims need) and returns what dsy_sync_respond_dev returns.  Up to three
 * batches are in flight per ctx, each with its own workspace; they run back to back on the ctx stream, so the GPU
 * goes from one batch's packing straight into the next one's selection while the host stages batches and collects
 * results.  Results are the same as the synchronous call's; a batch's
 * output buffers stay valid until its slot is reused: submit takes the least recently used free slot, so two more
 * submits at the earliest -- or any synchronous responder call (dsy_sync_respond / _dev always run in slot 0).
 * While a batch is in flight the store must not change (append, prune, delete, replace and free return DSY_EINVAL)
 * and the synchronous responder calls return DSY_EINVAL; d_filters must stay valid until wait returns.  A fourth
 * submit returns DSY_EINVAL. */
int dsy_sync_respond_submit(dsy_ctx* ctx, const dsy_store* store, const dsy_request* reqs, uint32_t R,
                            const uint8_t* d_filters, const dsy_meta* metas, uint32_t nmeta,
                            uint64_t responder_global_time, int include_inactive, int64_t byte_limit,
                            uint64_t random_seed, uint64_t* out_ticket);
int dsy_sync_respond_wait(dsy_ctx* ctx, uint64_t ticket, const uint64_t** d_out_idx, const uint64_t** d_out_offsets,
                          uint64_t* out_total_pairs);

/* Union of G partial filters of one (m, k, prefix) built over disjoint key shards (the large-filter
 * build shards keys over GPUs; RCCL reduces only sum/prod/min/max, so the partials are all-gathered over xGMI and
 * OR-ed here): d_out[w] = OR_g d_parts[g * words + w].  Device pointers; enqueued on the ctx stream. */
int dsy_filter_or_reduce(dsy_ctx* ctx, const uint32_t* d_parts, uint32_t n_parts, uint64_t words, uint32_t* d_out);

/* ------------------------------------------------------------------------------- sync block wire codec */
/* The sync part of an introduction-request payload (conversion.py:712-730 encode, :732-799 decode): struct
 * '>QQHHBH' (time_low, time_high, modulo, offset, functions, size in bits), the 1-byte prefix, then size/8 filter
 * bytes up to the end of the payload.  DSY_SYNC_HEADER = 23 + 1.  Decoding a batch gives per-item status codes
 * (the reference's DropPacket reasons, checked in its order) and, for the good items, dsy_request records whose
 * filters are packed 4-byte aligned into out_filters -- exactly what dsy_sync_respond takes. */
#define DSY_SYNC_HEADER 24
#define DSY_DROP_OK 0
#define DSY_DROP_SIZE 1        /* "Insufficient packet size"                 conversion.py:763-764 */
#define DSY_DROP_TIME_LOW 2    /* "Invalid time_low value"                   :772-773 */
#define DSY_DROP_TIME_HIGH 3   /* "Invalid time_high value"                  :774-775 */
#define DSY_DROP_MODULO 4      /* "Invalid modulo value"                     :776-777 */
#define DSY_DROP_OFFSET 5      /* "Invalid offset value"                     :778-779 */
#define DSY_DROP_FUNCTIONS 6   /* "Invalid functions value"                  :780-781 */
#define DSY_DROP_SIZE_VALUE 7  /* "Invalid size value"                       :782-783 */
#define DSY_DROP_SIZE_MULT8 8  /* "Invalid size value, must be a multiple of eight"  :784-785 */
#define DSY_DROP_LENGTH 9      /* "Invalid number of bytes available"        :787-789 */
/* Not a DropPacket: BloomFilter(bytes, k, prefix) (conversion.py:791) asserts when k > m or (m, k) needs more than 512
 * digest bits (bloomfilter.py:129, :144).  That AssertionError leaves _decode_introduction_request uncaught (only
 * DropPacket is caught, community.py:2086), so the reference abandons the whole receive batch; the Python binding
 * raises AssertionError for it (pinned by tests/golden/codec_vectors.json). */
#define DSY_DECODE_ASSERT 10
/* blob + offsets[n+1]: each item is one sync block (from its first byte to the end of the payload).  When
 * responder_global_time != 0, time_high == 0 is resolved to it and both bounds are clamped to 2^63-1 as
 * on_introduction_request does (community.py:2545-2553).  If out_filters is too small, DSY_ECAPACITY is returned
 * with the space needed so far in *out_filters_len (at most 8 KiB per item). */
int dsy_sync_decode(const uint8_t* blob, const uint64_t* offsets, uint32_t n, uint64_t responder_global_time,
                    dsy_request* out_reqs, uint8_t* out_filters, uint64_t filters_cap, uint64_t* out_filters_len,
                    int32_t* out_status);
/* Encode n claims (prefix_len 1, 0 < k < 256, m % 8 == 0 -- the asserts of conversion.py:723-726 --, and m, modulo,
 * offset < 2^16 -- the '>QQHHBH' field widths) into out; out_offsets[n+1] delimit the blocks.  Values only the
 * decoder rejects (time_low 0, offset >= modulo, ...) are encoded as given, as the reference does. */
int dsy_sync_encode(const dsy_request* reqs, uint32_t n, const uint8_t* filters, uint8_t* out, uint64_t out_cap,
                    uint64_t* out_offsets);

/* ------------------------------------------------------------------ epidemic-sync simulator (config 3) */
/* Simulated peers run the reference protocol once per round (see dispersy_amd/csrc/dsy_sim_kernels.hip):
 * requester claim = _dispersy_claim_sync_bloom_filter_largest's below-capacity branch (community.py:808-821),
 * responder = _get_packets_for_bloomfilters + the byte-limited loop (community.py:2555-2567), then the requester
 * stores what it got.  Peers are block-sharded over ranks; claims and responses are fixed-size records the host
 * exchanges between ranks (RCCL all-to-all(v)).  Stores are bitsets over a universe of packets whose global time
 * is index + 1.  All buffers are device pointers.  build_claims, respond (out_tested NULL) and merge enqueue
 * without waiting: their work counters stay on the device until a synchronising accessor (dsy_ctx_synchronize,
 * _kernel_time, _work, dsy_sim_stats) folds them, and a response overflow is reported by the next dsy_sim_stats.
 * The count queries (claim_counts, resp_counts, claim_matrix) return host values and wait for what they need. */
#define DSY_SIM_RESP_MAX 64

typedef struct dsy_sim_config {
    uint64_t n_peers;        /* P, all ranks */
    uint64_t peer_begin;     /* this rank's peers [peer_begin, peer_end) */
    uint64_t peer_end;
    uint64_t peers_per_rank; /* owner(p) = p / peers_per_rank */
    uint32_t universe;       /* U packets, id 0..U-1, global_time = id + 1; U <= 65536 */
    uint32_t words;          /* bitset words per peer (set by dsy_sim_setup) */
    uint64_t m_bits;         /* claim filter (community.py:637-666), m <= 65536 */
    uint32_t k;
    int32_t hash_kind;
    uint32_t chunk_bytes;
    uint32_t capacity;       /* BloomFilter.get_capacity(f) (community.py:774) */
    int64_t byte_limit;      /* dispersy_sync_response_limit (community.py:935-941) */
    uint64_t seed;
    uint32_t claim_bytes;    /* record sizes (set by dsy_sim_setup) */
    uint32_t resp_bytes;
} dsy_sim_config;

typedef struct dsy_sim_claim_header {
    uint64_t requester, responder, time_high;
    uint32_t prefix, n_sent;
} dsy_sim_claim_header;  /* followed by the filter words */

typedef struct dsy_sim_resp_header {
    uint64_t requester;
    uint32_t count, overflow;
} dsy_sim_resp_header;   /* followed by count uint16 packet ids */

int dsy_sim_setup(dsy_sim_config* cfg);
int dsy_sim_seed(dsy_ctx* ctx, const dsy_sim_config* cfg, uint32_t* d_bits, uint32_t initial);
/* claims this rank's requesters send to each rank in `round` (h_counts[n_ranks]) */
int dsy_sim_claim_counts(dsy_ctx* ctx, const dsy_sim_config* cfg, uint32_t round, uint32_t* h_counts, uint32_t n_ranks);
/* The claim traffic of n_rounds rounds from round0, all ranks: h_matrix[r][src][dst] (n_rounds x n_ranks x n_ranks)
 * = claims the requesters of rank src send to rank dst in round round0 + r.  Pairing is a counter RNG, so every rank
 * computes the same matrix and needs no count exchange.  Runs on a second stream of the ctx: it waits only for itself,
 * not for the work queued on the ctx stream. */
int dsy_sim_claim_matrix(dsy_ctx* ctx, const dsy_sim_config* cfg, uint32_t round0, uint32_t n_rounds,
                         uint32_t* h_matrix, uint32_t n_ranks);
/* build the claim records into d_out, grouped by destination rank at h_offsets[dest] (records, exclusive scan) */
int dsy_sim_build_claims(dsy_ctx* ctx, const dsy_sim_config* cfg, uint32_t round, const uint8_t* d_ublob,
                         const uint64_t* d_uoff, const uint32_t* d_bits, uint8_t* d_out, const uint32_t* h_offsets,
                         uint32_t n_ranks);
int dsy_sim_resp_counts(dsy_ctx* ctx, const dsy_sim_config* cfg, const uint8_t* d_claims, uint64_t n_claims,
                        uint32_t* h_counts, uint32_t n_ranks);
/* answer the received claims (responders are this rank's peers); responses grouped by the requester's rank at
 * h_offsets[rank].  out_tested (may be NULL: no wait) receives the (claim, packet) pairs this call tested. */
int dsy_sim_respond(dsy_ctx* ctx, const dsy_sim_config* cfg, const uint8_t* d_ublob, const uint64_t* d_uoff,
                    const uint32_t* d_bits, const uint8_t* d_claims, uint64_t n_claims, uint8_t* d_out,
                    const uint32_t* h_offsets, uint32_t n_ranks, uint64_t* out_tested);
/* store the received packets (each requester gets exactly one response per round) */
int dsy_sim_merge(dsy_ctx* ctx, const dsy_sim_config* cfg, uint32_t* d_bits, const uint8_t* d_resps, uint64_t n_resps);
/* out[0] = packets held by this rank's peers, out[1] = order-independent checksum of their stores */
int dsy_sim_stats(dsy_ctx* ctx, const dsy_sim_config* cfg, const uint32_t* d_bits, uint64_t* out);

#ifdef __cplusplus
}
#endif
#endif /* DSYBLOOM_H */

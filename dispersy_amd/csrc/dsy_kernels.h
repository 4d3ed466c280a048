// dsy_kernels.h -- launch descriptors shared by the C-ABI (dsy_capi.hip) and the kernel translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

#include "../../include/dsybloom.h"
#include "dsy_message.h"

namespace dsy {

// Device copy of one filter's hashing parameters (the prefix must live in device memory: lanes index it).
struct DevParams {
    uint64_t m_bits;
    uint32_t k;
    uint32_t prefix_len;
    uint8_t prefix[256];
};

enum class BloomOp { Add, Test, Indices };

// One (claim, packet) pair -- or one key of a single-filter batch -- as a hashing kernel consumes it, written in
// hashing order (sorted by block count): where the packet starts in the blob, its length, and its slot (the
// window slot / key index whose result it produces).
struct __attribute__((aligned(16))) PairTask {
    uint64_t off;
    uint32_t len;
    uint32_t slot;
};

// One (claim, packet) pair of a pooled family (k_pool_scatter -> k_pair_test<POOL>): the family's pairs of every
// active claim in one block-count order, so a hashing wave mixes claims and its 64 lanes run the same number of
// blocks.  The packet is line `line` of the store's line copy (+ kLineBias); a_slot / slot name the claim's window
// slot and the pair's place in its window.
struct __attribute__((aligned(16))) PoolTask {
    uint32_t line;
    uint32_t len;
    uint32_t a_slot;
    uint32_t slot;
};
// per hash family: block-count histogram of the window's pooled pairs (k_fill) and the scatter's cursors
static constexpr uint32_t kPoolBins = 1024;
static constexpr uint32_t kFamilies = 5 * 3 * 2;  // (hash kind x chunk class) x long-prefix flag, as respond_core
struct PoolCounts {
    uint32_t hist[kFamilies][kPoolBins];
    uint32_t cur[kFamilies][kPoolBins];
    uint32_t total[kFamilies];  // the family's pooled pairs in this window (k_pool_scatter)
    uint32_t next[kFamilies];   // wave-task queue head (k_pair_test<POOL> with pool_queue)
    uint32_t split[kFamilies];  // 1: a claim of the family filled a split window (its pairs have no pool_tab rows)
};

// A store row's packet in the line copy: starts kLineBias (dsy_message.h) bytes into a 128-byte line of
// StoreView::lines.
struct RowRec {
    uint64_t off;
    uint32_t len;
    uint32_t pad;
};

struct BloomLaunch {
    BloomOp op;
    int kind;
    uint32_t chunk;
    const DevParams* prm;
    uint32_t prm_prefix_len;  // host copy of prm->prefix_len (kernel choice)
    const uint8_t* blob;
    const uint64_t* offsets;
    const uint64_t* rows;     // optional indirection (add by store row)
    const RowRec* rec;        // with rows: key i is rec[rows[i]] in blob (a store's line copy); offsets unused
    const PairTask* tasks;    // optional length-bucketed order of the n keys (launch_len_sort)
    uint64_t n;
    uint32_t* filter;
    uint32_t nwords;
    int use_lds;
    uint8_t* present;
    uint64_t* indices;
    uint32_t max_grid;
    hipStream_t stream;
    int diag;               // k_bloom DIAG: 0 = the product kernel, 1 / 2 = compute / gather ceiling diagnostics
    int or_mode;            // filter build: filter_set_all OR_MODE (dsy_message.h)
    uint32_t line_kinds;    // bit k: hash kind k may use the line-aligned staging (bloom_staging)
    hipEvent_t ev_start, ev_stop;  // when set: recorded by the hashing kernel's own dispatch (launch_timed)
};

// A kernel launch whose start/stop events, when given, are recorded by the dispatch itself
// (hipExtLaunchKernelGGL: the timestamps of the kernel's AQL packet, no marker packets between kernels -- an event
// record between two dispatches leaves a ~6 us gap on the queue)
template <typename F, typename... Args>
inline void launch_timed(F kern, dim3 grid, dim3 block, size_t lds, hipStream_t stream, hipEvent_t ev_start,
                         hipEvent_t ev_stop, Args... args) {
    if (ev_start) hipExtLaunchKernelGGL(kern, grid, block, (uint32_t)lds, stream, ev_start, ev_stop, 0, args...);
    else hipLaunchKernelGGL(kern, grid, block, lds, stream, args...);
}

hipError_t launch_bloom(const BloomLaunch& L);
int bloom_staging(const BloomLaunch& L);  // 2: line-aligned LDS-DMA, 1: LDS-DMA windows, 0: direct loads
hipError_t launch_or_reduce(const uint32_t* parts, uint32_t n_parts, uint64_t words, uint32_t* out, uint32_t max_grid,
                            hipStream_t stream);

// Length-bucketed order of a key batch: tasks[0..n) sorted by compression-block count, longest first.
struct LenSort {
    uint32_t plen, blk, lenb;
    uint32_t line_mode = 0;  // bin by line stages (hash_key_dma_packed) instead of blocks
    uint32_t base_lo = 0;    // the blob's address mod 128 (line_mode)
};
hipError_t launch_len_sort(const LenSort& s, const uint64_t* offsets, const uint64_t* rows, const RowRec* rec, uint64_t n,
                           uint32_t* d_bins /* kLenSortBins */, PairTask* d_tasks, uint32_t max_grid, hipStream_t stream);
static constexpr uint32_t kLenSortBins = 1024;  // bins of the length sort (dsy_bloom_kernels.hip kLenBins)

// ------------------------------------------------------------------------------------------ responder
// One hashing wave-task as DSY_PAIR_TRACE records it: where it ran (HW_ID, XCC_ID), when (s_memrealtime, 100 MHz)
// and how long its longest lane was (blocks).
struct WaveTrace {
    uint32_t hw_id, xcc_id;
    uint64_t t0, t1;
    uint32_t blocks, task;
};

// Store view the responder kernels read.  `live` rows are the rows with undone == 0, in index order.

// (The packed upload -- blob + offsets -- is not in the view: store_release_raw frees it once the line copy is built,
// so no responder kernel can be handed a freed pointer; every packet is reached through `rec` into `lines`.)
struct StoreView {
    const uint8_t* lines;     // line copy of the packets (each starts on a 128-byte line)
    const RowRec* rec;        // [n_rows] where row i's packet sits in `lines`
    const uint64_t* live_gt;  // [n_live] global_time of live row i
    const uint64_t* live_row; // [n_live] store row of live row i (nullptr: identity)
    uint64_t n_live;
    uint64_t lines_bytes;     // bytes of `lines` (both DSY_BLOB_GUARD guards included): the hashing's bounds check
    uint64_t max_len;         // longest packet ever stored: the line-staged pieces keep 16-bit limits (kLinePathMaxLen)
};

// DmaLinePieces packs two per-piece live-byte limits into the 16-bit halves of a word; a padded message's limit is
// 64 x blocks - 8 of `1-byte prefix || packet`, which reaches 65536 at 65527-byte packets.  Stores holding a longer
// packet hash every family with the direct loads (the reference's own UDP cap, 65476 bytes, stays below).
constexpr uint64_t kLinePathMaxLen = 65526;

// Per (claim, meta) selection plan.
struct Plan {
    uint64_t a, b;     // live-row span [a, b) with lo' <= gt <= hi, inside the meta's segment
    uint64_t g0;       // first candidate global_time (enumerate mode)
    uint64_t ncand;    // size of the candidate space
    uint32_t mode;     // 0: scan live rows a..b   1: enumerate global times g0 + i*modulo
    uint32_t dir;      // DSY_ASC / DSY_DESC / DSY_RANDOM
    uint64_t perm_key; // RANDOM: permutation key
    uint32_t perm_bits;// RANDOM: Feistel half-width
    uint32_t dense;    // the span's global times are exactly g_lo..g_hi, one row each (row = a + g - g_lo)
    uint64_t g_lo, g_hi; // global_time at the span's ends (enumerate mode's one-round position guess)
};

// Work counters of the responder (device u64[8], accumulated over a call's windows).
// Spread over kCntSpread copies (a workgroup adds into copy blockIdx % kCntSpread): thousands of same-address
// atomics at the end of a launch serialise into its tail; the host sums the copies.
enum { kCntPairs = 0, kCntBlocks = 1, kCntBytes = 2, kCntUseful = 3, kCntSlots = 4, kCntN = 8 };
// host-mapped status words after the kCntN totals: [kStatusOverflow] a claim overflowed its output capacity
// (k_compact); [kStatusGuard] one byte per device-side bounds check that tripped (kGuard*): an index the responder
// computed fell outside the buffer it addresses -- the access is skipped and the call fails with DSY_EINTERNAL
enum { kStatusOverflow = kCntN, kStatusGuard = kCntN + 1, kStatusSeq = kCntN + 2 };
// [kStatusSeq] the number of the window whose pack kernel folded the status (counter slot kCntSeq keeps the count on
// the device): the host checks it after the window's completion event
static constexpr uint32_t kCntSeq = kCntN - 1;
enum { kGuardSortPos = 0, kGuardTask = 1, kGuardPack = 2, kGuardWindow = 3 };
__device__ __forceinline__ void guard_trip(uint64_t* h_status, int which) {
    ((volatile uint8_t*)&h_status[kStatusGuard])[which] = 1;
}
// a task record's packet lies inside the line copy with its guard bytes on both sides; overflow-safe, so a record
// the fill did not write this window (say 0xFF.. in recycled memory) cannot wrap around the check
__device__ __forceinline__ bool packet_in_lines(uint64_t off, uint64_t len, uint64_t lines_bytes) {
    return off >= DSY_BLOB_GUARD && len + 2 * DSY_BLOB_GUARD <= lines_bytes && off <= lines_bytes - DSY_BLOB_GUARD - len;
}
static constexpr uint32_t kCntSpread = 64;
__device__ __forceinline__ unsigned long long* counter(uint64_t* counters, uint32_t which) {
    return (unsigned long long*)&counters[(blockIdx.x % kCntSpread) * kCntN + which];
}

// Per-claim window state.
struct ReqState {
    uint32_t meta;     // current meta index
    uint32_t done;     // 1 once the byte limit is reached or every candidate was visited
    uint64_t cand;     // next candidate (iteration order) within the current meta
    uint64_t sub;      // rows of that candidate already emitted
    uint64_t n_window; // pairs placed in the current window
    uint64_t emitted;  // packets sent so far
    int64_t spent;     // bytes sent so far
    uint64_t cap;      // output capacity of this claim
    uint64_t out_base; // where this claim's output starts
    uint32_t exhausted;// every candidate of every meta visited
    uint32_t overflow; // output capacity exceeded (host retries with a larger capacity)
    uint64_t cand_next;// a split window's next cursor (k_fill's parts run concurrently): k_compact commits it to cand
    uint32_t commit;   // cand_next is pending
    uint32_t sort_later; // a big window filled by one workgroup: its histogram is in bulk_hist, k_fill_sort places it
    // the cursor at the start of the next window (written by k_compact): k_fill's workgroups decide on a split window
    // from it, not from the cursor its part 0 advances while the other parts may still be starting
    uint32_t win_meta;
    uint32_t pad;
    uint64_t win_cand;
    uint64_t win_sub;
};

// Device copy of one claim: the fields of dsy_request the kernels read, with the prefix bytes moved to a side
// buffer (a dsy_request is 296 B because of its 256-byte prefix array; claims carry 1 byte on the wire).
struct DevRequest {
    uint64_t time_low, time_high, filter_offset, m_bits;
    uint32_t modulo, offset, k, hash_kind, chunk_bytes, prefix_len;
    const uint8_t* prefix;  // device pointer into the call's prefix buffer
    uint32_t prefix_word;   // the first min(prefix_len, 4) prefix bytes, little-endian (the LDS-DMA paths' prefix)
    uint32_t m_recip;       // mod_recip(m_bits): bit positions by multiply-high (dsy_message.h bit_position)
    uint32_t pad[2];
};

struct SegMeta {          // one syncable meta in serving order, resolved against the store
    uint64_t seg_a, seg_b; // live-row segment of this meta id
    uint32_t dir;
    uint32_t has_pruning;
    uint64_t inactive;
};

enum { kFlagChunks = 0 };
struct RespondLaunch {
    StoreView st;
    const DevRequest* reqs;   // device [R]
    const SegMeta* metas;     // device [J]
    uint32_t R, J;
    const uint8_t* filters;   // device
    uint64_t responder_gt;
    int include_inactive;
    int64_t byte_limit;
    uint64_t seed;
    uint64_t window;          // W pairs per claim in this window
    const uint32_t* act;      // device [n_act]: window slot a serves claim act[a]
    uint32_t n_act;
    uint8_t* act_done;        // host-mapped [n_act]: written by k_compact, 1 once claim act[a] is done
    uint64_t* h_status;       // host-mapped [kCntN + 2]: counter totals (folded by the pack kernels), the
                              // overflow flag (k_compact) and the bounds-check bytes (kStatusGuard)
    Plan* plans;              // device [R*J]
    ReqState* state;          // device [R]
    uint64_t* upper;          // device [R]: upper bound of selected rows per claim
    uint64_t* emitted_n;      // device [R]: state[r].emitted, compact (written by k_compact, read by k_pack)
    uint32_t* ticket;         // device: k_setup's last-workgroup counter (zero between calls)
    uint64_t* pair_row;       // device [pool]: store row of window slot t
    uint64_t* pair_off;       // device [pool]: its packet's blob offset
    uint32_t* pair_len;       // device [pool]: its packet's length
    PairTask* task;           // device [R*W]: per-claim hashing order (window slots sorted by block count)
    uint32_t* bulk_hist;      // device [R][kSortBins]: a split window's block-count histogram (k_fill's parts), zero
                              // outside a window (k_compact clears what a window used)
    uint32_t* bulk_cur;       // device [R][kSortBins]: the split window's sort cursors (k_fill_sort)
    uint64_t* miss_mask;      // device [n_act * W / 64]: bit t of claim slot a = window pair t is missing
    uint64_t* out;            // device [sum cap]
    uint64_t packed_cap;      // rows the packed output holds (k_pack's bounds check)
    uint32_t* flags;          // device [16], zeroed by k_setup: [kFlagChunks] the window's longest claim in 64-pair
                              // chunks (k_fill atomicMax, read by k_pair_test, reset by k_compact)
    uint64_t* fill_clock;     // optional [n_act][4] s_memtime stamps of k_fill phases (DSY_FILL_PROFILE)
    WaveTrace* trace;         // optional (DSY_PAIR_TRACE): one record per k_pair_test wave-task, trace_n[0] counts them
    uint32_t* trace_n;
    uint32_t trace_cap;
    int diag;                 // k_pair_test DIAG (MD5 / SHA-1, 2-byte chunks): 0 product, 1 no loads, 2 loads only
    uint32_t direct_kinds;    // bit k: hash kind k hashes with direct loads, not the LDS-DMA line staging
    uint32_t grid_cap;        // k_pair_test workgroups at most (0: 2048)
    hipEvent_t ev_start, ev_stop;  // when set: recorded by k_pair_test's own dispatch (launch_timed)
    uint64_t* counters;       // device [kCntSpread][kCntN]: pairs hashed, compression blocks, packet bytes, pairs the reference
                              // would have hashed (it stops at the byte limit), lane-block slots of the hashing waves
    uint32_t pool_mask;       // bit f: family f's pairs are pooled across claims (k_fill counts, k_pool_scatter orders)
    int pool_queue;           // k_pair_test<POOL>: waves take wave-tasks from a queue instead of a grid stride
    int pool_deal;            // k_pair_test<POOL>: resident grid, wave-tasks dealt so each SIMD's waves sum to the mean
    int pair_prio;            // k_pair_test: wave priority by the wave-task's length (s_setprio)
    int bulk_zero;            // k_setup / k_fill_first zero the call's bulk_hist / bulk_cur rows (DSY_BULK_ZERO=0: not,
                              // a diagnostic of the state k_compact leaves between calls)
    PoolCounts* pool_counts;  // device, zero outside a window (k_pair_test<POOL> clears its family's)
    PoolTask* pool;           // device [pool]: the pooled order of the family being hashed
    uint32_t* pool_tab;       // device [2][R][kPoolBins] (pool_scan): k_fill's per-(claim, bin) counts and bin starts;
                              // k_pool_scan turns the starts into offsets in the family's pooled order
    int pool_scan;            // pooled families place pairs by the per-(claim, bin) scan, not by scatter atomics
    hipStream_t stream;
};

// the family id respond_core groups claims by
__device__ __host__ __forceinline__ uint32_t family_id(uint32_t kind, uint32_t chunk, uint32_t prefix_len) {
    return (kind * 3 + (chunk == 2 ? 0u : chunk == 4 ? 1u : 2u)) * 2 + (prefix_len > 4 || prefix_len == 0 ? 1u : 0u);
}

// copy the staged claims (pinned host h_src -> d_dst), zero d_zero, plans, upper bounds, and (per_claim_cap != 0)
// the per-claim capacities and states
hipError_t launch_setup(const RespondLaunch& L, const void* h_src, void* d_dst, size_t in_bytes, void* d_zero,
                        size_t zero_bytes, uint64_t per_claim_cap);
static constexpr uint32_t kPackFusedMax = 8192;  // claims packed by one launch (k_pack_fused)
hipError_t launch_fill(const RespondLaunch& L);
// diagnostics (DSY_FILL_SKEW, read when a ctx is created; process-wide): k_fill holds back waves 1-3 of a claim's
// one-workgroup fill by `sleeps` x s_sleep(127) before they read the window's cursor -- a wave scheduled late, on
// purpose (tests/test_fill_skew_gpu.py)
hipError_t set_fill_skew(uint32_t sleeps);
// first window of a one-meta call with device-side capacities: k_setup fused into k_fill (every claim's plan, state and
// window in one launch); h_act: the first active list in pinned host memory, or nullptr when window slot a is claim a
hipError_t launch_fill_first(const RespondLaunch& L, const void* h_src, void* d_dst, size_t in_bytes, void* d_counters,
                             size_t counter_bytes, uint64_t per_claim_cap, const uint32_t* h_act);
// hash + test the window's pairs of the listed window slots, all of one (hash kind, chunk) family
// long_prefix: the listed claims' prefixes are longer than 4 bytes (hashed without the LDS-DMA staging); padded: their
// prefixes are 1 byte (the line copy's padded messages, dsy_message.h line_bytes_for)
hipError_t launch_pair_test_list(const RespondLaunch& L, int kind, uint32_t chunk, bool long_prefix, bool padded,
                                 const uint32_t* d_list, uint32_t n);
// a pooled family (bit fam of L.pool_mask): its listed claims' window pairs into L.pool in block-count order
// (k_pool_scatter), then one hashing launch over the pool (k_pair_test<POOL>)
hipError_t launch_pair_test_pooled(const RespondLaunch& L, int kind, uint32_t chunk, bool long_prefix, bool padded,
                                   uint32_t fam, const uint32_t* d_list, uint32_t n);
hipError_t launch_compact(const RespondLaunch& L);
// diagnostics after a kGuardTask trip (k_task_audit): out[10] u64, zeroed by the caller
hipError_t launch_task_audit(const RespondLaunch& L, unsigned long long* out);
// done (optional): an event the last pack kernel's dispatch records when it completes
hipError_t launch_pack(const RespondLaunch& L, uint64_t* packed, uint64_t* packed_offsets, uint64_t* d_scan_tmp,
                       hipEvent_t done = nullptr);
// copy each row's packet from (blob, offsets) to its line-aligned place rec[i].off in lines
hipError_t launch_store_lines(const uint8_t* blob, const uint64_t* offsets, const RowRec* rec, uint64_t n,
                              uint8_t* lines, hipStream_t stream);

// ------------------------------------------------------------------------ duplicate check (dsy_dup_check)
// One slot of the store's (member, global_time) -> row table (open addressing, row == ~0: empty).
struct DupSlot {
    uint64_t member, gt, row, pad;
};
// A row's (member, global_time) key, kept per store row next to the table so a DELETE can find the row's slot.
struct DupKey {
    uint64_t member, gt;
};
// row == kDupTomb: a deleted row's slot -- not a match, not empty (probing continues past it); rehash drops it
static constexpr uint64_t kDupTomb = ~1ull;
hipError_t launch_dup_insert(const uint64_t* member, const uint64_t* gt, uint64_t first_row, uint64_t n, DupSlot* tab,
                             uint64_t mask, DupKey* keys, hipStream_t stream);
// tombstone the slots of rows[k] (or, rows == nullptr, of live_row[a .. a + k) / identity), keys from `keys`
hipError_t launch_dup_erase(const uint64_t* rows, const uint64_t* live_row, uint64_t a, uint64_t k, const DupKey* keys,
                            DupSlot* tab, uint64_t mask, hipStream_t stream);
hipError_t launch_dup_rehash(const DupSlot* old, uint64_t old_cap, DupSlot* tab, uint64_t mask, hipStream_t stream);
hipError_t launch_dup_check(const DupSlot* tab, uint64_t mask, const uint8_t* lines, const RowRec* rec,
                            const uint64_t* member, const uint64_t* gt, const uint8_t* blob, const uint64_t* offsets,
                            const uint32_t* sig_len, uint64_t m, uint8_t* verdict, uint64_t* out_row,
                            hipStream_t stream);
hipError_t launch_rec_scatter(RowRec* rec, const uint64_t* rows, const RowRec* src, uint64_t k, hipStream_t stream);

// ------------------------------------------------------------------------------- ingest (dsy_store_append)
// One appended row, the rows in (meta, global_time, rowid) order: its meta's live segment [seg_a, seg_b) in the old
// index ([x, x) at the meta's place when the meta is new) and its store row.
struct IngestRow {
    uint64_t gt, seg_a, seg_b, row;
};
// merge new index entries (appended or redone rows, in (meta, global_time, row) order) into the live index:
// (live_gt, live_row | identity)[n_live] + rows[a] -> (out_gt, out_row)[n_live + a]; rank[a] is scratch; present
// (optional): set to 1 when a row is in the index already
// GlobalTimePruning DELETE: k = rows of live_gt[a, b) with global_time <= max_gt (device u64), then the index
// without live rows [a, a + k) -> (out_gt, out_row)[n_out]
hipError_t launch_prune_count(const uint64_t* live_gt, uint64_t a, uint64_t b, uint64_t max_gt, uint64_t* out_k,
                              hipStream_t stream);
hipError_t launch_live_cut(const uint64_t* live_gt, const uint64_t* live_row, uint64_t n_out, uint64_t a, uint64_t k,
                           uint64_t* out_gt, uint64_t* out_row, uint32_t max_grid, hipStream_t stream);
// claim side, modulo strategy: rows of live segment [a, b) with (gt + offset) % modulo == 0 -> out_rows[*count++]
// (at most cap rows are written; *count still counts every hit)
hipError_t launch_claim_modulo(const uint64_t* live_gt, const uint64_t* live_row, uint64_t a, uint64_t b,
                               uint64_t offset, uint64_t modulo, uint64_t* out_rows, uint64_t cap,
                               unsigned long long* count, uint32_t max_grid, hipStream_t stream);
// Claim side, largest strategy: _select_and_fix (community.py:881-903) over the live segments of the syncable metas:
// up to to_select + 1 rows strictly above (higher) / below the pivot in global-time order across the metas; when
// over-full, the trailing equal-global-time group is dropped.  The result is a global-time interval: per meta the
// selected live-index span out_spans[2j .. 2j+1], and the counts below.  cand: scratch of J x (to_select + 1) u64
// (candidates ranked in it when the metas are more than one); cand_lds != 0: it fits LDS (dynamic shared memory).
struct SelResult {
    uint64_t count;     // rows selected (len(data))
    uint64_t first_gt;  // data[0] global time (ascending order), valid when count > 0
    uint64_t last_gt;   // data[-1] global time
    uint64_t total;     // candidates on the pivot's side
    uint32_t fixed;     // the selection was over-full (and the trailing group dropped)
    uint32_t pad;
};
hipError_t launch_select_and_fix(const uint64_t* live_gt, const uint64_t* spans, uint32_t J, uint64_t pivot,
                                 uint64_t to_select, int higher, uint64_t* cand, uint64_t* out_spans, SelResult* res,
                                 hipStream_t stream);
// rows of live-index spans (n_spans x (x, y)) -> out_rows, in span order; *total rows
hipError_t launch_span_rows(const uint64_t* live_row, const uint64_t* spans, uint32_t n_spans, uint64_t* out_rows,
                            hipStream_t stream);

// DELETE of arbitrary rows (dsy_store_delete): del_bits marks store rows; the live index loses every entry whose row is
// marked, stable.  Tiles of kDelTile entries: per-tile kept counts -> exclusive scan -> scatter; bounds[nb] (positions in
// the old index, ascending or not) are mapped to their positions in the new one.  d_tmp: (tiles + 1) u64 + 64 B.
static constexpr uint64_t kDelTile = 1024;
hipError_t launch_mark_rows(const uint64_t* rows, uint64_t k, uint64_t n_rows, uint32_t* del_bits, hipStream_t stream);
hipError_t launch_live_delete(const uint64_t* live_gt, const uint64_t* live_row, uint64_t n_live,
                              const uint32_t* del_bits, uint64_t* tile_tmp, uint64_t* out_gt, uint64_t* out_row,
                              uint64_t* bounds, uint32_t nb, hipStream_t stream);
hipError_t launch_ingest_merge(const uint64_t* live_gt, const uint64_t* live_row, uint64_t n_live,
                               const IngestRow* rows, uint64_t a, uint64_t* rank, uint64_t* out_gt, uint64_t* out_row,
                               unsigned int* present, uint32_t max_grid, hipStream_t stream);
// the P pending index entries (meta[j], gt[j], row base + j), glo <= gt <= ghi, as IngestRows in (meta, global_time,
// row) order; metas: the nm distinct pending metas ascending, segs: their live segments (a, b) in the old index
// (gap_before, optional: slack rows kept before rank r's rows -- the caller fills them, launch_gap_rows)
size_t pend_order_scratch(uint64_t P);
hipError_t launch_pend_order(const uint32_t* meta, const uint64_t* gt, uint64_t P, uint64_t glo, uint64_t ghi,
                             const uint32_t* metas, const uint64_t* segs, const uint64_t* gap_before, uint32_t nm,
                             uint64_t base, void* scratch, size_t scratch_bytes, IngestRow* out, hipStream_t stream);
// The live index keeps slack after each meta's live segment: entries [b, next meta's a) hold row kGapRow.  An append
// whose new entries fit its metas' slack merges each meta's tail in place (O(batch + the tail after its first new
// entry)); otherwise one merge of the whole index re-lays it out with fresh slack (k_gap_rows' entries).
static constexpr uint64_t kGapRow = ~0ull;
hipError_t launch_gap_rows(IngestRow* out, uint64_t k, uint64_t end, hipStream_t stream);
hipError_t launch_first_rank(const uint64_t* live_gt, const uint64_t* live_row, const IngestRow* rows,
                             const uint64_t* starts, const uint64_t* counts, uint32_t nm, uint64_t* out,
                             hipStream_t stream);
hipError_t launch_rows_seg(IngestRow* rows, uint64_t k, uint64_t sa, uint64_t sb, hipStream_t stream);
// ---------------------------------------------------------------------------------------- simulator
static constexpr uint32_t kSimFilterWordsMax = 2048;  // m <= 65536 bits
static constexpr uint32_t kSimRespMax = DSY_SIM_RESP_MAX;
enum { kSimSeed = 0, kSimClaimCounts, kSimBuild, kSimRespCounts, kSimRespond, kSimMerge, kSimStats, kSimClaimSlots,
       kSimRespSlots, kSimClaimMatrix, kSimCursorInit };
static constexpr uint32_t kSimMaxRanks = 64;  // cursor starts travel as a kernel argument up to this many ranks

// the per-destination record cursors of a build / respond call, passed by value (no host-to-device copy of
// pageable memory, which would wait for the stream)
struct SimCursorInit {
    uint32_t n;
    uint32_t start[kSimMaxRanks];
};
static constexpr uint32_t kSimTestedSlots = 64;  // k_sim_respond spreads its tested-pair counter over 64 words

struct SimLaunch {
    dsy_sim_config cfg;
    uint32_t round;
    uint32_t initial;
    const uint8_t* ublob;
    const uint64_t* uoff;
    uint32_t* bits;
    const uint8_t* in;
    uint64_t n_in;
    uint8_t* out;
    uint32_t* cursor;
    uint32_t* slots;
    uint32_t* counts;
    unsigned long long* tested;
    unsigned long long* stats;
    unsigned long long* work;  // [kSimTestedSlots][4]: build blocks, build lane-block slots, respond blocks, respond slots
    int or_mode;               // claim filter build: filter_set_all OR_MODE (dsy_message.h)
    uint32_t n_rounds;         // kSimClaimMatrix: rounds round .. round + n_rounds - 1
    uint32_t n_ranks;          // kSimClaimMatrix: matrix side
    SimCursorInit cursor_init; // kSimCursorInit
    hipStream_t stream;
};

hipError_t launch_sim(int op, const SimLaunch& L);

}  // namespace dsy

// dsy_capi.hip -- the extern "C" boundary (include/dsybloom.h): contexts, workspaces, validation that mirrors
// the reference's asserts, staging of host buffers, and orchestration of the responder windows.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "dsy_kernels.h"

using namespace dsy;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess) return fail(DSY_EHIP, "%s failed: %s", #expr, hipGetErrorString(_e)); \
    } while (0)

struct DevBuf {
    void* ptr = nullptr;
    size_t bytes = 0;
};

enum TimerClass { kTimePairTest = 0, kTimeBuild = 1, kTimeSelect = 2, kTimeCompact = 3, kTimeSimBuild = 4,
                  kTimeSimRespond = 5, kTimeClasses = 6 };

struct PendingTimer {
    int cls;
    hipEvent_t a, b;
};

}  // namespace

// grow-only named device buffers plus one grow-only pinned staging buffer
struct Workspace {
    std::map<std::string, DevBuf> ws;
    std::unordered_map<const char*, DevBuf*> by_name;  // ws_get's cache, keyed by the literal's address
    void* stage = nullptr;  // pinned: the responder's uploads and its host-mapped status
    size_t stage_bytes = 0;
    void release() {
        for (auto& kv : ws) if (kv.second.ptr) hipFree(kv.second.ptr);
        ws.clear();
        by_name.clear();
        if (stage) hipHostFree(stage);
        stage = nullptr;
        stage_bytes = 0;
    }
};

// One responder batch between its first window and its end (respond_core's state across the host syncs).
struct RespondJob {
    uint32_t R = 0, J = 0;
    const dsy_store* s = nullptr;
    std::vector<std::vector<uint32_t>> fam_active;  // per family: its active claims
    std::vector<int> fam_id;
    std::vector<uint8_t> pad1;  // per claim: a 1-byte prefix (the line copy's padded messages, hash_key_dma_lines)
    RespondLaunch L{};
    uint64_t pool = 0;
    uint8_t* h_in = nullptr;   // pinned staging (upload region, then host-mapped status)
    uint8_t* h_io = nullptr;
    uint32_t* h_act0 = nullptr;
    uint32_t* h_act_next = nullptr;  // pinned: a later window's active list (never the staged upload k_fill_first reads)
    uint64_t windows = 0;            // windows enqueued; the pack kernel numbers each in the status (kStatusSeq)
    bool act0_identity = true;  // h_act0[a] == a (k_fill_first may then map slot a to claim a without the list)
    const uint32_t* d_slots = nullptr;
    uint32_t* d_act = nullptr;
    void* d_in = nullptr;
    void* d_io = nullptr;
    void* d_packed = nullptr;
    void* d_packed_off = nullptr;
    size_t in_b = 0, cnt_b = 0;
    uint64_t per_claim = 0;
    uint64_t cap_pairs = 0;    // pairs the bound per-pair buffers hold (job_pair_buffers)
    bool fused_first = false, first = true, ran = false, first_fill = true;
    double hp[4] = {0, 0, 0, 0};
    double hp_wait = 0;
};

// A responder slot: its own workspace and job, so several batches can be in flight (dsy_sync_respond_submit).  Every
// batch runs on the ctx stream: the GPU executes the batches back to back, the next batch's selection right behind
// this one's packing, while the host stages the next batch and waits for this one on its own event (ev_done, recorded
// after each window's packing) instead of on the stream.  Measured and dropped (same box, tools/pipe_timeline.py):
// each slot on streams of its own, and selection / compaction on high-priority streams beside a low-priority hashing
// stream -- concurrent launches only slowed each other (a k_compact beside a hashing launch took 50-145 us instead of
// 6, the hashing launch 280-355 us instead of 210).
// dsy_sync_respond_refs: the claims' filters, copied into pinned staging and uploaded after the first window's
// selection is enqueued (job_window), so the host gathers them while the GPU selects
static constexpr size_t kOutPinMax = 64ull << 20;  // results of a host-buffer responder call kept in pinned memory

struct FilterGather {
    const uint64_t* refs = nullptr;  // claim r's filter bytes at refs[2r + 1]
    const uint64_t* foff = nullptr;  // and their place in the filters workspace
    uint32_t R = 0;
    uint64_t total = 0;              // bytes of the laid-out filters
    uint8_t* d_dst = nullptr;        // the filters workspace
};

struct RespondSlot {
    FilterGather gather;     // pending for the slot's next first window (dsy_sync_respond_refs), else empty
    Workspace w;
    hipEvent_t ev_done = nullptr;
    bool busy = false;       // submitted, not yet waited for
    uint64_t ticket = 0;
    uint64_t last_use = 0;   // when a job last started here: submit takes the least recently used free slot
    RespondJob job;
};

struct dsy_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    Workspace main;  // every entry point but the responder's
    static constexpr int kSlots = 3;  // responder batches in flight at most (dsy_sync_respond_submit)
    RespondSlot rs[kSlots];
    uint64_t next_ticket = 1;
    uint64_t use_clock = 0;  // RespondSlot::last_use
    uint32_t max_grid = 2048;
    int bloom_diag = 0;  // DSY_BLOOM_DIAG at creation: single-filter ceiling diagnostics (k_bloom DIAG)
    int pair_diag = 0;   // DSY_PAIR_DIAG at creation: responder ceiling diagnostics (k_pair_test DIAG)
    uint32_t bloom_grid = 0; // DSY_BLOOM_GRID at creation: k_bloom grid cap (0: 2 x max_grid)
    uint32_t pair_grid = 0;  // DSY_PAIR_GRID at creation: k_pair_test grid cap (0: max_grid, 8 workgroups per CU)
    int or_mode = 1;     // DSY_OR_MODE at creation: filter-build atomics (filter_set_all OR_MODE, dsy_message.h)
    // DSY_BLOOM_LINES at creation: bit k = hash kind k's single-filter hashing (k_bloom) stages whole lines
    // (hash_key_dma_packed); otherwise LDS-DMA windows at each key's own alignment (hash_key_dma_reg).  Same box,
    // config 1's 10 M-key test (profiles/cfg1_ab_r6.json): MD5 2248 us with lines vs 2294 us with windows; SHA-1
    // (VALU-bound) 3101 vs 3071 us, kept on lines for 1.18x instead of 1.51x the algorithmic HBM bytes
    uint32_t bloom_lines = (1u << DSY_MD5) | (1u << DSY_SHA1);
    // DSY_POOL at creation: bit k = hash kind k's responder pairs are pooled across claims (k_pool_scatter) -- MD5,
    // SHA-1 and SHA-256 only; DSY_POOL_QUEUE: the pooled hashing takes its wave-tasks from a queue.  Off by default:
    // on the SHA-1 leg pooling takes k_pair_test 104 -> 95 us (lane use 0.82 -> 1.00) but k_pool_scatter costs 18 us
    // (1024 workgroups' atomics on the same ~20 bin cursors), 0.149 -> 0.157 ms per step; MD5 headline 0.28 -> 0.30
    uint32_t pool_kinds = 0;
    int pool_queue = 0;
    int pool_scan = 0;   // DSY_POOL_SCAN=1: pooled pairs placed by the per-(claim, bin) scan (k_pool_scan), not the
                         // scatter's atomics -- measured slower (profiles/pool_scan_ab_r5.json)
    int pool_deal = 0;   // DSY_POOL_DEAL: the pooled hashing's resident-grid deal (k_pair_test<POOL>)
    int pair_prio = 1;   // DSY_PAIR_PRIO: k_pair_test raises the wave priority of long wave-tasks (0 off)
    int bulk_zero = 1;   // DSY_BULK_ZERO=0: the calls do not zero their split-window sort state (diagnostic)
    uint32_t direct_kinds = 0;  // DSY_PAIR_DIRECT: bit k = hash kind k's responder hashing uses direct loads
    uint32_t timing = 0;  // bit i: bracket class i with events
    std::vector<PendingTimer> pending;
    std::vector<hipEvent_t> event_pool;
    double time_ms[kTimeClasses] = {};
    uint64_t launches[kTimeClasses] = {};
    uint64_t blocks[kTimeClasses] = {};
    uint64_t bytes[kTimeClasses] = {};
    uint64_t useful[kTimeClasses] = {};  // pairs the reference would have hashed (responder)
    uint64_t slots[kTimeClasses] = {};   // lane-block slots of the hashing waves (load balance)
    void* pinned = nullptr;  // small pinned staging for flags/counters
    uint64_t window_cap = 0; // dsy_ctx_set_window: upper bound on the responder's window (0: the default 2^18)
    hipStream_t aux = nullptr;  // dsy_sim_claim_matrix: work that depends on nothing queued on `stream`
    hipEvent_t xev = nullptr;   // dsy_ctx_wait_stream / dsy_ctx_signal_stream
    hipEvent_t gev = nullptr;   // dsy_sync_respond_refs: the filters' upload on `aux` is done
    // host-buffer responder calls: the pack kernel writes the results (offsets, then rows) straight into this pinned,
    // device-visible buffer, so no download follows the step (respond_to_host; grow-only, up to kOutPinMax bytes)
    bool host_out = false;
    uint8_t* out_pin = nullptr;
    size_t out_pin_bytes = 0;
    // pinned staging of dsy_store_append's small columns (offsets, records, global times, metas, members): one
    // upload per append; the next append synchronises the stream before it writes here again
    uint8_t* in_stage = nullptr;
    size_t in_stage_bytes = 0;
    // pinned staging of store_flush's small table (metas, segments, slack, starts, counts): an asynchronous upload; a
    // flush only has work after an append, and every append synchronises the stream first, so the next flush may
    // rewrite it
    uint8_t* flush_pin = nullptr;
    size_t flush_pin_bytes = 0;
    // the simulator's device-side counters (work of build / respond, pairs tested, response overflow): the calls
    // enqueue without reading them back; the synchronising accessors fold them (sim_collect)
    void* sim_acc = nullptr;
    bool sim_pending = false;
    bool sim_overflow = false;
    int inflight() const {
        int n = 0;
        for (const auto& x : rs) n += x.busy;
        return n;
    }
};

struct dsy_store {
    dsy_ctx* ctx = nullptr;
    uint64_t n = 0, n_live = 0, blob_len = 0, min_len = 0;
    uint64_t max_len = 0;  // longest packet ever stored (grow-only): the line-staged hashing's 16-bit piece limits
    const uint8_t* d_blob = nullptr;
    const uint64_t* d_offsets = nullptr;
    const uint64_t* d_live_gt = nullptr;
    const uint64_t* d_live_row = nullptr;
    const uint8_t* d_lines = nullptr;  // line copy of the packets (the responder hashes from it)
    const RowRec* d_rec = nullptr;
    std::vector<void*> owned;
    std::unordered_map<uint32_t, std::pair<uint64_t, uint64_t>> segs;
    // capacities for dsy_store_append (0: exactly the built size)
    uint64_t lines_used = 0;  // bytes of d_lines in use (front guard + line-aligned packets)
    uint64_t lines_cap = 0;   // bytes of d_lines (the tail guard included)
    uint64_t rec_cap = 0;     // entries of d_rec
    uint64_t live_cap = 0;    // entries of d_live_gt / d_live_row when they are the ingest's own buffers
    DupSlot* dup = nullptr;   // (member, global_time) -> row table (dsy_store_index_members), or none
    uint64_t dup_cap = 0, dup_count = 0;
    DupKey* dup_keys = nullptr;  // every row's (member, global_time), for DELETEs to find the row's slot
    uint64_t keys_cap = 0;
    uint64_t* spare_gt = nullptr;   // the ingest's second index buffer pair (the next merge's target)
    uint64_t* spare_row = nullptr;
    uint64_t spare_cap = 0;
    // appended rows not yet in the live index (dsy_store_append is O(batch): the index absorbs every pending row in
    // ONE merge when something next reads it -- store_flush, called by every reader of the index)
    // on the device: (meta, global_time) of pending entry j, whose row is pend_base + j (appended rows are contiguous)
    uint32_t* d_pend_meta = nullptr;
    uint64_t* d_pend_gt = nullptr;
    uint64_t pend_n = 0, pend_cap = 0, pend_base = 0, pend_glo = 0, pend_ghi = 0;
    std::map<uint32_t, uint64_t> pend_cnt;  // pending entries per meta
    // entries of the live index arrays: the live ones (n_live) and each meta region's slack (store_flush)
    uint64_t n_phys = 0;
    uint64_t ix_fast = 0, ix_full = 0, ix_bytes = 0;  // in-place tail merges, whole-index merges, index bytes moved
};

namespace {

// grow-only named workspace buffer
int ws_get(Workspace& W, const char* name, size_t bytes, void** out, bool* fresh = nullptr) {
    // names are string literals: their address finds the buffer without building a std::string per call
    DevBuf*& slot = W.by_name[name];
    if (!slot) slot = &W.ws[name];  // std::map nodes do not move
    DevBuf& b = *slot;
    if (fresh) *fresh = b.bytes < bytes;
    if (b.bytes < bytes) {
        if (b.ptr) hipFree(b.ptr);
        b.ptr = nullptr;
        b.bytes = 0;
        size_t want = std::max<size_t>(bytes + bytes / 4, 256);
        if (hipMalloc(&b.ptr, want) != hipSuccess) {
            b.ptr = nullptr;
            return fail(DSY_ENOMEM, "hipMalloc(%zu) for workspace '%s' failed", want, name);
        }
        b.bytes = want;
    }
    *out = b.ptr;
    return DSY_OK;
}
int ws_get(dsy_ctx* c, const char* name, size_t bytes, void** out, bool* fresh = nullptr) {
    return ws_get(c->main, name, bytes, out, fresh);
}

// grow-only pinned host staging (one H2D upload and one D2H status read per responder window)
int stage_get(Workspace& W, size_t bytes, uint8_t** out) {
    if (W.stage_bytes < bytes) {
        if (W.stage) hipHostFree(W.stage);
        W.stage = nullptr;
        W.stage_bytes = 0;
        const size_t want = std::max<size_t>(bytes + bytes / 4, 4096);
        if (hipHostMalloc(&W.stage, want, hipHostMallocDefault) != hipSuccess) {
            W.stage = nullptr;
            return fail(DSY_ENOMEM, "hipHostMalloc(%zu) for the staging buffer failed", want);
        }
        W.stage_bytes = want;
    }
    *out = (uint8_t*)W.stage;
    return DSY_OK;
}

hipEvent_t take_event(dsy_ctx* c) {
    if (!c->event_pool.empty()) {
        hipEvent_t e = c->event_pool.back();
        c->event_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    hipEventCreate(&e);
    return e;
}

void timer_begin(dsy_ctx* c, PendingTimer* t, int cls, hipStream_t st = nullptr) {
    t->cls = cls;
    t->a = t->b = nullptr;
    if (!(c->timing & (1u << cls))) return;
    t->a = take_event(c);
    t->b = take_event(c);
    hipEventRecord(t->a, st ? st : c->stream);
}

void timer_end(dsy_ctx* c, PendingTimer* t, hipStream_t st = nullptr) {
    if (!t->a) return;
    hipEventRecord(t->b, st ? st : c->stream);
    c->pending.push_back(*t);
}

// the same timer for one kernel launched with launch_timed: its events are handed to the dispatch (*a, *b), not
// recorded on the stream around it; timer_dispatched files them after the launch
void timer_dispatch(dsy_ctx* c, PendingTimer* t, int cls, hipEvent_t* a, hipEvent_t* b) {
    t->cls = cls;
    t->a = t->b = nullptr;
    *a = *b = nullptr;
    if (!(c->timing & (1u << cls))) return;
    *a = t->a = take_event(c);
    *b = t->b = take_event(c);
}

void timer_dispatched(dsy_ctx* c, PendingTimer* t) {
    if (t->a) c->pending.push_back(*t);
}

// fold completed timers; timers whose events have not completed yet stay pending
void timers_collect(dsy_ctx* c) {
    size_t keep = 0;
    for (auto& t : c->pending) {
        float ms = 0;
        const hipError_t e = hipEventElapsedTime(&ms, t.a, t.b);
        if (e == hipErrorNotReady) {
            c->pending[keep++] = t;
            continue;
        }
        if (e == hipSuccess) {
            c->time_ms[t.cls] += ms;
            c->launches[t.cls] += 1;
        }
        c->event_pool.push_back(t.a);
        c->event_pool.push_back(t.b);
    }
    c->pending.resize(keep);
}

// entry points fold their timers lazily (hipEventElapsedTime costs host time per event pair); the
// synchronising accessors (dsy_ctx_kernel_time, _synchronize, _reset_timing) fold everything
void timers_collect_lazy(dsy_ctx* c) {
    if (c->pending.size() >= 512) timers_collect(c);
}

int check_family(uint64_t m, uint32_t k, int32_t* kind, uint32_t* chunk) {
    // bloomfilter.py:125-156
    if (m == 0 || m % 8 != 0) return fail(DSY_EINVAL, "size must be a positive multiple of eight (%llu)", (unsigned long long)m);
    if (k == 0 || k > m) return fail(DSY_EINVAL, "0 < k <= m violated (k=%u, m=%llu)", k, (unsigned long long)m);
    uint32_t c = m >= (1ull << 31) ? 8 : (m >= (1ull << 15) ? 4 : 2);
    uint64_t bits = (uint64_t)c * k * 8;
    if (bits > 512) return fail(DSY_EINVAL, "Combining multiple hashfunctions is not implemented, cannot create a hash for %llu bits", (unsigned long long)bits);
    int32_t kd = bits > 384 ? DSY_SHA512 : bits > 256 ? DSY_SHA384 : bits > 160 ? DSY_SHA256 : bits > 128 ? DSY_SHA1 : DSY_MD5;
    *kind = kd;
    *chunk = c;
    return DSY_OK;
}

int check_params(const dsy_bloom_params* p) {
    if (!p) return fail(DSY_EINVAL, "params is NULL");
    int32_t kind;
    uint32_t chunk;
    int rc = check_family(p->m_bits, p->k, &kind, &chunk);
    if (rc) return rc;
    if (kind != p->hash_kind || chunk != p->chunk_bytes)
        return fail(DSY_EINVAL, "hash_kind/chunk (%d/%u) disagree with bloomfilter.py for m=%llu k=%u (%d/%u)", p->hash_kind,
                    p->chunk_bytes, (unsigned long long)p->m_bits, p->k, kind, chunk);
    if (p->prefix_len > 255) return fail(DSY_EINVAL, "prefix too long (%u)", p->prefix_len);
    return DSY_OK;
}

uint64_t filter_words(uint64_t m) { return (m + 31) / 32; }

// batches of at least this many keys are hashed in length-bucketed order
const uint64_t kLenSortMin = 1 << 15;

int upload_params(dsy_ctx* c, const dsy_bloom_params* p, DevParams** out) {
    DevParams hp{};
    hp.m_bits = p->m_bits;
    hp.k = p->k;
    hp.prefix_len = p->prefix_len;
    std::memcpy(hp.prefix, p->prefix, p->prefix_len);
    void* d;
    int rc = ws_get(c, "params", sizeof(DevParams), &d);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(d, &hp, sizeof hp, hipMemcpyHostToDevice, c->stream));
    *out = (DevParams*)d;
    return DSY_OK;
}

int check_offsets(const uint64_t* offsets, uint64_t n, uint64_t blob_len) {
    if (!offsets) return fail(DSY_EINVAL, "offsets is NULL");
    for (uint64_t i = 0; i < n; ++i) {
        if (offsets[i + 1] < offsets[i]) return fail(DSY_EINVAL, "offsets not monotone at %llu", (unsigned long long)i);
        if (offsets[i + 1] - offsets[i] > 0xffffffffull) return fail(DSY_EINVAL, "key %llu longer than 4 GiB", (unsigned long long)i);
    }
    if (offsets[n] > blob_len) return fail(DSY_EINVAL, "offsets[n]=%llu beyond blob_len=%llu", (unsigned long long)offsets[n], (unsigned long long)blob_len);
    return DSY_OK;
}

// stage a packed key set (blob + offsets) into the workspace, with the read guard after the blob
int stage_keys(dsy_ctx* c, const uint8_t* blob, uint64_t blob_len, const uint64_t* offsets, uint64_t n,
               uint8_t** d_blob, uint64_t** d_off) {
    int rc = check_offsets(offsets, n, blob_len);
    if (rc) return rc;
    void *b, *o;
    if ((rc = ws_get(c, "keys_blob", blob_len + 2 * DSY_BLOB_GUARD, &b))) return rc;
    if ((rc = ws_get(c, "keys_off", (n + 1) * 8, &o))) return rc;
    HIP_TRY(hipMemsetAsync(b, 0, DSY_BLOB_GUARD, c->stream));
    b = (uint8_t*)b + DSY_BLOB_GUARD;  // the kernels may read a few bytes before the first key and a block past the last
    if (blob_len) HIP_TRY(hipMemcpyAsync(b, blob, blob_len, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemsetAsync((uint8_t*)b + blob_len, 0, DSY_BLOB_GUARD, c->stream));
    HIP_TRY(hipMemcpyAsync(o, offsets, (n + 1) * 8, hipMemcpyHostToDevice, c->stream));
    *d_blob = (uint8_t*)b;
    *d_off = (uint64_t*)o;
    return DSY_OK;
}

int run_bloom(dsy_ctx* c, BloomOp op, const dsy_bloom_params* p, const uint8_t* d_blob, const uint64_t* d_off,
              const uint64_t* d_rows, uint64_t n, uint32_t* d_filter, uint8_t* d_present, uint64_t* d_idx,
              const RowRec* d_rec = nullptr) {
    DevParams* dp;
    int rc = upload_params(c, p, &dp);
    if (rc) return rc;
    if (n == 0) return DSY_OK;
    BloomLaunch L{};
    L.op = op;
    L.kind = p->hash_kind;
    L.chunk = p->chunk_bytes;
    L.prm = dp;
    L.prm_prefix_len = p->prefix_len;
    L.blob = d_blob;
    L.offsets = d_off;
    L.rows = d_rows;
    L.rec = d_rec;
    L.n = n;
    L.filter = d_filter;
    L.nwords = (uint32_t)filter_words(p->m_bits);
    L.use_lds = (uint64_t)L.nwords * 4 <= 64 * 1024;
    L.present = d_present;
    L.indices = d_idx;
    // 16 workgroups per CU for the hashing kernels (same-box A/B over 10 M keys, grid 1024 / 1536 / 2048 / 4096 /
    // 8192 / 16384: MD5 test 2.39-2.42 / 2.38-2.42 / 2.38-2.40 / 2.34-2.37 / 2.36-2.38 / 2.40 ms, SHA-1 within 1 % of
    // 4096 from 4096 up; profiles/ab_bloom_grid_r2.json)
    L.max_grid = c->bloom_grid ? c->bloom_grid : 2 * c->max_grid;
    L.stream = c->stream;
    L.diag = c->bloom_diag;
    L.or_mode = c->or_mode;
    L.line_kinds = c->bloom_lines;
    // Large batches hash in length-bucketed order (a wave's 64 lanes then run the same number of blocks); the
    // sort costs ~40 B of traffic per key next to the key bytes themselves.
    if (op != BloomOp::Indices && n >= kLenSortMin) {
        void *bins, *tasks;
        int rc2;
        if ((rc2 = ws_get(c, "len_bins", kLenSortBins * 4, &bins))) return rc2;
        if ((rc2 = ws_get(c, "len_tasks", n * sizeof(PairTask), &tasks))) return rc2;
        const bool wide = p->hash_kind >= DSY_SHA384;
        LenSort ls{p->prefix_len, wide ? 128u : 64u, wide ? 16u : 8u};
        if (bloom_staging(L) == 2) {  // the line-staged hashing's lanes run line stages, not blocks
            ls.line_mode = 1;
            ls.base_lo = (uint32_t)(uintptr_t)d_blob & 127u;
        }
        HIP_TRY(launch_len_sort(ls, d_off, d_rows, d_rec, n, (uint32_t*)bins, (PairTask*)tasks, c->max_grid, c->stream));
        L.tasks = (const PairTask*)tasks;
    }
    PendingTimer t;
    timer_dispatch(c, &t, kTimeBuild, &L.ev_start, &L.ev_stop);
    HIP_TRY(launch_bloom(L));
    timer_dispatched(c, &t);
    return DSY_OK;
}

// the simulator's accumulators: [kSimTestedSlots][4] work (build blocks, build slots, respond blocks, respond slots),
// [kSimTestedSlots] pairs tested, then the response-overflow flag
constexpr size_t kSimAccWork = 32 * kSimTestedSlots, kSimAccTested = 8 * kSimTestedSlots;
constexpr size_t kSimAccBytes = kSimAccWork + kSimAccTested + 16;

int sim_acc_get(dsy_ctx* c, uint8_t** out) {
    bool fresh = false;
    void* d;
    int rc = ws_get(c, "sim_acc", kSimAccBytes, &d, &fresh);
    if (rc) return rc;
    if (fresh) HIP_TRY(hipMemsetAsync(d, 0, kSimAccBytes, c->stream));
    c->sim_acc = d;
    c->sim_pending = true;
    *out = (uint8_t*)d;
    return DSY_OK;
}

// fold the simulator's device counters into the ctx totals (the stream must be idle)
int sim_collect(dsy_ctx* c) {
    if (!c->sim_pending || !c->sim_acc) return DSY_OK;
    std::vector<uint64_t> h(kSimAccBytes / 8);
    HIP_TRY(hipMemcpy(h.data(), c->sim_acc, kSimAccBytes, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < kSimTestedSlots; ++i) {
        c->blocks[kTimeSimBuild] += h[4 * i];
        c->slots[kTimeSimBuild] += h[4 * i + 1];
        c->blocks[kTimeSimRespond] += h[4 * i + 2];
        c->slots[kTimeSimRespond] += h[4 * i + 3];
        c->useful[kTimeSimRespond] += h[kSimAccWork / 8 + i];
    }
    if (h[(kSimAccWork + kSimAccTested) / 8]) c->sim_overflow = true;
    HIP_TRY(hipMemsetAsync(c->sim_acc, 0, kSimAccBytes, c->stream));
    c->sim_pending = false;
    return DSY_OK;
}

struct Guard {
    dsy_ctx* c;
    explicit Guard(dsy_ctx* c) : c(c) { c->mu.lock(); hipSetDevice(c->device); }
    ~Guard() { c->mu.unlock(); }
};

}  // namespace

extern "C" {

int dsy_abi_version(void) { return DSY_ABI_VERSION; }
const char* dsy_last_error(void) { return g_err.c_str(); }
uint64_t dsy_filter_words(uint64_t m_bits) { return filter_words(m_bits); }

int dsy_hash_family(uint64_t m_bits, uint32_t k, int32_t* out_kind, uint32_t* out_chunk) {
    int32_t kind;
    uint32_t chunk;
    int rc = check_family(m_bits, k, &kind, &chunk);
    if (rc) return rc;
    if (out_kind) *out_kind = kind;
    if (out_chunk) *out_chunk = chunk;
    return DSY_OK;
}

int dsy_ctx_create(int device, dsy_ctx** out) {
    if (!out) return fail(DSY_EINVAL, "out is NULL");
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(DSY_EINVAL, "device %d out of range (%d devices)", device, ndev);
    HIP_TRY(hipSetDevice(device));
    dsy_ctx* c = new dsy_ctx();
    c->device = device;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return fail(DSY_EHIP, "hipStreamCreate: %s", hipGetErrorString(e));
    }
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    c->max_grid = (uint32_t)std::max(cus, 1) * 8;
    if (const char* v = getenv("DSY_BLOOM_DIAG")) c->bloom_diag = atoi(v);
    if (const char* v = getenv("DSY_PAIR_DIAG")) c->pair_diag = atoi(v);
    if (const char* v = getenv("DSY_OR_MODE")) c->or_mode = atoi(v);
    if (const char* v = getenv("DSY_BLOOM_LINES")) c->bloom_lines = (uint32_t)strtoul(v, nullptr, 0);
    if (const char* v = getenv("DSY_PAIR_GRID")) c->pair_grid = (uint32_t)atoi(v);
    if (const char* v = getenv("DSY_BLOOM_GRID")) c->bloom_grid = (uint32_t)atoi(v);
    if (const char* v = getenv("DSY_POOL")) c->pool_kinds = (uint32_t)strtoul(v, nullptr, 0);
    if (const char* v = getenv("DSY_POOL_QUEUE")) c->pool_queue = atoi(v);
    if (const char* v = getenv("DSY_POOL_DEAL")) c->pool_deal = atoi(v);
    {  // diagnostics, process-wide: every ctx creation sets it (0 without the variable)
        const char* v = getenv("DSY_FILL_SKEW");
        set_fill_skew(v ? (uint32_t)strtoul(v, nullptr, 0) : 0u);
    }
    if (const char* v = getenv("DSY_POOL_SCAN")) c->pool_scan = atoi(v);
    if (const char* v = getenv("DSY_PAIR_PRIO")) c->pair_prio = atoi(v);
    if (const char* v = getenv("DSY_BULK_ZERO")) c->bulk_zero = atoi(v);
    if (const char* v = getenv("DSY_PAIR_DIRECT")) c->direct_kinds = (uint32_t)strtoul(v, nullptr, 0);
    c->pool_kinds &= (1u << DSY_MD5) | (1u << DSY_SHA1) | (1u << DSY_SHA256);
    hipHostMalloc(&c->pinned, 4096, hipHostMallocDefault);
    *out = c;
    return DSY_OK;
}

int dsy_ctx_destroy(dsy_ctx* c) {
    if (!c) return DSY_OK;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        hipSetDevice(c->device);
        hipStreamSynchronize(c->stream);
        timers_collect(c);
        for (auto& sl : c->rs) {
            if (sl.ev_done) hipEventDestroy(sl.ev_done);
            sl.w.release();
        }
        c->main.release();
        for (auto e : c->event_pool) hipEventDestroy(e);
        if (c->xev) hipEventDestroy(c->xev);
        if (c->aux) hipStreamDestroy(c->aux);
        if (c->gev) hipEventDestroy(c->gev);
        if (c->out_pin) hipHostFree(c->out_pin);
        if (c->pinned) hipHostFree(c->pinned);
        if (c->in_stage) hipHostFree(c->in_stage);
        if (c->flush_pin) hipHostFree(c->flush_pin);
        hipStreamDestroy(c->stream);
    }
    delete c;
    return DSY_OK;
}

int dsy_ctx_synchronize(dsy_ctx* c) {
    if (!c) return fail(DSY_EINVAL, "ctx is NULL");
    Guard g(c);
    HIP_TRY(hipStreamSynchronize(c->stream));
    timers_collect(c);
    return sim_collect(c);
}

void* dsy_ctx_stream(dsy_ctx* c) { return c ? (void*)c->stream : nullptr; }

static int xev_get(dsy_ctx* c) {
    if (!c->xev) HIP_TRY(hipEventCreateWithFlags(&c->xev, hipEventDisableTiming));
    return DSY_OK;
}

int dsy_ctx_wait_stream(dsy_ctx* c, void* stream) {
    if (!c) return fail(DSY_EINVAL, "ctx is NULL");
    Guard g(c);
    int rc = xev_get(c);
    if (rc) return rc;
    HIP_TRY(hipEventRecord(c->xev, (hipStream_t)stream));
    HIP_TRY(hipStreamWaitEvent(c->stream, c->xev, 0));
    return DSY_OK;
}

int dsy_ctx_wait_event(dsy_ctx* c, void* event) {
    if (!c || !event) return fail(DSY_EINVAL, "NULL argument");
    Guard g(c);
    HIP_TRY(hipStreamWaitEvent(c->stream, (hipEvent_t)event, 0));
    return DSY_OK;
}

int dsy_ctx_signal_stream(dsy_ctx* c, void* stream) {
    if (!c) return fail(DSY_EINVAL, "ctx is NULL");
    Guard g(c);
    int rc = xev_get(c);
    if (rc) return rc;
    HIP_TRY(hipEventRecord(c->xev, c->stream));
    HIP_TRY(hipStreamWaitEvent((hipStream_t)stream, c->xev, 0));
    return DSY_OK;
}

int dsy_ctx_set_timing(dsy_ctx* c, int enable) {
    if (!c) return fail(DSY_EINVAL, "ctx is NULL");
    Guard g(c);
    c->timing = (enable & 0x100) ? (uint32_t)(enable & 0xff) : enable ? 0xffu : 0u;
    return DSY_OK;
}

int dsy_ctx_kernel_time(dsy_ctx* c, int which, double* out_ms, uint64_t* out_launches, uint64_t* out_blocks,
                        uint64_t* out_bytes) {
    if (!c || which < 0 || which >= kTimeClasses) return fail(DSY_EINVAL, "bad ctx or timer class");
    Guard g(c);
    HIP_TRY(hipStreamSynchronize(c->stream));
    timers_collect(c);
    int rc = sim_collect(c);
    if (rc) return rc;
    if (out_ms) *out_ms = c->time_ms[which];
    if (out_launches) *out_launches = c->launches[which];
    if (out_blocks) *out_blocks = c->blocks[which];
    if (out_bytes) *out_bytes = c->bytes[which];
    return DSY_OK;
}

int dsy_ctx_reset_timing(dsy_ctx* c) {
    if (!c) return fail(DSY_EINVAL, "ctx is NULL");
    Guard g(c);
    HIP_TRY(hipStreamSynchronize(c->stream));
    timers_collect(c);
    int rc = sim_collect(c);
    if (rc) return rc;
    for (int i = 0; i < kTimeClasses; ++i)
        c->time_ms[i] = 0, c->launches[i] = 0, c->blocks[i] = 0, c->bytes[i] = 0, c->useful[i] = 0, c->slots[i] = 0;
    return DSY_OK;
}

int dsy_ctx_set_window(dsy_ctx* c, uint64_t max_pairs) {
    if (!c || (max_pairs && (max_pairs < 64 || max_pairs % 64))) return fail(DSY_EINVAL, "window must be 0 or a multiple of 64");
    Guard g(c);
    c->window_cap = max_pairs;
    return DSY_OK;
}

int dsy_ctx_work(dsy_ctx* c, int which, uint64_t* out4) {
    if (!c || !out4 || which < 0 || which >= kTimeClasses) return fail(DSY_EINVAL, "bad ctx, output or class");
    Guard g(c);
    if (c->sim_pending) {  // the simulator's counters live on the device until the stream is idle
        HIP_TRY(hipStreamSynchronize(c->stream));
        int rc = sim_collect(c);
        if (rc) return rc;
    }
    out4[0] = c->blocks[which];
    out4[1] = c->bytes[which];
    out4[2] = c->useful[which];
    out4[3] = c->slots[which];
    return DSY_OK;
}

// ------------------------------------------------------------------------------------------ bloom ops
int dsy_bloom_add(dsy_ctx* c, const dsy_bloom_params* p, const uint8_t* blob, uint64_t blob_len,
                  const uint64_t* offsets, uint64_t n, uint8_t* filter_inout) {
    if (!c || !filter_inout) return fail(DSY_EINVAL, "NULL ctx or filter");
    int rc = check_params(p);
    if (rc) return rc;
    Guard g(c);
    uint8_t* db;
    uint64_t* dof;
    if ((rc = stage_keys(c, blob, blob_len, offsets, n, &db, &dof))) return rc;
    const uint64_t nbytes = p->m_bits / 8, words = filter_words(p->m_bits);
    void* df;
    if ((rc = ws_get(c, "filter", words * 4, &df))) return rc;
    HIP_TRY(hipMemsetAsync(df, 0, words * 4, c->stream));
    HIP_TRY(hipMemcpyAsync(df, filter_inout, nbytes, hipMemcpyHostToDevice, c->stream));
    if ((rc = run_bloom(c, BloomOp::Add, p, db, dof, nullptr, n, (uint32_t*)df, nullptr, nullptr))) return rc;
    HIP_TRY(hipMemcpyAsync(filter_inout, df, nbytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    timers_collect_lazy(c);
    return DSY_OK;
}

int dsy_bloom_test(dsy_ctx* c, const dsy_bloom_params* p, const uint8_t* blob, uint64_t blob_len,
                   const uint64_t* offsets, uint64_t n, const uint8_t* filter, uint8_t* out_present) {
    if (!c || !filter || (!out_present && n)) return fail(DSY_EINVAL, "NULL ctx, filter or output");
    int rc = check_params(p);
    if (rc) return rc;
    Guard g(c);
    uint8_t* db;
    uint64_t* dof;
    if ((rc = stage_keys(c, blob, blob_len, offsets, n, &db, &dof))) return rc;
    const uint64_t nbytes = p->m_bits / 8, words = filter_words(p->m_bits);
    void *df, *dp;
    if ((rc = ws_get(c, "filter", words * 4, &df))) return rc;
    if ((rc = ws_get(c, "present", n + 1, &dp))) return rc;
    HIP_TRY(hipMemsetAsync(df, 0, words * 4, c->stream));
    HIP_TRY(hipMemcpyAsync(df, filter, nbytes, hipMemcpyHostToDevice, c->stream));
    if ((rc = run_bloom(c, BloomOp::Test, p, db, dof, nullptr, n, (uint32_t*)df, (uint8_t*)dp, nullptr))) return rc;
    if (n) HIP_TRY(hipMemcpyAsync(out_present, dp, n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    timers_collect_lazy(c);
    return DSY_OK;
}

int dsy_bloom_indices(dsy_ctx* c, const dsy_bloom_params* p, const uint8_t* blob, uint64_t blob_len,
                      const uint64_t* offsets, uint64_t n, uint64_t* out_idx) {
    if (!c || (!out_idx && n)) return fail(DSY_EINVAL, "NULL ctx or output");
    int rc = check_params(p);
    if (rc) return rc;
    Guard g(c);
    uint8_t* db;
    uint64_t* dof;
    if ((rc = stage_keys(c, blob, blob_len, offsets, n, &db, &dof))) return rc;
    void* di;
    if ((rc = ws_get(c, "indices", (n * p->k + 1) * 8, &di))) return rc;
    if ((rc = run_bloom(c, BloomOp::Indices, p, db, dof, nullptr, n, nullptr, nullptr, (uint64_t*)di))) return rc;
    if (n) HIP_TRY(hipMemcpyAsync(out_idx, di, n * p->k * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    timers_collect_lazy(c);
    return DSY_OK;
}

int dsy_bloom_add_dev(dsy_ctx* c, const dsy_bloom_params* p, const uint8_t* d_blob, const uint64_t* d_offsets,
                      uint64_t n, uint32_t* d_filter) {
    if (!c || !d_filter) return fail(DSY_EINVAL, "NULL ctx or filter");
    int rc = check_params(p);
    if (rc) return rc;
    Guard g(c);
    return run_bloom(c, BloomOp::Add, p, d_blob, d_offsets, nullptr, n, d_filter, nullptr, nullptr);
}

int dsy_bloom_test_dev(dsy_ctx* c, const dsy_bloom_params* p, const uint8_t* d_blob, const uint64_t* d_offsets,
                       uint64_t n, const uint32_t* d_filter, uint8_t* d_present) {
    if (!c || !d_filter) return fail(DSY_EINVAL, "NULL ctx or filter");
    int rc = check_params(p);
    if (rc) return rc;
    Guard g(c);
    return run_bloom(c, BloomOp::Test, p, d_blob, d_offsets, nullptr, n, (uint32_t*)d_filter, d_present, nullptr);
}

int dsy_filter_or_reduce(dsy_ctx* c, const uint32_t* d_parts, uint32_t n_parts, uint64_t words, uint32_t* d_out) {
    if (!c || !d_out || (n_parts && !d_parts) || !n_parts) return fail(DSY_EINVAL, "NULL argument or no parts");
    Guard g(c);
    HIP_TRY(launch_or_reduce(d_parts, n_parts, words, d_out, c->max_grid, c->stream));
    return DSY_OK;
}

// ------------------------------------------------------------------------------------------------ store
static int store_index(dsy_store* s, const uint64_t* offsets, const uint64_t* gt, const uint32_t* meta,
                       const uint8_t* undone, std::vector<uint64_t>* live_gt, std::vector<uint64_t>* live_row,
                       bool* identity) {
    // Build the live index (undone == 0) and the per-meta segments; check the (meta, global_time) order the
    // export promises (the sync_meta_message_undone_global_time_index order, dispersydatabase.py:63).
    const uint64_t n = s->n;
    *identity = true;
    uint64_t minlen = ~0ull, maxlen = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (i && (meta[i] < meta[i - 1] || (meta[i] == meta[i - 1] && gt[i] < gt[i - 1])))
            return fail(DSY_EUNSORTED, "store rows not sorted by (meta, global_time) at row %llu", (unsigned long long)i);
        minlen = std::min(minlen, offsets[i + 1] - offsets[i]);
        maxlen = std::max(maxlen, offsets[i + 1] - offsets[i]);
        if (undone && undone[i]) *identity = false;
    }
    s->min_len = n ? minlen : 0;
    s->max_len = maxlen;
    if (!*identity) {
        live_gt->reserve(n);
        live_row->reserve(n);
    }
    uint64_t li = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (undone && undone[i]) continue;
        auto it = s->segs.find(meta[i]);
        if (it == s->segs.end()) s->segs[meta[i]] = {li, li + 1};
        else it->second.second = li + 1;
        if (!*identity) {
            live_gt->push_back(gt[i]);
            live_row->push_back(i);
        }
        ++li;
    }
    s->n_live = li;
    s->n_phys = li;
    return DSY_OK;
}

static int store_finish(dsy_ctx* c, dsy_store* s, const uint64_t* h_gt_or_null, const uint64_t* d_gt,
                        std::vector<uint64_t>& live_gt, std::vector<uint64_t>& live_row, bool identity) {
    if (identity) {
        if (d_gt) {
            s->d_live_gt = d_gt;
        } else {
            void* p;
            if (hipMalloc(&p, std::max<uint64_t>(s->n, 1) * 8) != hipSuccess) return fail(DSY_ENOMEM, "store gt alloc");
            s->owned.push_back(p);
            if (s->n) HIP_TRY(hipMemcpyAsync(p, h_gt_or_null, s->n * 8, hipMemcpyHostToDevice, c->stream));
            s->d_live_gt = (uint64_t*)p;
        }
        s->d_live_row = nullptr;
    } else {
        void *pg, *pr;
        if (hipMalloc(&pg, std::max<uint64_t>(s->n_live, 1) * 8) != hipSuccess) return fail(DSY_ENOMEM, "store live alloc");
        s->owned.push_back(pg);
        if (hipMalloc(&pr, std::max<uint64_t>(s->n_live, 1) * 8) != hipSuccess) return fail(DSY_ENOMEM, "store live alloc");
        s->owned.push_back(pr);
        if (s->n_live) {
            HIP_TRY(hipMemcpyAsync(pg, live_gt.data(), s->n_live * 8, hipMemcpyHostToDevice, c->stream));
            HIP_TRY(hipMemcpyAsync(pr, live_row.data(), s->n_live * 8, hipMemcpyHostToDevice, c->stream));
        }
        s->d_live_gt = (uint64_t*)pg;
        s->d_live_row = (uint64_t*)pr;
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    return DSY_OK;
}

// The responder's line copy: row i's packet at rec[i].off, kLineBias bytes past a multiple of 128, so every LDS-DMA
// piece of the hashing kernel is one whole line and a 1-byte-prefixed message is line-aligned (dsy_message.h
// hash_key_dma_lines); 0x80 and zeros after the packet up to its padded message's bit length (line_bytes_for).
// Costs < 192 bytes per row.
static int store_build_lines(dsy_ctx* c, dsy_store* s, const uint64_t* h_off) {
    const uint64_t n = s->n;
    std::vector<RowRec> rec(std::max<uint64_t>(n, 1));
    uint64_t at = DSY_BLOB_GUARD;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t len = h_off[i + 1] - h_off[i];
        rec[i] = RowRec{at + kLineBias, (uint32_t)len, 0u};
        at += line_bytes_for(len);
    }
    const uint64_t bytes = at + DSY_BLOB_GUARD;
    void *pl, *pr;
    if (hipMalloc(&pl, bytes) != hipSuccess) return fail(DSY_ENOMEM, "store line copy alloc (%llu B)", (unsigned long long)bytes);
    s->owned.push_back(pl);
    if (hipMalloc(&pr, rec.size() * sizeof(RowRec)) != hipSuccess) return fail(DSY_ENOMEM, "store row records alloc");
    s->owned.push_back(pr);
    HIP_TRY(hipMemsetAsync(pl, 0, bytes, c->stream));
    HIP_TRY(hipMemcpyAsync(pr, rec.data(), rec.size() * sizeof(RowRec), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(launch_store_lines(s->d_blob, s->d_offsets, (const RowRec*)pr, n, (uint8_t*)pl, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    s->d_lines = (const uint8_t*)pl;
    s->d_rec = (const RowRec*)pr;
    s->lines_used = at;
    s->lines_cap = bytes;
    s->rec_cap = rec.size();
    return DSY_OK;
}

// The packed blob/offsets only feed the line copy; free them when they are ours.
static void store_release_raw(dsy_store* s) {
    if (s->d_blob) {
        auto it = std::find(s->owned.begin(), s->owned.end(), (const void*)(s->d_blob - DSY_BLOB_GUARD));
        if (it != s->owned.end()) { hipFree(*it); s->owned.erase(it); }
    }
    if (s->d_offsets) {
        auto it = std::find(s->owned.begin(), s->owned.end(), (const void*)s->d_offsets);
        if (it != s->owned.end()) { hipFree(*it); s->owned.erase(it); }
    }
    s->d_blob = nullptr;
    s->d_offsets = nullptr;
}

int dsy_store_upload(dsy_ctx* c, const uint8_t* blob, uint64_t blob_len, const uint64_t* offsets, uint64_t n,
                     const uint64_t* global_time, const uint32_t* meta, const uint8_t* undone, dsy_store** out) {
    if (!c || !out || !offsets || (n && (!global_time || !meta))) return fail(DSY_EINVAL, "NULL argument");
    int rc = check_offsets(offsets, n, blob_len);
    if (rc) return rc;
    Guard g(c);
    dsy_store* s = new dsy_store();
    s->ctx = c;
    s->n = n;
    s->blob_len = blob_len;
    std::vector<uint64_t> lg, lr;
    bool identity;
    if ((rc = store_index(s, offsets, global_time, meta, undone, &lg, &lr, &identity))) { delete s; return rc; }
    void *pb, *po;
    if (hipMalloc(&pb, blob_len + 2 * DSY_BLOB_GUARD) != hipSuccess) { delete s; return fail(DSY_ENOMEM, "store blob alloc (%llu B)", (unsigned long long)blob_len); }
    s->owned.push_back(pb);
    HIP_TRY(hipMemsetAsync(pb, 0, DSY_BLOB_GUARD, c->stream));
    pb = (uint8_t*)pb + DSY_BLOB_GUARD;
    if (hipMalloc(&po, (n + 1) * 8) != hipSuccess) { dsy_store_free(s); return fail(DSY_ENOMEM, "store offsets alloc"); }
    s->owned.push_back(po);
    if (blob_len) HIP_TRY(hipMemcpyAsync(pb, blob, blob_len, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemsetAsync((uint8_t*)pb + blob_len, 0, DSY_BLOB_GUARD, c->stream));
    HIP_TRY(hipMemcpyAsync(po, offsets, (n + 1) * 8, hipMemcpyHostToDevice, c->stream));
    s->d_blob = (uint8_t*)pb;
    s->d_offsets = (uint64_t*)po;
    if ((rc = store_finish(c, s, global_time, nullptr, lg, lr, identity))) { dsy_store_free(s); return rc; }
    if ((rc = store_build_lines(c, s, offsets))) { dsy_store_free(s); return rc; }
    // every kernel reads the packets from the line copy from here on: the packed upload is not kept
    store_release_raw(s);
    *out = s;
    return DSY_OK;
}

int dsy_store_attach(dsy_ctx* c, const uint8_t* d_blob, uint64_t blob_len, const uint64_t* d_offsets, uint64_t n,
                     const uint64_t* d_global_time, const uint32_t* d_meta, const uint8_t* d_undone, dsy_store** out) {
    if (!c || !out || !d_offsets || (n && (!d_global_time || !d_meta || !d_blob))) return fail(DSY_EINVAL, "NULL argument");
    Guard g(c);
    std::vector<uint64_t> off(n + 1), gt(n);
    std::vector<uint32_t> meta(n);
    std::vector<uint8_t> und;
    HIP_TRY(hipMemcpy(off.data(), d_offsets, (n + 1) * 8, hipMemcpyDeviceToHost));
    if (n) {
        HIP_TRY(hipMemcpy(gt.data(), d_global_time, n * 8, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(meta.data(), d_meta, n * 4, hipMemcpyDeviceToHost));
        if (d_undone) {
            und.resize(n);
            HIP_TRY(hipMemcpy(und.data(), d_undone, n, hipMemcpyDeviceToHost));
        }
    }
    int rc = check_offsets(off.data(), n, blob_len);
    if (rc) return rc;
    dsy_store* s = new dsy_store();
    s->ctx = c;
    s->n = n;
    s->blob_len = blob_len;
    s->d_blob = d_blob;
    s->d_offsets = d_offsets;
    std::vector<uint64_t> lg, lr;
    bool identity;
    if ((rc = store_index(s, off.data(), gt.data(), meta.data(), d_undone ? und.data() : nullptr, &lg, &lr, &identity))) {
        delete s;
        return rc;
    }
    if ((rc = store_finish(c, s, nullptr, d_global_time, lg, lr, identity))) { dsy_store_free(s); return rc; }
    if ((rc = store_build_lines(c, s, off.data()))) { dsy_store_free(s); return rc; }
    store_release_raw(s);  // the caller's buffers: no longer read
    *out = s;
    return DSY_OK;
}

int dsy_store_free(dsy_store* s) {
    if (!s) return DSY_OK;
    if (s->ctx) {
        std::lock_guard<std::mutex> lk(s->ctx->mu);
        if (s->ctx->inflight()) return fail(DSY_EINVAL, "the store cannot be freed while submitted responder batches are in flight");
        hipSetDevice(s->ctx->device);
        hipStreamSynchronize(s->ctx->stream);
        for (void* p : s->owned) hipFree(p);
    }
    delete s;
    return DSY_OK;
}

uint64_t dsy_store_rows(const dsy_store* s) { return s ? s->n : 0; }

// ------------------------------------------------------------------------------------------------ ingest
namespace {

void store_release(dsy_store* s, const void* p) {
    auto it = std::find(s->owned.begin(), s->owned.end(), p);
    if (it == s->owned.end()) return;  // a caller's buffer (dsy_store_attach): not ours to free
    hipFree(*it);
    s->owned.erase(it);
}

uint64_t grown(uint64_t need, uint64_t have) { return std::max<uint64_t>(need, have + have / 4 + 4096); }

// make room for the line copy to reach `at` bytes (its tail guard after); zero the bytes past what is in use
int lines_reserve(dsy_ctx* c, dsy_store* s, uint64_t at) {
    if (at + DSY_BLOB_GUARD > s->lines_cap) {
        const uint64_t cap = grown(at + DSY_BLOB_GUARD, s->lines_cap);
        void* nl;
        if (hipMalloc(&nl, cap) != hipSuccess) return fail(DSY_ENOMEM, "store line copy growth (%llu B)", (unsigned long long)cap);
        HIP_TRY(hipMemcpyAsync(nl, s->d_lines, s->lines_used, hipMemcpyDeviceToDevice, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        store_release(s, s->d_lines);
        s->owned.push_back(nl);
        s->d_lines = (const uint8_t*)nl;
        s->lines_cap = cap;
    }
    HIP_TRY(hipMemsetAsync(const_cast<uint8_t*>(s->d_lines) + s->lines_used, 0, at + DSY_BLOB_GUARD - s->lines_used,
                           c->stream));
    return DSY_OK;
}

// keep the (member, global_time) table at most half full: a power-of-two capacity, rehashed on growth
int dup_reserve(dsy_ctx* c, dsy_store* s, uint64_t count) {
    if (s->dup && count * 2 <= s->dup_cap) return DSY_OK;
    uint64_t cap = 1024;
    while (cap < count * 2) cap <<= 1;
    void* nt;
    if (hipMalloc(&nt, cap * sizeof(DupSlot)) != hipSuccess) return fail(DSY_ENOMEM, "duplicate table (%llu slots)", (unsigned long long)cap);
    s->owned.push_back(nt);
    HIP_TRY(hipMemsetAsync(nt, 0xff, cap * sizeof(DupSlot), c->stream));
    if (s->dup) {
        HIP_TRY(launch_dup_rehash(s->dup, s->dup_cap, (DupSlot*)nt, cap - 1, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        store_release(s, s->dup);
    }
    s->dup = (DupSlot*)nt;
    s->dup_cap = cap;
    return DSY_OK;
}

// insert rows first_row .. first_row+n-1 of the given (member, global_time) host arrays into the table
// (member, global_time) keys of rows first_row .. first_row+n-1 into the table, from device columns (stream-ordered)
int dup_insert_dev(dsy_ctx* c, dsy_store* s, const uint64_t* d_member, const uint64_t* d_gt, uint64_t first_row,
                   uint64_t n) {
    int rc;
    if (!n) return DSY_OK;
    if ((rc = dup_reserve(c, s, s->dup_count + n))) return rc;
    if (first_row + n > s->keys_cap) {
        const uint64_t cap = grown(first_row + n, s->keys_cap);
        void* nk;
        if (hipMalloc(&nk, cap * sizeof(DupKey)) != hipSuccess) return fail(DSY_ENOMEM, "row keys (%llu rows)", (unsigned long long)cap);
        if (s->dup_keys && first_row) HIP_TRY(hipMemcpyAsync(nk, s->dup_keys, first_row * sizeof(DupKey), hipMemcpyDeviceToDevice, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        store_release(s, s->dup_keys);
        s->owned.push_back(nk);
        s->dup_keys = (DupKey*)nk;
        s->keys_cap = cap;
    }
    HIP_TRY(launch_dup_insert(d_member, d_gt, first_row, n, s->dup, s->dup_cap - 1, s->dup_keys, c->stream));
    s->dup_count += n;
    return DSY_OK;
}

// the same from host columns
int dup_insert(dsy_ctx* c, dsy_store* s, const uint64_t* member, const uint64_t* gt, uint64_t first_row, uint64_t n) {
    int rc;
    if (!n) return DSY_OK;
    void* d;
    if ((rc = ws_get(c, "dup_keys", n * 16, &d))) return rc;
    HIP_TRY(hipMemcpyAsync(d, member, n * 8, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync((uint64_t*)d + n, gt, n * 8, hipMemcpyHostToDevice, c->stream));
    if ((rc = dup_insert_dev(c, s, (const uint64_t*)d, (const uint64_t*)d + n, first_row, n))) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return DSY_OK;
}

}  // namespace

// The live index: per meta, in meta order, a region [a, next meta's a) (the last: [a, n_phys)) holding its live
// entries [a, b) in (global_time, row) order and then slack entries (row kGapRow) that appends fill in place.
static uint64_t region_end(const dsy_store* s, uint32_t meta) {
    uint64_t end = s->n_phys;
    for (auto& e : s->segs)
        if (e.first > meta) end = std::min(end, e.second.first);
    return end;
}

// a meta's live segment, or -- for a meta without one -- the empty segment at its place (the next meta's region start)
static std::pair<uint64_t, uint64_t> seg_or_place(const dsy_store* s, uint32_t meta) {
    auto it = s->segs.find(meta);
    if (it != s->segs.end()) return it->second;
    const uint64_t p = region_end(s, meta);
    return {p, p};
}

static int spare_reserve(dsy_store* s, uint64_t need, uint64_t have) {
    if (s->spare_cap >= need) return DSY_OK;
    // (merges do not wait on the host: an earlier one may still read the buffer pair being replaced)
    if (s->spare_gt || s->spare_row) HIP_TRY(hipStreamSynchronize(s->ctx->stream));
    store_release(s, s->spare_gt);
    store_release(s, s->spare_row);
    s->spare_gt = s->spare_row = nullptr;
    s->spare_cap = 0;
    const uint64_t cap = grown(need, have);
    void *pg, *pr;
    if (hipMalloc(&pg, cap * 8) != hipSuccess) return fail(DSY_ENOMEM, "store live index growth");
    s->owned.push_back(pg);
    if (hipMalloc(&pr, cap * 8) != hipSuccess) { store_release(s, pg); return fail(DSY_ENOMEM, "store live index growth"); }
    s->owned.push_back(pr);
    s->spare_gt = (uint64_t*)pg;
    s->spare_row = (uint64_t*)pr;
    s->spare_cap = cap;
    return DSY_OK;
}

// the spare buffer pair holds the new index: swap (double-buffered -- the previous index becomes the next target)
static void spare_swap(dsy_store* s) {
    uint64_t* prev_gt = const_cast<uint64_t*>(s->d_live_gt);
    uint64_t* prev_row = const_cast<uint64_t*>(s->d_live_row);
    const uint64_t prev_cap = s->live_cap;
    s->d_live_gt = s->spare_gt;
    s->d_live_row = s->spare_row;
    s->live_cap = s->spare_cap;
    if (prev_cap) {  // the index an earlier merge built: the next target
        s->spare_gt = prev_gt;
        s->spare_row = prev_row;
        s->spare_cap = prev_cap;
    } else {         // the index of the upload/attach (possibly the caller's global_time column)
        store_release(s, prev_gt);
        store_release(s, prev_row);
        s->spare_gt = s->spare_row = nullptr;
        s->spare_cap = 0;
    }
}

// Merge `a` entries -- device IngestRows in (meta_message, global_time, row) order; cnt: per meta (live entries, slack
// entries), the slack ones last in their meta and ranked at its region's end -- into the whole index on the device,
// into the spare buffer pair, which then becomes the index.  check_present: fail (index unchanged) when a row is in the
// index already.  Caller holds the ctx lock.
static int live_merge(dsy_ctx* c, dsy_store* s, const IngestRow* d_rows, uint64_t a,
                      const std::map<uint32_t, std::pair<uint64_t, uint64_t>>& cnt, bool check_present) {
    if (!a) return DSY_OK;
    void* d_tmp;
    int rc;
    if ((rc = ws_get(c, "live_merge", a * 8 + 64, &d_tmp))) return rc;
    uint64_t* d_rank = (uint64_t*)d_tmp;
    unsigned int* d_present = (unsigned int*)(d_rank + a);
    if (check_present) HIP_TRY(hipMemsetAsync(d_present, 0, 4, c->stream));
    const uint64_t phys = s->n_phys + a;
    if ((rc = spare_reserve(s, phys, s->n_phys))) return rc;
    HIP_TRY(launch_ingest_merge(s->d_live_gt, s->d_live_row, s->n_phys, d_rows, a, d_rank, s->spare_gt, s->spare_row,
                                check_present ? d_present : nullptr, c->max_grid, c->stream));
    unsigned int present = 0;
    if (check_present) {  // (otherwise no host wait: the index's next reader is stream-ordered behind the merge)
        HIP_TRY(hipMemcpyAsync(&present, d_present, 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    if (present) return fail(DSY_EINVAL, "a row to insert is in the live index already");
    spare_swap(s);
    // segments: a meta's segment moves by every entry of the smaller metas and grows by its own live ones; a meta new
    // to the index starts at its place
    std::map<uint32_t, std::pair<uint64_t, uint64_t>> all;
    for (auto& e : s->segs) all[e.first] = e.second;
    for (auto& m : cnt)
        if (!all.count(m.first)) all[m.first] = seg_or_place(s, m.first);
    uint64_t before = 0, live_add = 0;
    for (auto& e : all) {
        auto own = cnt.find(e.first);
        const uint64_t real = own == cnt.end() ? 0 : own->second.first;
        const uint64_t gap = own == cnt.end() ? 0 : own->second.second;
        s->segs[e.first] = {e.second.first + before, e.second.second + before + real};
        before += real + gap;
        live_add += real;
    }
    s->n_live += live_add;
    s->n_phys = phys;
    s->ix_full += 1;
    s->ix_bytes += 32 * (s->n_phys - a) + 48 * a;  // the old index read and written, the new entries read and written
    return DSY_OK;
}

// New live-index entries given on the host: rows (store positions, any order) with their meta and global time join
// the index at their (meta_message, global_time, row) place -- redone rows (dsy_store_set_undone).  Caller holds the
// ctx lock.
static int live_insert(dsy_ctx* c, dsy_store* s, const uint32_t* meta, const uint64_t* gt, const uint64_t* row,
                       uint64_t a, bool check_present) {
    if (!a) return DSY_OK;
    // the new entries in index order (meta_message, global_time, row)
    std::vector<uint64_t> ord(a);
    for (uint64_t j = 0; j < a; ++j) ord[j] = j;
    std::sort(ord.begin(), ord.end(), [&](uint64_t x, uint64_t y) {
        return meta[x] != meta[y] ? meta[x] < meta[y] : gt[x] != gt[y] ? gt[x] < gt[y] : row[x] < row[y];
    });
    std::vector<IngestRow> rows(a);
    std::map<uint32_t, std::pair<uint64_t, uint64_t>> cnt;
    for (uint64_t t = 0; t < a; ++t) {
        const uint64_t j = ord[t];
        const auto sg = seg_or_place(s, meta[j]);
        rows[t] = IngestRow{gt[j], sg.first, sg.second, row[j]};
        ++cnt[meta[j]].first;
    }
    void* d_rows;
    int rc;
    if ((rc = ws_get(c, "live_insert", a * sizeof(IngestRow), &d_rows))) return rc;
    HIP_TRY(hipMemcpyAsync(d_rows, rows.data(), a * sizeof(IngestRow), hipMemcpyHostToDevice, c->stream));
    return live_merge(c, s, (const IngestRow*)d_rows, a, cnt, check_present);
}

// slack a meta's region gets when the whole index is re-laid out: a quarter of its entries, at least kSlackMin
static constexpr uint64_t kSlackMin = 16384;

// Merge the rows appended since the last read into the live index.  Every reader of the index calls it first; the
// caller holds the ctx lock and nothing is in flight on the store.  The pending (meta, global_time) columns are on the
// device already (dsy_store_append uploads them with the packets) and are put in index order there (two radix sorts,
// launch_pend_order).  When every meta's new entries fit its region's slack, each meta's tail from its first new entry
// on is merged in place -- O(batch + that tail), the common case of new global times at or near the top; otherwise one
// merge of the whole index lays it out again with fresh slack.
// DSY_FLUSH_PROFILE: one stderr line per flush with its phases in microseconds (each phase synchronised: diagnostics)
struct FlushClock {
    bool on;
    hipStream_t st;
    double t0, last;
    char buf[256];
    int at = 0;
    explicit FlushClock(hipStream_t s) : st(s) {
        static const bool env = getenv("DSY_FLUSH_PROFILE") != nullptr;
        on = env;
        t0 = last = on ? now() : 0;
        buf[0] = 0;
    }
    static double now() {
        return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
    }
    void mark(const char* what) {
        if (!on) return;
        hipStreamSynchronize(st);
        const double t = now();
        at += snprintf(buf + at, sizeof(buf) - at > 0 ? sizeof(buf) - at : 0, " %s=%.1f", what, t - last);
        last = t;
    }
    void done(uint64_t P, const char* mode) {
        if (on) fprintf(stderr, "flush_profile P=%llu mode=%s%s total=%.1f\n", (unsigned long long)P, mode, buf, now() - t0);
    }
};

static int store_flush(dsy_ctx* c, const dsy_store* cs) {
    dsy_store* s = const_cast<dsy_store*>(cs);
    const uint64_t P = s->pend_n;
    if (!P) return DSY_OK;
    FlushClock fc(c->stream);
    std::map<uint32_t, uint64_t> cntm(s->pend_cnt.begin(), s->pend_cnt.end());
    for (auto& e : s->segs) cntm.emplace(e.first, 0);
    const uint32_t nm = (uint32_t)cntm.size();
    std::vector<uint32_t> metas;
    std::vector<uint64_t> segs, ends, cnt, starts, gap_before, extra;
    bool fast = s->d_live_row != nullptr;
    uint64_t at = 0, gaps = 0;
    for (auto& m : cntm) {
        const bool known = s->segs.count(m.first) != 0;
        const auto sg = seg_or_place(s, m.first);
        const uint64_t end = region_end(s, m.first);
        metas.push_back(m.first);
        segs.push_back(sg.first);
        segs.push_back(sg.second);
        ends.push_back(end);
        cnt.push_back(m.second);
        starts.push_back(at);
        at += m.second;
        if (m.second && (!known || end - sg.second < m.second)) fast = false;
        const uint64_t live = sg.second - sg.first, want = std::max(kSlackMin, (live + m.second) / 4);
        const uint64_t slack = known ? end - sg.second : 0;
        extra.push_back((live || m.second) && want > slack ? want - slack : 0);
        gap_before.push_back(gaps);
        gaps += extra.back();
    }
    // 256-byte aligned parts: the metas | segments | gap_before | starts | counts | first ranks | the ordered rows (with
    // room for the whole merge's slack entries) | the sort's scratch
    const uint64_t total = P + gaps;
    const size_t b_m = ((size_t)nm * 4 + 255) / 256 * 256, b_u = ((size_t)nm * 8 + 255) / 256 * 256;
    const size_t b_tab = b_m + 2 * b_u + 4 * b_u;
    const size_t b_scr = pend_order_scratch(P), b_rows = ((size_t)total * sizeof(IngestRow) + 255) / 256 * 256;
    void* d_tab;
    int rc;
    if ((rc = ws_get(c, "pend_order", b_tab + b_rows + b_scr, &d_tab))) return rc;
    uint8_t* tab = (uint8_t*)d_tab;
    uint64_t* d_segs = (uint64_t*)(tab + b_m);
    uint64_t* d_gapb = (uint64_t*)(tab + b_m + 2 * b_u);
    uint64_t* d_starts = (uint64_t*)(tab + b_m + 3 * b_u);
    uint64_t* d_cnt = (uint64_t*)(tab + b_m + 4 * b_u);
    uint64_t* d_first = (uint64_t*)(tab + b_m + 5 * b_u);
    IngestRow* d_rows = (IngestRow*)(tab + b_tab);
    {  // one asynchronous upload of the table through pinned staging (the first ranks are written on the device)
        const size_t hb = b_m + 5 * b_u;
        if (c->flush_pin_bytes < hb) {
            if (c->flush_pin) hipHostFree(c->flush_pin);
            c->flush_pin = nullptr;
            c->flush_pin_bytes = 0;
            if (hipHostMalloc((void**)&c->flush_pin, std::max<size_t>(hb, 4096), hipHostMallocDefault) != hipSuccess) {
                c->flush_pin = nullptr;
                return fail(DSY_ENOMEM, "hipHostMalloc for the index flush table failed");
            }
            c->flush_pin_bytes = std::max<size_t>(hb, 4096);
        }
        uint8_t* h = c->flush_pin;
        std::memcpy(h, metas.data(), (size_t)nm * 4);
        std::memcpy(h + b_m, segs.data(), (size_t)nm * 16);
        std::memcpy(h + b_m + 2 * b_u, gap_before.data(), (size_t)nm * 8);
        std::memcpy(h + b_m + 3 * b_u, starts.data(), (size_t)nm * 8);
        std::memcpy(h + b_m + 4 * b_u, cnt.data(), (size_t)nm * 8);
        HIP_TRY(hipMemcpyAsync(tab, h, hb, hipMemcpyHostToDevice, c->stream));
    }
    fc.mark("table");
    // the pending entries in index order (with_gaps: laid out for the whole merge, each meta's rows after the slack
    // of the metas before it) and, for the in-place path, each meta's first new entry's place (first).  (A one-workgroup
    // bitonic sort in LDS for batches of <= 16 K entries was measured and dropped: 176-184 us per 10 k-entry flush
    // against 42 us for the radix sorts, gpurun_out r6c1d)
    auto order = [&](bool with_gaps, uint64_t* first) -> int {
        HIP_TRY(launch_pend_order(s->d_pend_meta, s->d_pend_gt, P, s->pend_glo, s->pend_ghi, (const uint32_t*)tab,
                                  d_segs, with_gaps ? d_gapb : nullptr, nm, s->pend_base, (uint8_t*)d_rows + b_rows,
                                  b_scr, d_rows, c->stream));
        if (first) HIP_TRY(launch_first_rank(s->d_live_gt, s->d_live_row, d_rows, d_starts, d_cnt, nm, first, c->stream));
        return DSY_OK;
    };
    bool ordered_whole = false;  // d_rows hold the whole merge's layout already
whole:
    if (!fast) {
        if (!ordered_whole && (rc = order(true, nullptr))) return rc;
        fc.mark("order");
        std::map<uint32_t, std::pair<uint64_t, uint64_t>> cm;
        for (uint32_t r = 0; r < nm; ++r) {
            HIP_TRY(launch_gap_rows(d_rows + starts[r] + cnt[r] + gap_before[r], extra[r], ends[r], c->stream));
            if (cnt[r] || extra[r]) cm[metas[r]] = {cnt[r], extra[r]};
        }
        if ((rc = live_merge(c, s, d_rows, total, cm, false))) return rc;
        fc.mark("whole_merge");
        fc.done(P, "whole");
        s->pend_n = 0;
        s->pend_cnt.clear();
        return DSY_OK;
    }
    // in place: each meta's tail [p, b) -- p: its first new entry's position -- is copied aside and merged with the
    // meta's new entries back into [p, b + k), inside the region's slack
    std::vector<uint64_t> first(nm);
    if ((rc = order(false, d_first))) return rc;
    fc.mark("order");
    HIP_TRY(hipMemcpyAsync(first.data(), d_first, (size_t)nm * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    fc.mark("first_rank");
    uint64_t tail_max = 0, tail_sum = 0;
    for (uint32_t r = 0; r < nm; ++r)
        if (cnt[r]) {
            tail_max = std::max(tail_max, segs[2 * r + 1] - first[r]);
            tail_sum += segs[2 * r + 1] - first[r];
        }
    if (64 * tail_sum > 32 * s->n_phys) {  // 64 B per tail entry (copied out and back) vs 32: the whole merge instead
        fast = false;
        // (with no slack before any meta's rows the in-place order is the whole merge's layout already)
        ordered_whole = true;
        for (uint32_t r = 0; r < nm; ++r) ordered_whole = ordered_whole && gap_before[r] == 0;
        goto whole;
    }
    void* d_tmp;
    if ((rc = ws_get(c, "live_merge", P * 8 + 64 + tail_max * 16, &d_tmp))) return rc;
    uint64_t* d_rank = (uint64_t*)d_tmp;
    uint64_t* tail_gt = d_rank + P + 8;
    uint64_t* tail_row = tail_gt + tail_max;
    uint64_t* live_gt = const_cast<uint64_t*>(s->d_live_gt);
    uint64_t* live_row = const_cast<uint64_t*>(s->d_live_row);
    uint64_t moved = 0;
    for (uint32_t r = 0; r < nm; ++r) {
        if (!cnt[r]) continue;
        const uint64_t p = first[r], b = segs[2 * r + 1], L = b - p;
        if (L) {
            HIP_TRY(hipMemcpyAsync(tail_gt, live_gt + p, L * 8, hipMemcpyDeviceToDevice, c->stream));
            HIP_TRY(hipMemcpyAsync(tail_row, live_row + p, L * 8, hipMemcpyDeviceToDevice, c->stream));
        }
        HIP_TRY(launch_rows_seg(d_rows + starts[r], cnt[r], 0, L, c->stream));
        HIP_TRY(launch_ingest_merge(tail_gt, tail_row, L, d_rows + starts[r], cnt[r], d_rank, live_gt + p,
                                    live_row + p, nullptr, c->max_grid, c->stream));
        // (the copies on one stream: the next meta's tail copy waits for this merge's reads of the scratch)
        moved += L;
        s->segs[metas[r]].second += cnt[r];
    }
    // (no host wait: the index's next reader is stream-ordered behind the merges)
    fc.mark("tail_merge");
    fc.done(P, "in_place");
    s->n_live += P;
    s->ix_fast += 1;
    s->ix_bytes += 16 * P + 64 * moved;  // the new entries written; each tail entry copied out and merged back
    s->pend_n = 0;
    s->pend_cnt.clear();
    return DSY_OK;
}

// dsy_store_append and dsy_store_append_gather: the packets are blob[offsets[j], offsets[j+1]) (blob form, addrs NULL)
// or addrs[j] with offsets[] their running lengths from 0 (gather form: copied into the pinned staging here, one
// upload with the columns).  The caller has checked the arguments.
static int store_append(dsy_ctx* c, dsy_store* s, const uint8_t* blob, const uint64_t* offsets, const uint64_t* addrs,
                        uint64_t a, const uint64_t* gt, const uint32_t* meta, const uint64_t* member) {
    int rc;
    Guard g(c);
    if (c->inflight()) return fail(DSY_EINVAL, "the store cannot change while submitted responder batches are in flight");
    const uint64_t n0 = s->n, base0 = offsets[0], add = offsets[a] - base0;
    uint64_t minlen = ~0ull, maxlen = 0;
    for (uint64_t j = 0; j < a; ++j) {
        minlen = std::min(minlen, offsets[j + 1] - offsets[j]);
        maxlen = std::max(maxlen, offsets[j + 1] - offsets[j]);
    }

    HIP_TRY(hipStreamSynchronize(c->stream));  // nothing in flight reads a buffer that is about to be replaced
    // the small columns, staged in pinned memory for one upload: [offsets | row records | global times | metas |
    // members]
    const size_t b_off = (a + 1) * 8, b_rec = a * sizeof(RowRec), b_gt = a * 8, b_meta = (a * 4 + 15) / 16 * 16,
                 b_mem = member ? a * 8 : 0, b_cols = b_off + b_rec + b_gt + b_meta + b_mem;
    const size_t b_blob = (add + 15) / 16 * 16, b_stage = b_cols + (addrs ? b_blob : 0);
    if (c->in_stage_bytes < b_stage) {
        if (c->in_stage) hipHostFree(c->in_stage);
        c->in_stage = nullptr;
        c->in_stage_bytes = 0;
        const size_t want = std::max<size_t>(b_stage + b_stage / 4, 4096);
        if (hipHostMalloc((void**)&c->in_stage, want, hipHostMallocDefault) != hipSuccess) {
            c->in_stage = nullptr;
            return fail(DSY_ENOMEM, "hipHostMalloc(%zu) for the ingest staging failed", want);
        }
        c->in_stage_bytes = want;
    }
    uint64_t* h_off = (uint64_t*)c->in_stage;
    RowRec* h_rec = (RowRec*)(c->in_stage + b_off);
    // the line copy the responder hashes from, and its row records
    uint64_t at = s->lines_used;
    for (uint64_t j = 0; j < a; ++j) {
        const uint64_t len = offsets[j + 1] - offsets[j];
        h_rec[j] = RowRec{at + kLineBias, (uint32_t)len, 0u};
        at += line_bytes_for(len);
    }
    for (uint64_t j = 0; j <= a; ++j) h_off[j] = offsets[j] - base0;
    std::memcpy(c->in_stage + b_off + b_rec, gt, a * 8);
    std::memcpy(c->in_stage + b_off + b_rec + b_gt, meta, a * 4);
    if (member) std::memcpy(c->in_stage + b_off + b_rec + b_gt + b_meta, member, a * 8);
    if (addrs)  // the packets, gathered from the caller's objects
        for (uint64_t j = 0; j < a; ++j)
            std::memcpy(c->in_stage + b_cols + offsets[j], (const void*)(uintptr_t)addrs[j], offsets[j + 1] - offsets[j]);
    if ((rc = lines_reserve(c, s, at))) return rc;
    if (n0 + a > s->rec_cap) {
        const uint64_t cap = grown(n0 + a, s->rec_cap);
        void* nr;
        if (hipMalloc(&nr, cap * sizeof(RowRec)) != hipSuccess) return fail(DSY_ENOMEM, "store row records growth");
        HIP_TRY(hipMemcpyAsync(nr, s->d_rec, n0 * sizeof(RowRec), hipMemcpyDeviceToDevice, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        store_release(s, s->d_rec);
        s->owned.push_back(nr);
        s->d_rec = (const RowRec*)nr;
        s->rec_cap = cap;
    }
    // the new rows join the live index (positions n0 .. n0+a-1: after every stored row of equal global time) at the
    // next read of the index (store_flush): their (meta, global_time) entries wait on the device
    if (s->pend_n + a > s->pend_cap) {
        const uint64_t cap = grown(s->pend_n + a, s->pend_cap);
        void *pg, *pm;
        if (hipMalloc(&pg, cap * 8) != hipSuccess) return fail(DSY_ENOMEM, "store pending index growth");
        if (hipMalloc(&pm, cap * 4) != hipSuccess) { hipFree(pg); return fail(DSY_ENOMEM, "store pending index growth"); }
        if (s->pend_n) {
            HIP_TRY(hipMemcpyAsync(pg, s->d_pend_gt, s->pend_n * 8, hipMemcpyDeviceToDevice, c->stream));
            HIP_TRY(hipMemcpyAsync(pm, s->d_pend_meta, s->pend_n * 4, hipMemcpyDeviceToDevice, c->stream));
        }
        HIP_TRY(hipStreamSynchronize(c->stream));
        store_release(s, s->d_pend_gt);
        store_release(s, s->d_pend_meta);
        s->owned.push_back(pg);
        s->owned.push_back(pm);
        s->d_pend_gt = (uint64_t*)pg;
        s->d_pend_meta = (uint32_t*)pm;
        s->pend_cap = cap;
    }

    // uploads (one workspace): the packets from the caller's buffer, the staged columns in one copy; the packets then
    // move to their line-aligned places
    void* d_up;
    if ((rc = ws_get(c, "ingest", b_blob + b_cols, &d_up))) return rc;
    uint8_t* up = (uint8_t*)d_up;
    uint8_t* up_off = up + b_blob;
    uint8_t* up_rec = up_off + b_off;
    uint8_t* up_gt = up_rec + b_rec;
    uint8_t* up_meta = up_gt + b_gt;
    uint8_t* up_mem = up_meta + b_meta;
    if (add) HIP_TRY(hipMemcpyAsync(up, addrs ? c->in_stage + b_cols : blob + base0, add, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(up_off, c->in_stage, b_cols, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(const_cast<RowRec*>(s->d_rec) + n0, up_rec, b_rec, hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(s->d_pend_gt + s->pend_n, up_gt, b_gt, hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(s->d_pend_meta + s->pend_n, up_meta, a * 4, hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(launch_store_lines(up, (const uint64_t*)up_off, s->d_rec + n0, a, const_cast<uint8_t*>(s->d_lines),
                               c->stream));
    // the duplicate table first: if it cannot take the rows (DSY_ENOMEM growing it), nothing below is committed -- the
    // queued index entries past pend_n are never read, and the store keeps its n rows
    if (s->dup && (rc = dup_insert_dev(c, s, (const uint64_t*)up_mem, (const uint64_t*)up_gt, n0, a))) return rc;
    if (!s->pend_n) {
        s->pend_base = n0;
        s->pend_glo = ~0ull;
        s->pend_ghi = 0;
    }
    for (uint64_t j = 0; j < a; ++j) {
        s->pend_glo = std::min(s->pend_glo, gt[j]);
        s->pend_ghi = std::max(s->pend_ghi, gt[j]);
    }
    for (uint64_t j = 0; j < a;) {  // runs of one meta: one map update each
        uint64_t e = j + 1;
        while (e < a && meta[e] == meta[j]) ++e;
        s->pend_cnt[meta[j]] += e - j;
        j = e;
    }
    s->pend_n += a;
    s->min_len = n0 ? std::min(s->min_len, minlen) : minlen;
    s->max_len = std::max(s->max_len, maxlen);
    s->n += a;
    s->blob_len += add;
    s->lines_used = at;
    return DSY_OK;
}

int dsy_store_append(dsy_ctx* c, dsy_store* s, const uint8_t* blob, uint64_t blob_len, const uint64_t* offsets,
                     uint64_t a, const uint64_t* gt, const uint32_t* meta, const uint64_t* member) {
    if (!c || !s || !offsets || (a && (!gt || !meta || (blob_len && !blob)))) return fail(DSY_EINVAL, "NULL argument");
    if (s->ctx != c) return fail(DSY_EINVAL, "store belongs to another context");
    if (s->dup && a && !member) return fail(DSY_EINVAL, "the store has a (member, global_time) table: members required");
    int rc = check_offsets(offsets, a, blob_len);
    if (rc) return rc;
    if (a == 0) return DSY_OK;
    return store_append(c, s, blob, offsets, nullptr, a, gt, meta, member);
}

int dsy_store_append_gather(dsy_ctx* c, dsy_store* s, const uint64_t* addrs, const uint64_t* lengths, uint64_t a,
                            const uint64_t* gt, const uint32_t* meta, const uint64_t* member) {
    if (!c || !s || (a && (!addrs || !lengths || !gt || !meta))) return fail(DSY_EINVAL, "NULL argument");
    if (s->ctx != c) return fail(DSY_EINVAL, "store belongs to another context");
    if (s->dup && a && !member) return fail(DSY_EINVAL, "the store has a (member, global_time) table: members required");
    if (a == 0) return DSY_OK;
    std::vector<uint64_t> off(a + 1);
    off[0] = 0;
    for (uint64_t j = 0; j < a; ++j) {
        if (lengths[j] && !addrs[j]) return fail(DSY_EINVAL, "packet %llu: NULL address", (unsigned long long)j);
        if (lengths[j] > 0xFFFFFFFFull) return fail(DSY_EINVAL, "packet %llu longer than 4 GiB", (unsigned long long)j);
        off[j + 1] = off[j] + lengths[j];
    }
    return store_append(c, s, nullptr, off.data(), addrs, a, gt, meta, member);
}


int dsy_store_index_stats(const dsy_store* s, uint64_t* out) {
    if (!s || !out) return fail(DSY_EINVAL, "NULL argument");
    out[0] = s->n_live;
    out[1] = s->n_phys;
    out[2] = s->ix_fast;
    out[3] = s->ix_full;
    out[4] = s->ix_bytes;
    out[5] = s->pend_n;
    return DSY_OK;
}

int dsy_store_prune(dsy_ctx* c, dsy_store* s, uint32_t meta, uint64_t max_gt, uint64_t* out_deleted) {
    if (!c || !s || !out_deleted) return fail(DSY_EINVAL, "NULL argument");
    if (s->ctx != c) return fail(DSY_EINVAL, "store belongs to another context");
    *out_deleted = 0;
    Guard g(c);
    if (c->inflight()) return fail(DSY_EINVAL, "the store cannot change while submitted responder batches are in flight");
    if (int rc = store_flush(c, s)) return rc;
    auto it = s->segs.find(meta);
    if (it == s->segs.end() || it->second.first == it->second.second) return DSY_OK;
    const uint64_t a = it->second.first, b = it->second.second;
    void* d_k;
    int rc;
    if ((rc = ws_get(c, "prune_k", 64, &d_k))) return rc;
    HIP_TRY(launch_prune_count(s->d_live_gt, a, b, max_gt, (uint64_t*)d_k, c->stream));
    uint64_t k = 0;
    HIP_TRY(hipMemcpyAsync(&k, d_k, 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (!k) return DSY_OK;
    // the deleted rows leave the (member, global_time) table too: a later lookup finds nothing (dispersy.py:868)
    if (s->dup) HIP_TRY(launch_dup_erase(nullptr, s->d_live_row, a, k, s->dup_keys, s->dup, s->dup_cap - 1, c->stream));
    const uint64_t n_out = s->n_phys - k;  // the index arrays without the k entries (slack included)
    if ((rc = spare_reserve(s, std::max<uint64_t>(n_out, 1), s->n_phys))) return rc;
    HIP_TRY(launch_live_cut(s->d_live_gt, s->d_live_row, n_out, a, k, s->spare_gt, s->spare_row, c->max_grid, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    spare_swap(s);
    for (auto& e : s->segs) {  // this meta's segment loses its first k rows; later segments move down by k
        if (e.first == meta) e.second.second -= k;
        else if (e.second.first >= b) { e.second.first -= k; e.second.second -= k; }
    }
    s->n_live -= k;
    s->n_phys = n_out;
    *out_deleted = k;
    return DSY_OK;
}

// The given rows leave the live index (a stable compaction on the device; rows not in it are ignored); erase_dup: their
// (member, global_time) slots become tombstones too (a DELETE; an undo keeps them).  *out_removed = index entries
// removed.  The caller holds the ctx lock and has validated the rows.
static int live_remove(dsy_ctx* c, dsy_store* s, const uint64_t* rows, uint64_t k, bool erase_dup,
                       uint64_t* out_removed) {
    uint64_t* out_deleted = out_removed;
    // segment bounds (old positions) to remap: every meta's [a, b)
    std::vector<uint32_t> seg_ids;
    std::vector<uint64_t> bounds;
    for (auto& e : s->segs) {
        seg_ids.push_back(e.first);
        bounds.push_back(e.second.first);
        bounds.push_back(e.second.second);
    }
    bounds.push_back(s->n_phys);
    const uint64_t words = (s->n + 31) / 32, tiles = (s->n_phys + kDelTile - 1) / kDelTile;
    const size_t b_bits = (words * 4 + 15) / 16 * 16, b_rows = k * 8, b_tiles = (tiles + 1) * 8,
                 b_bounds = bounds.size() * 8;
    void* d;
    int rc;
    if ((rc = ws_get(c, "delete", b_bits + b_rows + b_tiles + b_bounds, &d))) return rc;
    uint8_t* p = (uint8_t*)d;
    uint32_t* d_bits = (uint32_t*)p;
    uint64_t *d_rows = (uint64_t*)(p + b_bits), *d_tiles = (uint64_t*)(p + b_bits + b_rows),
             *d_bounds = (uint64_t*)(p + b_bits + b_rows + b_tiles);
    HIP_TRY(hipMemsetAsync(d_bits, 0, words * 4, c->stream));
    HIP_TRY(hipMemcpyAsync(d_rows, rows, b_rows, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(d_bounds, bounds.data(), b_bounds, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(launch_mark_rows(d_rows, k, s->n, d_bits, c->stream));
    // the deleted rows' (member, global_time) slots become tombstones (also rows outside the live index: undone ones)
    if (erase_dup && s->dup) HIP_TRY(launch_dup_erase(d_rows, nullptr, 0, k, s->dup_keys, s->dup, s->dup_cap - 1, c->stream));
    // (the compaction drops the slack entries too: the new index is dense)
    if ((rc = spare_reserve(s, std::max<uint64_t>(s->n_phys, 1), s->n_phys))) return rc;
    HIP_TRY(launch_live_delete(s->d_live_gt, s->d_live_row, s->n_phys, d_bits, d_tiles, s->spare_gt, s->spare_row,
                               d_bounds, (uint32_t)bounds.size(), c->stream));
    HIP_TRY(hipMemcpyAsync(bounds.data(), d_bounds, b_bounds, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    const uint64_t live = bounds.back();
    *out_deleted = s->n_live - live;
    if (live == s->n_live) return DSY_OK;  // none of the rows was in the live index: the old index stays
    spare_swap(s);
    for (size_t j = 0; j < seg_ids.size(); ++j) s->segs[seg_ids[j]] = {bounds[2 * j], bounds[2 * j + 1]};
    s->n_live = live;
    s->n_phys = live;
    return DSY_OK;
}

int dsy_store_delete(dsy_ctx* c, dsy_store* s, const uint64_t* rows, uint64_t k, uint64_t* out_deleted) {
    if (!c || !s || !out_deleted || (k && !rows)) return fail(DSY_EINVAL, "NULL argument");
    if (s->ctx != c) return fail(DSY_EINVAL, "store belongs to another context");
    for (uint64_t i = 0; i < k; ++i)
        if (rows[i] >= s->n) return fail(DSY_EINVAL, "row %llu out of range (%llu rows)", (unsigned long long)rows[i], (unsigned long long)s->n);
    *out_deleted = 0;
    if (!k) return DSY_OK;
    Guard g(c);
    if (c->inflight()) return fail(DSY_EINVAL, "the store cannot change while submitted responder batches are in flight");
    if (int rc = store_flush(c, s)) return rc;
    return live_remove(c, s, rows, k, true, out_deleted);
}

int dsy_store_set_undone(dsy_ctx* c, dsy_store* s, const uint64_t* rows, uint64_t k, const uint32_t* meta,
                         const uint64_t* gt, int undone, uint64_t* out_changed) {
    if (!c || !s || !out_changed || (k && (!rows || (!undone && (!meta || !gt))))) return fail(DSY_EINVAL, "NULL argument");
    if (s->ctx != c) return fail(DSY_EINVAL, "store belongs to another context");
    for (uint64_t i = 0; i < k; ++i)
        if (rows[i] >= s->n) return fail(DSY_EINVAL, "row %llu out of range (%llu rows)", (unsigned long long)rows[i], (unsigned long long)s->n);
    *out_changed = 0;
    if (!k) return DSY_OK;
    Guard g(c);
    if (c->inflight()) return fail(DSY_EINVAL, "the store cannot change while submitted responder batches are in flight");
    if (int rc = store_flush(c, s)) return rc;
    if (undone) return live_remove(c, s, rows, k, false, out_changed);
    std::vector<uint64_t> r(rows, rows + k);
    std::vector<uint64_t> sorted_r(r);
    std::sort(sorted_r.begin(), sorted_r.end());
    if (std::adjacent_find(sorted_r.begin(), sorted_r.end()) != sorted_r.end()) return fail(DSY_EINVAL, "a row is given twice");
    int rc = live_insert(c, s, meta, gt, r.data(), k, true);
    if (rc) return rc;
    *out_changed = k;
    return DSY_OK;
}

int dsy_store_index_members(dsy_ctx* c, dsy_store* s, const uint64_t* member, const uint64_t* gt, uint64_t n) {
    if (!c || !s || (n && (!member || !gt))) return fail(DSY_EINVAL, "NULL argument");
    if (s->ctx != c) return fail(DSY_EINVAL, "store belongs to another context");
    if (n != s->n) return fail(DSY_EINVAL, "%llu members for a store of %llu rows", (unsigned long long)n, (unsigned long long)s->n);
    Guard g(c);
    if (s->dup) {  // rebuild from scratch (the row keys are rewritten by the insert)
        store_release(s, s->dup);
        s->dup = nullptr;
        s->dup_cap = s->dup_count = 0;
    }
    int rc = dup_reserve(c, s, n);
    if (rc) return rc;
    return dup_insert(c, s, member, gt, 0, n);
}

int dsy_dup_check(dsy_ctx* c, const dsy_store* s, const uint64_t* member, const uint64_t* gt, const uint8_t* blob,
                  uint64_t blob_len, const uint64_t* offsets, uint64_t m, const uint32_t* sig_len, uint8_t* out_verdict,
                  uint64_t* out_row) {
    if (!c || !s || !offsets || (m && (!member || !gt || !sig_len || !out_verdict || !out_row || (blob_len && !blob))))
        return fail(DSY_EINVAL, "NULL argument");
    if (!s->dup) return fail(DSY_EINVAL, "the store has no (member, global_time) table (dsy_store_index_members)");
    int rc = check_offsets(offsets, m, blob_len);
    if (rc) return rc;
    if (!m) return DSY_OK;
    Guard g(c);
    const uint64_t base0 = offsets[0], add = offsets[m] - base0;
    std::vector<uint64_t> noff(m + 1);
    for (uint64_t j = 0; j <= m; ++j) noff[j] = offsets[j] - base0;
    const size_t b_blob = (add + 15) / 16 * 16, b_k = m * 8, b_off = (m + 1) * 8, b_sl = (m * 4 + 15) / 16 * 16,
                 b_v = (m + 15) / 16 * 16;
    void* d;
    if ((rc = ws_get(c, "dup_check", b_blob + 2 * b_k + b_off + b_sl + b_v + b_k, &d))) return rc;
    uint8_t* p = (uint8_t*)d;
    uint8_t *d_blob = p, *d_mem = p + b_blob, *d_gt = d_mem + b_k, *d_off = d_gt + b_k, *d_sl = d_off + b_off,
            *d_v = d_sl + b_sl, *d_row = d_v + b_v;
    if (add) HIP_TRY(hipMemcpyAsync(d_blob, blob + base0, add, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(d_mem, member, b_k, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(d_gt, gt, b_k, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(d_off, noff.data(), b_off, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(d_sl, sig_len, m * 4, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(launch_dup_check(s->dup, s->dup_cap - 1, s->d_lines, s->d_rec, (const uint64_t*)d_mem,
                             (const uint64_t*)d_gt, d_blob, (const uint64_t*)d_off, (const uint32_t*)d_sl, m, d_v,
                             (uint64_t*)d_row, c->stream));
    HIP_TRY(hipMemcpyAsync(out_verdict, d_v, m, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(out_row, d_row, m * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return DSY_OK;
}

int dsy_store_replace(dsy_ctx* c, dsy_store* s, const uint64_t* rows, const uint8_t* blob, uint64_t blob_len,
                      const uint64_t* offsets, uint64_t k) {
    if (!c || !s || !offsets || (k && (!rows || (blob_len && !blob)))) return fail(DSY_EINVAL, "NULL argument");
    if (s->ctx != c) return fail(DSY_EINVAL, "store belongs to another context");
    int rc = check_offsets(offsets, k, blob_len);
    if (rc) return rc;
    for (uint64_t i = 0; i < k; ++i)
        if (rows[i] >= s->n) return fail(DSY_EINVAL, "row %llu out of range (%llu rows)", (unsigned long long)rows[i], (unsigned long long)s->n);
    if (!k) return DSY_OK;
    Guard g(c);
    if (c->inflight()) return fail(DSY_EINVAL, "the store cannot change while submitted responder batches are in flight");
    HIP_TRY(hipStreamSynchronize(c->stream));
    const uint64_t base0 = offsets[0], add = offsets[k] - base0;
    std::vector<RowRec> nrec(k);
    std::vector<uint64_t> noff(k + 1);
    uint64_t at = s->lines_used, minlen = s->min_len;
    for (uint64_t i = 0; i < k; ++i) {
        const uint64_t len = offsets[i + 1] - offsets[i];
        nrec[i] = RowRec{at + kLineBias, (uint32_t)len, 0u};
        at += line_bytes_for(len);
        minlen = std::min(minlen, len);
        s->max_len = std::max(s->max_len, len);
    }
    for (uint64_t i = 0; i <= k; ++i) noff[i] = offsets[i] - base0;
    if ((rc = lines_reserve(c, s, at))) return rc;
    const size_t b_blob = (add + 15) / 16 * 16, b_off = (k + 1) * 8, b_rec = k * sizeof(RowRec), b_rows = k * 8;
    void* d;
    if ((rc = ws_get(c, "replace", b_blob + b_off + b_rec + b_rows, &d))) return rc;
    uint8_t *d_blob = (uint8_t*)d, *d_off = d_blob + b_blob, *d_rec = d_off + b_off, *d_rows = d_rec + b_rec;
    if (add) HIP_TRY(hipMemcpyAsync(d_blob, blob + base0, add, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(d_off, noff.data(), b_off, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(d_rec, nrec.data(), b_rec, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(d_rows, rows, b_rows, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(launch_store_lines(d_blob, (const uint64_t*)d_off, (const RowRec*)d_rec, k, const_cast<uint8_t*>(s->d_lines),
                               c->stream));
    HIP_TRY(launch_rec_scatter(const_cast<RowRec*>(s->d_rec), (const uint64_t*)d_rows, (const RowRec*)d_rec, k,
                               c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    s->lines_used = at;
    s->min_len = minlen;
    return DSY_OK;
}

int dsy_bloom_add_rows(dsy_ctx* c, const dsy_bloom_params* p, const dsy_store* s, const uint64_t* rows, uint64_t n,
                       uint8_t* filter_inout) {
    if (!c || !s || !filter_inout || (n && !rows)) return fail(DSY_EINVAL, "NULL argument");
    int rc = check_params(p);
    if (rc) return rc;
    for (uint64_t i = 0; i < n; ++i)
        if (rows[i] >= s->n) return fail(DSY_EINVAL, "row %llu out of range (%llu rows)", (unsigned long long)rows[i], (unsigned long long)s->n);
    Guard g(c);
    const uint64_t nbytes = p->m_bits / 8, words = filter_words(p->m_bits);
    void *df, *dr;
    if ((rc = ws_get(c, "filter", words * 4, &df))) return rc;
    if ((rc = ws_get(c, "rows", (n + 1) * 8, &dr))) return rc;
    HIP_TRY(hipMemsetAsync(df, 0, words * 4, c->stream));
    HIP_TRY(hipMemcpyAsync(df, filter_inout, nbytes, hipMemcpyHostToDevice, c->stream));
    if (n) HIP_TRY(hipMemcpyAsync(dr, rows, n * 8, hipMemcpyHostToDevice, c->stream));
    // the packets come from the store's line copy (row -> rec[row]): the responder's own copy, grown by appends
    if ((rc = run_bloom(c, BloomOp::Add, p, s->d_lines, nullptr, (uint64_t*)dr, n, (uint32_t*)df, nullptr, nullptr,
                        s->d_rec)))
        return rc;
    HIP_TRY(hipMemcpyAsync(filter_inout, df, nbytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    timers_collect_lazy(c);
    return DSY_OK;
}

int dsy_claim_modulo(dsy_ctx* c, const dsy_bloom_params* p, const dsy_store* s, const uint32_t* meta_ids,
                     uint32_t nmeta, uint64_t offset, uint64_t modulo, uint8_t* filter_inout, uint64_t* out_count) {
    if (!c || !s || !filter_inout || !out_count || (nmeta && !meta_ids)) return fail(DSY_EINVAL, "NULL argument");
    if (s->ctx != c) return fail(DSY_EINVAL, "store belongs to another context");
    if (modulo == 0 || offset >= modulo)
        return fail(DSY_EINVAL, "need 0 <= offset < modulo (offset=%llu modulo=%llu)", (unsigned long long)offset,
                    (unsigned long long)modulo);
    int rc = check_params(p);
    if (rc) return rc;
    *out_count = 0;
    Guard g(c);
    if ((rc = store_flush(c, s))) return rc;
    std::vector<std::pair<uint64_t, uint64_t>> spans;
    uint64_t total = 0;
    // `meta_message IN (...)` counts each row once, however often an id is listed
    std::vector<uint32_t> ids(meta_ids, meta_ids + nmeta);
    std::sort(ids.begin(), ids.end());
    ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    for (uint32_t id : ids) {
        auto it = s->segs.find(id);
        if (it == s->segs.end() || it->second.first >= it->second.second) continue;
        spans.push_back(it->second);
        total += it->second.second - it->second.first;
    }
    const uint64_t nbytes = p->m_bits / 8, words = filter_words(p->m_bits);
    void *df, *dr, *dn;
    if ((rc = ws_get(c, "filter", words * 4, &df))) return rc;
    if ((rc = ws_get(c, "rows", (total + 1) * 8, &dr))) return rc;
    if ((rc = ws_get(c, "claim_n", 64, &dn))) return rc;
    HIP_TRY(hipMemsetAsync(df, 0, words * 4, c->stream));
    HIP_TRY(hipMemcpyAsync(df, filter_inout, nbytes, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemsetAsync(dn, 0, 8, c->stream));
    for (auto& sp : spans)
        HIP_TRY(launch_claim_modulo(s->d_live_gt, s->d_live_row, sp.first, sp.second, offset, modulo, (uint64_t*)dr,
                                    total, (unsigned long long*)dn, c->max_grid, c->stream));
    uint64_t n = 0;
    HIP_TRY(hipMemcpyAsync(&n, dn, 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (n > total) return fail(DSY_EHIP, "claim selection counted %llu of %llu rows", (unsigned long long)n,
                               (unsigned long long)total);
    if ((rc = run_bloom(c, BloomOp::Add, p, s->d_lines, nullptr, (uint64_t*)dr, n, (uint32_t*)df, nullptr, nullptr,
                        s->d_rec)))
        return rc;
    HIP_TRY(hipMemcpyAsync(filter_inout, df, nbytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    timers_collect_lazy(c);
    *out_count = n;
    return DSY_OK;
}

// ------------------------------------------------------------------------------- claim, largest strategy
namespace {

struct SelData {      // one _select_and_fix result: the rows are spans[J] of the live index (device), ascending gt
    uint64_t count = 0, first_gt = 0, last_gt = 0;
    bool fixed = false;
    uint64_t* d_spans = nullptr;
};

struct ClaimCtx {
    dsy_ctx* c;
    const dsy_store* s;
    uint64_t* d_segs;     // J x (a, b)
    uint32_t J;
    uint64_t* d_cand;     // J x (capacity + 2) scratch
    uint64_t* d_spans;    // 4 x J x 2: one span set per select call
    SelResult* d_res;     // 4 results
    int calls = 0;
};

int select_and_fix_dev(ClaimCtx& k, uint64_t pivot, uint64_t to_select, bool higher, SelData* out) {
    dsy_ctx* c = k.c;
    const int i = k.calls++;
    out->d_spans = k.d_spans + (size_t)i * k.J * 2;
    HIP_TRY(launch_select_and_fix(k.s->d_live_gt, k.d_segs, k.J, pivot, to_select, higher ? 1 : 0, k.d_cand,
                                  out->d_spans, k.d_res + i, c->stream));
    SelResult r;
    HIP_TRY(hipMemcpyAsync(&r, k.d_res + i, sizeof r, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    out->count = r.count;
    out->first_gt = r.first_gt;
    out->last_gt = r.last_gt;
    out->fixed = r.fixed != 0;
    return DSY_OK;
}

struct RangeData {    // _select_bloomfilter_range's result: [lo, hi, count] and the (one or two) span sets
    uint64_t lo = 0, hi = 0, count = 0;
    std::vector<uint64_t*> spans;
};

// community.py:839-879 (IndexError when no row is selected: DSY_EEMPTY)
int select_range_dev(ClaimCtx& k, uint64_t gt, uint64_t to_select, bool higher, uint64_t acceptable, RangeData* out) {
    SelData data, more;
    int rc = select_and_fix_dev(k, gt, to_select, higher, &data);
    if (rc) return rc;
    bool lowerfixed = true, higherfixed = true;
    bool have_more = false;
    if (data.count < to_select) {
        const uint64_t remain = to_select - data.count;
        if (remain > 25) {
            if ((rc = select_and_fix_dev(k, higher ? gt + 1 : gt - 1, remain, !higher, &more))) return rc;
            have_more = true;
            (higher ? lowerfixed : higherfixed) = more.fixed;
        }
    }
    const uint64_t n = data.count + (have_more ? more.count : 0);
    if (n == 0) return fail(DSY_EEMPTY, "no rows around global time %llu (community.py:857 raises IndexError)",
                            (unsigned long long)gt);
    // data[0] / data[-1]: `more` comes before data (higher: lowerdata + data) or after it (data + higherdata)
    uint64_t first, last;
    if (higher) {
        first = have_more && more.count ? more.first_gt : data.first_gt;
        last = data.count ? data.last_gt : more.last_gt;
    } else {
        first = data.count ? data.first_gt : more.first_gt;
        last = have_more && more.count ? more.last_gt : data.last_gt;
    }
    uint64_t lo = first, hi = last;
    if (higher) {
        lo = std::min(lo, gt + 1);
        if (!data.fixed) hi = acceptable;
        if (!lowerfixed) lo = 1;
    } else {
        hi = std::max(hi, gt - 1);
        if (!data.fixed) lo = 1;
        if (!higherfixed) hi = acceptable;
    }
    out->lo = lo;
    out->hi = hi;
    out->count = n;
    out->spans.push_back(data.d_spans);
    if (have_more) out->spans.push_back(more.d_spans);
    return DSY_OK;
}

}  // namespace

int dsy_claim_largest(dsy_ctx* c, const dsy_bloom_params* p, const dsy_store* s, const uint32_t* meta_ids,
                      uint32_t nmeta, uint64_t from_gbtime, uint64_t capacity, uint64_t nrsyncpackets,
                      uint64_t acceptable_global_time, uint8_t* filter_inout, uint64_t* out_claim) {
    if (!c || !s || !filter_inout || !out_claim || (nmeta && !meta_ids)) return fail(DSY_EINVAL, "NULL argument");
    if (s->ctx != c) return fail(DSY_EINVAL, "store belongs to another context");
    if (capacity == 0) return fail(DSY_EINVAL, "capacity must be positive");
    int rc = check_params(p);
    if (rc) return rc;
    Guard g(c);
    if ((rc = store_flush(c, s))) return rc;
    // the syncable metas' live segments (`meta_message IN (...)`: each id once)
    std::vector<uint32_t> ids(meta_ids, meta_ids + nmeta);
    std::sort(ids.begin(), ids.end());
    ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    std::vector<uint64_t> segs;
    for (uint32_t id : ids) {
        auto it = s->segs.find(id);
        if (it == s->segs.end() || it->second.first >= it->second.second) continue;
        segs.push_back(it->second.first);
        segs.push_back(it->second.second);
    }
    const uint32_t J = (uint32_t)(segs.size() / 2);
    out_claim[0] = out_claim[1] = out_claim[2] = 0;
    out_claim[3] = nrsyncpackets;
    const size_t b_segs = (size_t)J * 16, b_cand = (size_t)J * (capacity + 2) * 8, b_spans = (size_t)4 * J * 16,
                 b_res = 4 * sizeof(SelResult);
    void* d;
    if ((rc = ws_get(c, "claim_largest", b_segs + b_cand + b_spans + b_res, &d))) return rc;
    uint8_t* q = (uint8_t*)d;
    ClaimCtx k{c, s, (uint64_t*)q, J, (uint64_t*)(q + b_segs), (uint64_t*)(q + b_segs + b_cand),
               (SelResult*)(q + b_segs + b_cand + b_spans)};
    HIP_TRY(hipMemcpyAsync(k.d_segs, segs.data(), b_segs, hipMemcpyHostToDevice, c->stream));
    // community.py:783-830, after the random draws (the caller passes from_gbtime)
    RangeData chosen;
    std::vector<uint64_t*> spans;
    uint64_t lo, hi, count;
    if (from_gbtime > 1 && nrsyncpackets >= capacity) {
        RangeData right;
        if ((rc = select_range_dev(k, from_gbtime - 1, capacity, true, acceptable_global_time, &right))) return rc;
        if (right.count == capacity) {
            RangeData left;
            if ((rc = select_range_dev(k, from_gbtime + 1, capacity, false, acceptable_global_time, &left))) return rc;
            // `(left[1] or self.global_time) - left[0]`: the bounds are >= 1 here, so the `or` never applies
            const int64_t left_range = (int64_t)left.hi - (int64_t)left.lo, right_range = (int64_t)right.hi - (int64_t)right.lo;
            chosen = left_range > right_range ? left : right;
        } else {
            chosen = right;
        }
        lo = chosen.lo;
        hi = chosen.hi;
        count = chosen.count;
        spans = chosen.spans;
    } else {
        SelData data;
        if ((rc = select_and_fix_dev(k, 0, capacity, true, &data))) return rc;
        lo = 1;
        hi = acceptable_global_time;
        if (data.count && data.fixed) {
            hi = data.last_gt;
            out_claim[3] = capacity + 1;
        }
        count = data.count;
        spans.push_back(data.d_spans);
    }
    if (count == 0) return DSY_OK;  // the empty claim
    // add_keys over the selected rows (community.py:821), hashed from the store's line copy
    void* dr;
    if ((rc = ws_get(c, "rows", (count + 1) * 8, &dr))) return rc;
    uint64_t at = 0;
    for (uint64_t* sp : spans) {
        // one span set's rows, after the previous set's: compact copy of J spans
        HIP_TRY(launch_span_rows(s->d_live_row, sp, J, (uint64_t*)dr + at, c->stream));
        std::vector<uint64_t> h(2 * J);
        HIP_TRY(hipMemcpyAsync(h.data(), sp, 16 * J, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        for (uint32_t j = 0; j < J; ++j) at += h[2 * j + 1] - h[2 * j];
    }
    if (at != count) return fail(DSY_EHIP, "claim selection: %llu rows gathered, %llu selected", (unsigned long long)at,
                                 (unsigned long long)count);
    const uint64_t nbytes = p->m_bits / 8, words = filter_words(p->m_bits);
    void* df;
    if ((rc = ws_get(c, "filter", words * 4, &df))) return rc;
    HIP_TRY(hipMemsetAsync(df, 0, words * 4, c->stream));
    HIP_TRY(hipMemcpyAsync(df, filter_inout, nbytes, hipMemcpyHostToDevice, c->stream));
    if ((rc = run_bloom(c, BloomOp::Add, p, s->d_lines, nullptr, (uint64_t*)dr, count, (uint32_t*)df, nullptr, nullptr,
                        s->d_rec)))
        return rc;
    HIP_TRY(hipMemcpyAsync(filter_inout, df, nbytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    timers_collect_lazy(c);
    out_claim[0] = std::min(lo, acceptable_global_time);
    out_claim[1] = std::min(hi, acceptable_global_time);
    out_claim[2] = count;
    return DSY_OK;
}

// -------------------------------------------------------------------------------------------- responder
// The window pool holds kWindow pairs per claim of the call, and at least kMinSlots claims' worth (16 M pairs,
// 400 MB of workspace); each window the active claims share it evenly, from kWindow up to kMaxWindow pairs each.
// Few long-running claims then take a handful of big windows: every window costs at least the serial digest of
// its longest packet on one lane (~1 ms for a 64 KB packet), so their number matters.
static const uint64_t kWindow = 4096;
static const uint64_t kMaxWindow = 1 << 18;
static const uint64_t kMinSlots = 4096;
// DSY_BIG_POOL (experiments; 0 by default): windows after the first share a pool of that many pairs, allocated the
// first time a call needs it, and W may reach 2^20.  Measured on config 5 (2^27 pairs): 9 -> 3 windows per step but
// the same 11.9 ms of hashing (3 x 3.97 ms instead of 9 x 1.32: a window is not bounded by its longest packet's serial
// digest) and a slower step, 16.8 -> 19.5 ms (one k_compact wave walks a 2^20-pair window's miss words).
static uint64_t big_pool_pairs() {
    static const uint64_t v = getenv("DSY_BIG_POOL") ? strtoull(getenv("DSY_BIG_POOL"), nullptr, 0) : 0;
    return v;
}

// (Re)bind a job's per-pair buffers for `pairs` pairs (window slots x W); grows the slot's workspace when needed.
static int job_pair_buffers(RespondSlot& sl, uint64_t pairs) {
    RespondJob& jb = sl.job;
    RespondLaunch& L = jb.L;
    Workspace& w = sl.w;
    void *d_pairs, *d_off, *d_len, *d_miss, *d_task;
    int rc;
    if ((rc = ws_get(w, "pairs", pairs * 8, &d_pairs))) return rc;
    if ((rc = ws_get(w, "pair_off", pairs * 8, &d_off))) return rc;
    if ((rc = ws_get(w, "pair_len", pairs * 4, &d_len))) return rc;
    if ((rc = ws_get(w, "miss_mask", pairs / 8 + 64, &d_miss))) return rc;
    if ((rc = ws_get(w, "task", pairs * sizeof(PairTask), &d_task))) return rc;
    L.pair_row = (uint64_t*)d_pairs;
    L.pair_off = (uint64_t*)d_off;
    L.pair_len = (uint32_t*)d_len;
    L.miss_mask = (uint64_t*)d_miss;
    L.task = (PairTask*)d_task;
    if (L.pool_mask) {
        void* d_pool;
        if ((rc = ws_get(w, "pool_task", pairs * sizeof(PoolTask), &d_pool))) return rc;
        L.pool = (PoolTask*)d_pool;
    }
    jb.cap_pairs = pairs;
    return DSY_OK;
}

// DSY_HOST_PROFILE: one stderr line per call with the host-side phases of respond_core (microseconds)
static double host_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static const bool g_host_profile = getenv("DSY_HOST_PROFILE") != nullptr;

// One window of a job: fill -> hash/test (one launch per hash family) -> compact -> speculative pack, enqueued on the
// slot's stream without waiting.  Only the active claims take part; as they finish, the rest share the pool in bigger
// windows.
static int job_window(dsy_ctx* c, RespondSlot& sl) {
    RespondJob& jb = sl.job;
    RespondLaunch& L = jb.L;
    const hipStream_t st = c->stream;
    L.stream = st;
    std::vector<std::pair<size_t, size_t>> runs;  // per family: (first slot, slots)
    size_t n_act = 0;
    for (auto& fa : jb.fam_active) {
        runs.push_back({n_act, fa.size()});
        n_act += fa.size();
    }
    const uint64_t pool_now = jb.first ? jb.pool : std::max<uint64_t>(jb.pool, std::min<uint64_t>(big_pool_pairs(),
                                                                                                 0xffffffffull));
    uint64_t W = pool_now / n_act / 64 * 64;
    W = std::min<uint64_t>(std::max<uint64_t>(W, kWindow), big_pool_pairs() ? kMaxWindow * 4 : kMaxWindow);
    if (c->window_cap) W = std::min<uint64_t>(W, c->window_cap);
    L.window = W;
    int rc;
    if (W * n_act > jb.cap_pairs) {  // a later window's bigger pool (this slot's earlier windows have completed)
        if ((rc = job_pair_buffers(sl, W * n_act))) return rc;
    }
    L.n_act = (uint32_t)n_act;
    if (!jb.first) {  // the first window's list went up with the claims
        uint32_t* h_act = jb.h_act_next;
        size_t a = 0;
        for (auto& fa : jb.fam_active)
            for (uint32_t r : fa) h_act[a++] = r;
        HIP_TRY(hipMemcpyAsync(jb.d_act, h_act, n_act * 4, hipMemcpyHostToDevice, st));
    }
    jb.first = false;
    jb.ran = true;
    static const bool fill_profile = getenv("DSY_FILL_PROFILE") != nullptr;
    void* d_fc = nullptr;
    if (fill_profile) {
        if ((rc = ws_get(sl.w, "fill_clock", n_act * 32 + 32, &d_fc))) return rc;
        HIP_TRY(hipMemsetAsync(d_fc, 0, n_act * 32, st));
        L.fill_clock = (uint64_t*)d_fc;
    }
    PendingTimer t;
    timer_begin(c, &t, kTimeSelect, st);
    if (jb.first_fill && jb.fused_first)
        HIP_TRY(launch_fill_first(L, jb.h_in, jb.d_in, jb.in_b, jb.d_io, jb.cnt_b, jb.per_claim,
                                  jb.act0_identity ? nullptr : jb.h_act0));
    else
        HIP_TRY(launch_fill(L));
    jb.first_fill = false;
    timer_end(c, &t, st);
    if (sl.gather.refs) {  // the claims' filters, gathered and uploaded while the selection runs
        // in chunks on the aux stream: chunk i's transfer overlaps chunk i+1's host copy and the selection kernel;
        // the ctx stream waits for the last one before the hashing
        FilterGather& fg = sl.gather;
        uint8_t* h;
        if ((rc = stage_get(c->main, fg.total + 64, &h))) return rc;
        if (!c->aux) HIP_TRY(hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
        if (!c->gev) HIP_TRY(hipEventCreateWithFlags(&c->gev, hipEventDisableTiming));
        const uint32_t chunks = fg.R >= 256 ? 4 : 1;
        uint64_t sent = 0;
        for (uint32_t k = 0; k < chunks; ++k) {
            const uint32_t r0 = (uint32_t)((uint64_t)fg.R * k / chunks), r1 = (uint32_t)((uint64_t)fg.R * (k + 1) / chunks);
            for (uint32_t r = r0; r < r1; ++r) {
                // two scattered objects per claim (its record, its filter bytes): touch those of the claim
                // kPrefetch ahead so their misses overlap this claim's copy
                constexpr uint32_t kPrefetch = 6;
                if (r + kPrefetch < fg.R) {
                    const uint8_t* nf = (const uint8_t*)(uintptr_t)fg.refs[2 * (size_t)(r + kPrefetch) + 1];
                    __builtin_prefetch((const void*)(uintptr_t)fg.refs[2 * (size_t)(r + kPrefetch)]);
                    __builtin_prefetch(nf);
                    __builtin_prefetch(nf + 64);
                }
                const uint64_t n = ((const dsy_request*)(uintptr_t)fg.refs[2 * (size_t)r])->m_bits / 8;
                uint8_t* dst = h + fg.foff[r];
                memcpy(dst, (const void*)(uintptr_t)fg.refs[2 * (size_t)r + 1], n);
                memset(dst + n, 0, ((n + 3) & ~uint64_t(3)) - n);
            }
            const uint64_t upto = k + 1 == chunks ? fg.total + 64 : fg.foff[r1];
            if (k + 1 == chunks) memset(h + fg.total, 0, 64);
            if (upto > sent) HIP_TRY(hipMemcpyAsync(fg.d_dst + sent, h + sent, upto - sent, hipMemcpyHostToDevice, c->aux));
            sent = upto;
        }
        HIP_TRY(hipEventRecord(c->gev, c->aux));
        HIP_TRY(hipStreamWaitEvent(st, c->gev, 0));
        fg = FilterGather{};
    }
    if (fill_profile) {  // per-window stderr line: k_fill phase durations over the workgroups (s_memtime ticks)
        std::vector<uint64_t> fc(n_act * 4);
        HIP_TRY(hipMemcpyAsync(fc.data(), d_fc, n_act * 32, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        uint64_t t0 = ~0ull, t2 = 0, sel = 0, srt = 0, stp = 0, mx_sel = 0, mx_srt = 0, mx_stp = 0, n = 0;
        for (size_t a = 0; a < n_act; ++a) {
            if (!fc[a * 4]) continue;
            t0 = std::min(t0, fc[a * 4 + 3]);
            t2 = std::max(t2, fc[a * 4 + 2]);
            stp += fc[a * 4] - fc[a * 4 + 3];
            sel += fc[a * 4 + 1] - fc[a * 4];
            srt += fc[a * 4 + 2] - fc[a * 4 + 1];
            mx_stp = std::max(mx_stp, fc[a * 4] - fc[a * 4 + 3]);
            mx_sel = std::max(mx_sel, fc[a * 4 + 1] - fc[a * 4]);
            mx_srt = std::max(mx_srt, fc[a * 4 + 2] - fc[a * 4 + 1]);
            ++n;
        }
        // shader-clock ticks; setup = k_fill_first's host reads + plan (0 for k_fill)
        if (n) fprintf(stderr, "fill_profile n=%llu span=%llu setup avg=%llu max=%llu select avg=%llu max=%llu "
                       "sort avg=%llu max=%llu\n", (unsigned long long)n, (unsigned long long)(t2 - t0),
                       (unsigned long long)(stp / n), (unsigned long long)mx_stp, (unsigned long long)(sel / n),
                       (unsigned long long)mx_sel, (unsigned long long)(srt / n), (unsigned long long)mx_srt);
        L.fill_clock = nullptr;
    }
    // DSY_PAIR_TRACE=<path>: every window's wave-task records are appended to <path> (WaveTrace, 32 B each, after a
    // 16-byte header {records, window, kernel start/end unknown}); diagnostics only, the window waits for them
    static const char* trace_path = getenv("DSY_PAIR_TRACE");
    void* d_tr = nullptr;
    const uint32_t trace_cap = 1u << 20;
    if (trace_path) {
        if ((rc = ws_get(sl.w, "pair_trace", (size_t)trace_cap * sizeof(WaveTrace) + 64, &d_tr))) return rc;
        HIP_TRY(hipMemsetAsync(d_tr, 0, 64, st));
        L.trace_n = (uint32_t*)d_tr;
        L.trace = (WaveTrace*)((uint8_t*)d_tr + 64);
        L.trace_cap = trace_cap;
    }
    for (size_t f = 0; f < jb.fam_active.size(); ++f) {
        if (!runs[f].second) continue;
        const int fid = jb.fam_id[f];
        const int kc = fid / 2;
        const uint32_t chunk = kc % 3 == 0 ? 2 : kc % 3 == 1 ? 4 : 8;
        if ((L.pool_mask >> fid) & 1u) {
            // (a pooled wave mixes claims: the padded messages only when every claim of the family has a 1-byte prefix)
            size_t p1 = 0;
            if (fid % 2 == 0)
                for (uint32_t r : jb.fam_active[f]) p1 += jb.pad1[r];
            timer_dispatch(c, &t, kTimePairTest, &L.ev_start, &L.ev_stop);
            HIP_TRY(launch_pair_test_pooled(L, kc / 3, chunk, fid % 2 == 1, p1 == runs[f].second, (uint32_t)fid,
                                            jb.d_slots + runs[f].first, (uint32_t)runs[f].second));
            timer_dispatched(c, &t);
            L.ev_start = L.ev_stop = nullptr;
            continue;
        }
        // the family's 1-byte-prefix claims lead its run (job_start): one launch over the padded messages, one over
        // the rest
        size_t n1 = 0;
        if (fid % 2 == 0)
            for (uint32_t r : jb.fam_active[f]) n1 += jb.pad1[r];
        const size_t part[2] = {n1, runs[f].second - n1};
        for (int k = 0; k < 2; ++k) {
            if (!part[k]) continue;
            timer_dispatch(c, &t, kTimePairTest, &L.ev_start, &L.ev_stop);
            HIP_TRY(launch_pair_test_list(L, kc / 3, chunk, fid % 2 == 1, k == 0,
                                          jb.d_slots + runs[f].first + (k ? n1 : 0), (uint32_t)part[k]));
            timer_dispatched(c, &t);
            L.ev_start = L.ev_stop = nullptr;
        }
    }
    if (trace_path) {
        uint32_t n = 0;
        HIP_TRY(hipMemcpyAsync(&n, d_tr, 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        n = std::min(n, trace_cap);
        std::vector<WaveTrace> rec(n);
        if (n) HIP_TRY(hipMemcpyAsync(rec.data(), L.trace, (size_t)n * sizeof(WaveTrace), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (FILE* fp = fopen(trace_path, "ab")) {
            const uint64_t head[2] = {n, L.window};
            fwrite(head, 8, 2, fp);
            if (n) fwrite(rec.data(), sizeof(WaveTrace), n, fp);
            fclose(fp);
        }
        L.trace = nullptr;
        L.trace_n = nullptr;
    }
    timer_begin(c, &t, kTimeCompact, st);
    HIP_TRY(launch_compact(L));
    timer_end(c, &t, st);
    // speculatively pack the output now (it is redone if another window follows): the GPU packs while the host wakes
    // up and reads the status
    static const bool ev_marker = getenv("DSY_EVENT_MARKER") != nullptr;  // A/B: the event as a separate record
    HIP_TRY(launch_pack(L, (uint64_t*)jb.d_packed, (uint64_t*)jb.d_packed_off, nullptr, ev_marker ? nullptr : sl.ev_done));
    ++jb.windows;
    if (ev_marker) HIP_TRY(hipEventRecord(sl.ev_done, st));
    if (g_host_profile && !jb.hp[2]) jb.hp[2] = host_us();  // first window enqueued
    return DSY_OK;
}

// The claims of a responder call as job_start reads them: an array of dsy_request records, or (dsy_sync_respond_refs)
// per claim its range (ranges[4r .. 4r+3]: time_low, time_high, modulo, offset) and the address of a record that
// carries its filter's shape and prefix (refs[2r]), with the filter offsets the library laid out (foff).
struct Claims {
    const dsy_request* reqs = nullptr;
    const uint64_t* ranges = nullptr;
    const uint64_t* refs = nullptr;
    const uint64_t* foff = nullptr;
    const dsy_request& shape(uint32_t r) const {
        return reqs ? reqs[r] : *(const dsy_request*)(uintptr_t)refs[2 * (size_t)r];
    }
    uint64_t field(uint32_t r, int i) const { return ranges[4 * (size_t)r + i]; }
    uint64_t time_low(uint32_t r) const { return reqs ? reqs[r].time_low : std::min<uint64_t>(field(r, 0), kMaxGtHost); }
    uint64_t time_high(uint32_t r) const { return reqs ? reqs[r].time_high : std::min<uint64_t>(field(r, 1), kMaxGtHost); }
    uint64_t modulo(uint32_t r) const { return reqs ? reqs[r].modulo : field(r, 2); }
    uint64_t offset(uint32_t r) const { return reqs ? reqs[r].offset : field(r, 3); }
    uint64_t filter_offset(uint32_t r) const { return reqs ? reqs[r].filter_offset : foff[r]; }
    static constexpr uint64_t kMaxGtHost = 0x7fffffffffffffffull;  // community.py:2545-2548
};

// Validate and stage a batch of claims into slot sl and enqueue its first window (no host wait).
static int job_start(dsy_ctx* c, RespondSlot& sl, const dsy_store* s, const Claims& cl, uint32_t R,
                     const uint8_t* d_filters, uint64_t filters_len, const dsy_meta* metas, uint32_t J,
                     uint64_t responder_gt, int include_inactive, int64_t byte_limit, uint64_t seed) {
    sl.job = RespondJob{};
    RespondJob& jb = sl.job;
    const hipStream_t st = c->stream;
    if (!sl.ev_done) HIP_TRY(hipEventCreate(&sl.ev_done));  // (recorded by a dispatch: hipExtLaunchKernelGGL)
    if (int rc = store_flush(c, s)) return rc;  // rows appended since the last read join the index first
    if (g_host_profile) jb.hp[0] = host_us();
    // ---- validate claims (payload.py:89-101, conversion.py:772-789) and their filters; group them by hash family
    // (kind x chunk width: one pair-test launch per family)
    // family id = (kind * 3 + chunk class) * 2 + long prefix (> 4 bytes: the byte-wise hashing path)
    std::vector<uint32_t> fam_members[kFamilies];
    uint64_t memo_m = 0;  // check_family of the previous claim's (m, k): a batch's claims share one filter shape
    uint32_t memo_k = 0, memo_chunk = 0;
    int32_t memo_kind = -1;
    for (uint32_t r = 0; r < R; ++r) {
        const dsy_request& q = cl.shape(r);
        const uint64_t q_modulo = cl.modulo(r), q_offset = cl.offset(r);
        if (q_modulo == 0 || q_offset >= q_modulo || q_modulo > 0xffffffffull)
            return fail(DSY_EINVAL, "claim %u: need 0 <= offset < modulo < 2^32 (offset=%llu modulo=%llu)", r,
                        (unsigned long long)q_offset, (unsigned long long)q_modulo);
        int32_t kind;
        uint32_t chunk;
        if (memo_kind >= 0 && q.m_bits == memo_m && q.k == memo_k) {
            kind = memo_kind;
            chunk = memo_chunk;
        } else {
            int rc = check_family(q.m_bits, q.k, &kind, &chunk);
            if (rc) return rc;
            memo_m = q.m_bits, memo_k = q.k, memo_kind = kind, memo_chunk = chunk;
        }
        if (kind != q.hash_kind || chunk != q.chunk_bytes) return fail(DSY_EINVAL, "claim %u: hash family mismatch", r);
        if (q.prefix_len > 255) return fail(DSY_EINVAL, "claim %u: prefix too long", r);
        const uint64_t q_foff = cl.filter_offset(r);
        if (q_foff % 4) return fail(DSY_EINVAL, "claim %u: filter_offset must be a multiple of 4", r);
        if (filters_len && q_foff + filter_words(q.m_bits) * 4 > filters_len)
            return fail(DSY_EINVAL, "claim %u: filter beyond the filters buffer", r);
        // prefixes of 1-4 bytes take the line-staged hashing; longer ones and the empty prefix the byte-wise path
        std::vector<uint32_t>& fm =
            fam_members[(kind * 3 + (chunk == 2 ? 0 : chunk == 4 ? 1 : 2)) * 2 + (q.prefix_len > 4 || q.prefix_len == 0)];
        if (fm.empty()) fm.reserve(R);
        fm.push_back(r);
    }
    // within a line-staged family, the claims of 1-byte prefixes (every reference claim) come first: their run hashes
    // the line copy's padded messages (one launch), the 2-4-byte prefixes' run shifts and masks (another)
    jb.pad1.assign(R, 0);
    for (uint32_t r = 0; r < R; ++r) jb.pad1[r] = cl.shape(r).prefix_len == 1;
    for (int f = 0; f < kFamilies; f += 2)
        std::stable_partition(fam_members[f].begin(), fam_members[f].end(), [&](uint32_t r) { return jb.pad1[r] != 0; });
    for (uint32_t j = 0; j < J; ++j)
        if (metas[j].direction < DSY_ASC || metas[j].direction > DSY_RANDOM)
            return fail(DSY_EINVAL, "meta %u: unknown synchronization direction %d", j, metas[j].direction);
    jb.R = R;
    jb.J = J;
    jb.s = s;
    jb.pool = kWindow * std::max<uint64_t>(R, kMinSlots);
    const uint64_t pool = jb.pool;
    // ---- device layout: one upload region [claims | metas | window slots 0..R-1 | first active list] and one
    // device status region [counters kCntSpread x 64 B | flags 64 B | upper R x u64] (counters and flags zeroed by
    // k_setup); host-mapped status [totals kCntN x u64 | overflow | act_done R B]: k_compact writes the done flags
    // and the overflow flag over the bus and the pack kernel folds the counters, so a window's status needs no
    // copy dispatch
    size_t prefix_b = 0;
    for (uint32_t r = 0; r < R; ++r) prefix_b += cl.shape(r).prefix_len;
    const size_t reqs_b = (size_t)R * sizeof(DevRequest), metas_b = (size_t)J * sizeof(SegMeta);
    const size_t in_b = (reqs_b + metas_b + (size_t)R * 8 + (prefix_b + 15) / 16 * 16 + 64 + 15) / 16 * 16;
    const size_t act_done_b = ((size_t)R + 15) / 16 * 16;
    const size_t cnt_b = kCntSpread * kCntN * 8, head_b = cnt_b + 64;
    const size_t io_b = head_b + (size_t)R * 8;
    constexpr size_t kHostHead = 128;
    jb.in_b = in_b;
    jb.cnt_b = cnt_b;
    int rc;
    void *d_in, *d_io, *d_plans, *d_state, *d_emit, *d_ticket;
    Workspace& w = sl.w;
    if ((rc = ws_get(w, "resp_in", in_b, &d_in))) return rc;
    if ((rc = ws_get(w, "emitted_n", std::max<size_t>(R, 1) * 8, &d_emit))) return rc;
    bool fresh = false;
    if ((rc = ws_get(w, "ticket", 64, &d_ticket, &fresh))) return rc;
    if (fresh) HIP_TRY(hipMemsetAsync(d_ticket, 0, 64, st));
    bool io_fresh = false;
    if ((rc = ws_get(w, "resp_io", io_b, &d_io, &io_fresh))) return rc;
    if (io_fresh) HIP_TRY(hipMemsetAsync(d_io, 0, io_b, st));  // flags start (and stay, k_compact) at zero
    if ((rc = ws_get(w, "plans", std::max<size_t>((size_t)R * J, 1) * sizeof(Plan), &d_plans))) return rc;
    if ((rc = ws_get(w, "state", std::max<size_t>(R, 1) * sizeof(ReqState), &d_state))) return rc;
    // split windows' sort state: [R][kSortBins] histogram + cursors, zeroed by the call's first kernel (k_setup or
    // k_fill_first) and kept zero between windows by k_compact
    void* d_bulk;
    const size_t bulk_b = (size_t)std::max<uint32_t>(R, 1) * 2 * 1024 * 4;
    if ((rc = ws_get(w, "bulk_sort", bulk_b, &d_bulk))) return rc;
    // pooled families (c->pool_kinds): the pooled order and the families' counts (zero outside a window)
    uint32_t pool_mask = 0;
    if (!c->pair_diag && pool <= 0xffffffffull)
        for (int f = 0; f < kFamilies; ++f)
            if (!fam_members[f].empty() && ((c->pool_kinds >> (f / 6)) & 1u)) pool_mask |= 1u << f;
    void* d_pool_counts = nullptr;
    void* d_pool_tab = nullptr;
    if (pool_mask) {
        if ((rc = ws_get(w, "pool_counts", sizeof(PoolCounts), &d_pool_counts))) return rc;
        // the per-(claim, bin) counts and offsets: every row a pooled window reads is written by that window's k_fill
        if (c->pool_scan && (rc = ws_get(w, "pool_tab", (size_t)std::max<uint32_t>(R, 1) * 2 * kPoolBins * 4, &d_pool_tab)))
            return rc;
        // every call starts from zero counts (k_pair_test<POOL> keeps them zero between windows; a call that ended
        // early may have left some)
        HIP_TRY(hipMemsetAsync(d_pool_counts, 0, sizeof(PoolCounts), st));
    }
    uint8_t* h_in;
    if ((rc = stage_get(w, in_b + kHostHead + act_done_b + (size_t)R * 4, &h_in))) return rc;
    jb.h_in = h_in;
    jb.d_in = d_in;
    jb.d_io = d_io;
    uint8_t* h_io = h_in + in_b;  // host-mapped status
    jb.h_io = h_io;
    jb.h_act_next = (uint32_t*)(h_io + kHostHead + act_done_b);
    jb.windows = 0;
    std::memset(h_io, 0, kHostHead);  // totals stay zero if no window runs (R == 0)
    {
        DevRequest* dq = (DevRequest*)h_in;
        uint8_t* h_pre = h_in + reqs_b + metas_b + (size_t)R * 8;
        const uint8_t* d_pre = (const uint8_t*)d_in + reqs_b + metas_b + (size_t)R * 8;
        size_t at = 0;
        for (uint32_t r = 0; r < R; ++r) {
            const dsy_request& q = cl.shape(r);
            DevRequest d;
            d.time_low = cl.time_low(r);
            d.time_high = cl.time_high(r);
            d.filter_offset = cl.filter_offset(r);
            d.m_bits = q.m_bits;
            d.modulo = (uint32_t)cl.modulo(r);
            d.offset = (uint32_t)cl.offset(r);
            d.k = q.k;
            d.hash_kind = (uint32_t)q.hash_kind;
            d.chunk_bytes = q.chunk_bytes;
            d.prefix_len = q.prefix_len;
            d.prefix = d_pre + at;
            d.prefix_word = 0;
            for (uint32_t j = 0; j < std::min<uint32_t>(q.prefix_len, 4); ++j) d.prefix_word |= (uint32_t)q.prefix[j] << (8 * j);
            d.m_recip = mod_recip(q.m_bits);
            d.pad[0] = d.pad[1] = 0;
            std::memcpy(h_pre + at, q.prefix, q.prefix_len);
            at += q.prefix_len;
            dq[r] = d;
        }
    }
    SegMeta* sm = (SegMeta*)(h_in + reqs_b);
    for (uint32_t j = 0; j < J; ++j) {
        auto it = s->segs.find(metas[j].meta_id);
        SegMeta m{};
        m.seg_a = it == s->segs.end() ? 0 : it->second.first;
        m.seg_b = it == s->segs.end() ? 0 : it->second.second;
        m.dir = (uint32_t)metas[j].direction;
        m.has_pruning = metas[j].has_pruning;
        m.inactive = metas[j].inactive_threshold;
        sm[j] = m;
    }
    uint32_t* h_slots = (uint32_t*)(h_in + reqs_b + metas_b);
    uint32_t* h_act0 = h_slots + R;
    jb.h_act0 = h_act0;
    // the active list, family by family (a family's active claims occupy a contiguous run of slots)
    for (int f = 0; f < kFamilies; ++f)
        if (!fam_members[f].empty()) {
            jb.fam_active.push_back(std::move(fam_members[f]));
            jb.fam_id.push_back(f);
        }
    {
        uint32_t a = 0;
        for (uint32_t i = 0; i < R; ++i) h_slots[i] = i;
        for (auto& fa : jb.fam_active)
            for (uint32_t r : fa) {
                jb.act0_identity &= r == a;
                h_act0[a++] = r;
            }
    }
    uint8_t* io = (uint8_t*)d_io;
    if (g_host_profile) jb.hp[1] = host_us();  // claims validated and staged

    RespondLaunch& L = jb.L;
    L.st.max_len = s->max_len;
    L.st.lines = s->d_lines;
    L.st.rec = s->d_rec;
    L.st.live_gt = s->d_live_gt;
    L.st.live_row = s->d_live_row;
    L.st.n_live = s->n_live;
    L.st.lines_bytes = s->lines_cap;
    L.reqs = (const DevRequest*)d_in;
    L.metas = (const SegMeta*)((uint8_t*)d_in + reqs_b);
    jb.d_slots = (const uint32_t*)((uint8_t*)d_in + reqs_b + metas_b);
    jb.d_act = (uint32_t*)(jb.d_slots + R);
    L.R = R;
    L.J = J;
    L.filters = d_filters;
    L.responder_gt = responder_gt;
    L.include_inactive = include_inactive;
    L.byte_limit = byte_limit;
    L.seed = seed;
    L.window = kWindow;
    L.act = jb.d_act;
    L.act_done = h_io + kHostHead;
    L.h_status = (uint64_t*)h_io;
    L.plans = (Plan*)d_plans;
    L.state = (ReqState*)d_state;
    L.upper = (uint64_t*)(io + head_b);
    L.emitted_n = (uint64_t*)d_emit;
    L.ticket = (uint32_t*)d_ticket;
    L.bulk_hist = (uint32_t*)d_bulk;
    L.bulk_cur = (uint32_t*)d_bulk + (size_t)std::max<uint32_t>(R, 1) * 1024;
    L.flags = (uint32_t*)(io + cnt_b);
    L.counters = (uint64_t*)io;
    L.stream = st;
    L.diag = c->pair_diag;
    L.direct_kinds = c->direct_kinds;
    L.grid_cap = c->pair_grid ? c->pair_grid : c->max_grid;
    L.pool_mask = pool_mask;
    L.pool_queue = c->pool_queue;
    L.pool_deal = c->pool_deal;
    L.pool_scan = c->pool_scan && d_pool_tab;
    L.pool_tab = (uint32_t*)d_pool_tab;
    L.pair_prio = c->pair_prio;
    L.bulk_zero = c->bulk_zero;
    L.pool_counts = (PoolCounts*)d_pool_counts;
    if ((rc = job_pair_buffers(sl, pool))) return rc;

    // ---- per-claim output capacity: every emitted packet but the last costs >= min_len bytes of budget, so a
    // claim sends at most byte_limit / min_len + 2 packets.  When that bound is small the capacities and output
    // bases are computed on the device (no host round-trip); otherwise from the plan's row counts on the host.
    // k_setup reads the staged claims straight from pinned host memory (its copy to d_in is what later kernels
    // read) and zeroes the status counters: no copy-engine or fill dispatch ahead of it.
    void* d_out;
    uint64_t cap_total = 0;
    const uint64_t per_claim = byte_limit <= 0 ? 1 : (s->min_len > 0 ? (uint64_t)byte_limit / s->min_len + 2 : ~0ull);
    const bool dev_caps = per_claim != ~0ull && per_claim <= (1ull << 26) / std::max<uint32_t>(R, 1);
    jb.per_claim = per_claim;
    PendingTimer t;
    // one meta and device-side capacities (the common case): the setup runs inside the first window's fill
    // (k_fill_first); otherwise k_setup plans every (claim, meta) first
    jb.fused_first = J == 1 && dev_caps && R > 0;
    if (!jb.fused_first) {
        timer_begin(c, &t, kTimeSelect, st);
        HIP_TRY(launch_setup(L, h_in, d_in, in_b, d_io, head_b, dev_caps ? per_claim : 0));
        timer_end(c, &t, st);
    }
    if (dev_caps) {
        cap_total = per_claim * R;
        if ((rc = ws_get(w, "out", std::max<uint64_t>(cap_total, 1) * 8, &d_out))) return rc;
        L.out = (uint64_t*)d_out;
    } else {
        std::vector<uint64_t> upper(R);
        if (R) HIP_TRY(hipMemcpyAsync(upper.data(), L.upper, (size_t)R * 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        std::vector<ReqState> rst(R);
        for (uint32_t r = 0; r < R; ++r) {
            rst[r] = ReqState{};
            rst[r].cap = std::min<uint64_t>(upper[r], per_claim);
            rst[r].out_base = cap_total;
            rst[r].done = upper[r] == 0;
            cap_total += rst[r].cap;
        }
        if ((rc = ws_get(w, "out", std::max<uint64_t>(cap_total, 1) * 8, &d_out))) return rc;
        L.out = (uint64_t*)d_out;
        if (R) {
            HIP_TRY(hipMemcpyAsync(d_state, rst.data(), (size_t)R * sizeof(ReqState), hipMemcpyHostToDevice, st));
            HIP_TRY(hipStreamSynchronize(st));  // rst is pageable and goes out of scope
        }
    }
    L.packed_cap = cap_total;
    const size_t b_pin = ((size_t)R + 1) * 8 + std::max<uint64_t>(cap_total, 1) * 8;
    if (c->host_out && b_pin <= kOutPinMax) {  // results straight into pinned host memory
        if (c->out_pin_bytes < b_pin) {
            if (c->out_pin) hipHostFree(c->out_pin);
            c->out_pin = nullptr;
            c->out_pin_bytes = 0;
            const size_t want = std::max<size_t>(b_pin + b_pin / 4, 1 << 16);
            if (hipHostMalloc((void**)&c->out_pin, want, hipHostMallocDefault) != hipSuccess) {
                c->out_pin = nullptr;
                return fail(DSY_ENOMEM, "hipHostMalloc(%zu) for the responder's results failed", want);
            }
            c->out_pin_bytes = want;
        }
        jb.d_packed_off = c->out_pin;
        jb.d_packed = c->out_pin + ((size_t)R + 1) * 8;
    } else {
        if ((rc = ws_get(w, "packed", std::max<uint64_t>(cap_total, 1) * 8, &jb.d_packed))) return rc;
        if ((rc = ws_get(w, "packed_off", ((size_t)R + 1) * 8, &jb.d_packed_off))) return rc;
    }
    size_t n_act = 0;
    for (auto& fa : jb.fam_active) n_act += fa.size();
    if (n_act) return job_window(c, sl);
    return DSY_OK;
}

// The host-mapped status a window's kernels leave: the output-capacity overflow flag (k_compact) and the bounds
// checks (kStatusGuard: an index the responder computed fell outside its buffer; the access was skipped).
static int job_status(const RespondJob& jb) {
    const volatile uint64_t* h = (const volatile uint64_t*)jb.h_io;
    if (h[kStatusOverflow]) return fail(DSY_ECAPACITY, "internal: a claim overflowed its output capacity");
    if (const uint64_t g = h[kStatusGuard]) {
        static const char* what[] = {"k_fill_sort placed a pair past its window", "k_pair_test read a task record "
                                     "naming a packet outside the line copy", "k_pack's output overflowed the "
                                     "packed buffer", "a window held more pairs than W"};
        for (int b = 0; b < 4; ++b)
            if ((g >> (8 * b)) & 0xff) return fail(DSY_EINTERNAL, "internal: bounds check tripped: %s", what[b]);
        return fail(DSY_EINTERNAL, "internal: bounds check tripped (0x%llx)", (unsigned long long)g);
    }
    return DSY_OK;
}

// A window's status check failed: when k_pair_test's task-record check tripped, audit the window's task records
// (k_task_audit: the window's state and records are intact until the next window) and name the first bad one.
static int job_status_audit(dsy_ctx* c, RespondSlot& sl, int rc) {
    const RespondJob& jb = sl.job;
    const uint64_t g = ((const volatile uint64_t*)jb.h_io)[kStatusGuard];
    if (!((g >> (8 * kGuardTask)) & 0xff)) return rc;
    const std::string first = dsy_last_error();
    void* d_out;
    if (ws_get(sl.w, "task_audit", 128, &d_out)) return rc;
    unsigned long long h[10] = {};
    if (hipMemsetAsync(d_out, 0, 80, c->stream) != hipSuccess || launch_task_audit(jb.L, (unsigned long long*)d_out) ||
        hipMemcpyAsync(h, d_out, 80, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        return rc;
    // that claim's records and state on the host: which slots are missing, which are placed twice, and the window's
    // path (split part / slice / one workgroup) from its cursor and plan
    std::string more;
    const uint64_t a = h[1], r = h[2], n = h[4], W = h[8];
    if (h[0] && n && n <= (1ull << 22)) {
        std::vector<PairTask> tk(n);
        ReqState S{};
        Plan P{};
        if (hipMemcpyAsync(tk.data(), jb.L.task + a * W, n * sizeof(PairTask), hipMemcpyDeviceToHost, c->stream) ==
                hipSuccess &&
            hipMemcpyAsync(&S, jb.L.state + r, sizeof S, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
            hipStreamSynchronize(c->stream) == hipSuccess) {
            if (S.win_meta < jb.J)
                (void)hipMemcpy(&P, jb.L.plans + r * jb.J + S.win_meta, sizeof P, hipMemcpyDeviceToHost);
            std::vector<uint32_t> seen(n, 0);
            uint64_t stale = 0, dup = 0, first_stale = ~0ull, last_stale = 0;
            for (uint64_t i = 0; i < n; ++i) {
                if (tk[i].slot >= n) {
                    ++stale;
                    first_stale = std::min(first_stale, i);
                    last_stale = i;
                } else if (seen[tk[i].slot]++) {
                    ++dup;
                }
            }
            uint64_t missing = 0, first_missing = ~0ull;
            for (uint64_t t = 0; t < n; ++t)
                if (!seen[t]) {
                    ++missing;
                    first_missing = std::min(first_missing, t);
                }
            char buf[512];
            snprintf(buf, sizeof buf, "; claim %llu: %llu stale positions [%llu..%llu], %llu slots placed twice, %llu "
                     "missing (first %llu); state meta %u cand %llu sub %llu win %u/%llu/%llu exhausted %u done %u; plan "
                     "mode %u dir %u ncand %llu dense %u span %llu..%llu",
                     (unsigned long long)r, (unsigned long long)stale, (unsigned long long)first_stale,
                     (unsigned long long)last_stale, (unsigned long long)dup, (unsigned long long)missing,
                     (unsigned long long)first_missing, S.meta, (unsigned long long)S.cand, (unsigned long long)S.sub,
                     S.win_meta, (unsigned long long)S.win_cand, (unsigned long long)S.win_sub, S.exhausted, S.done,
                     P.mode, P.dir, (unsigned long long)P.ncand, P.dense, (unsigned long long)P.a, (unsigned long long)P.b);
            more = buf;
        }
    }
    return fail(DSY_EINTERNAL, "%s; audit: %llu bad task records in %llu claims, e.g. window slot %llu (claim %llu) "
                "record %llu of n_window %llu: off %llu len %llu slot %llu (W %llu, line copy %llu B, call R %u J %u, "
                "window %llu)%s",
                first.c_str(), h[0], h[9], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8],
                (unsigned long long)jb.L.st.lines_bytes, jb.R, jb.J, (unsigned long long)jb.windows, more.c_str());
}

// Wait for the job's windows, run the further windows its unfinished claims need, and return its results.
static int job_finish(dsy_ctx* c, RespondSlot& sl, uint64_t** d_packed, uint64_t** d_packed_off, uint64_t* total_pairs) {
    RespondJob& jb = sl.job;
    RespondLaunch& L = jb.L;
    const hipStream_t st = c->stream;
    constexpr size_t kHostHead = 128;
    for (;;) {
        size_t n_act = 0;
        for (auto& fa : jb.fam_active) n_act += fa.size();
        if (!n_act) break;
        const double w0 = g_host_profile ? host_us() : 0.0;
        HIP_TRY(hipEventSynchronize(sl.ev_done));  // this job's window, not what later batches queued behind it
        if (g_host_profile) jb.hp_wait += host_us() - w0;
        // the window's status must be the one its pack kernel numbered: a status read before it is visible would
        // steer the next window (its claims, and the host's reuse of the staging) from the previous window's state
        if (((const volatile uint64_t*)jb.h_io)[kStatusSeq] != jb.windows) {
            HIP_TRY(hipStreamSynchronize(st));
            const uint64_t seq = ((const volatile uint64_t*)jb.h_io)[kStatusSeq];
            static bool noted = false;
            if (!noted) {
                noted = true;
                fprintf(stderr, "dsybloom: window %llu's status was not visible at its completion event (seq %llu); "
                        "synchronised the stream\n", (unsigned long long)jb.windows, (unsigned long long)seq);
            }
            if (seq != jb.windows)
                return fail(DSY_EINTERNAL, "internal: window %llu's status not visible after a stream synchronise "
                            "(seq %llu)", (unsigned long long)jb.windows, (unsigned long long)seq);
        }
        // capacity overflow can only come from a wrong min_len bound; report it loudly
        if (int rc = job_status(jb)) return job_status_audit(c, sl, rc);
        const volatile uint8_t* done = jb.h_io + kHostHead;
        size_t a = 0, left = 0;
        for (auto& fa : jb.fam_active) {
            size_t keep = 0;
            for (uint32_t r : fa)
                if (!done[a++]) fa[keep++] = r;
            fa.resize(keep);
            left += keep;
        }
        if (!left) break;
        int rc = job_window(c, sl);
        if (rc) return rc;
    }
    uint64_t h_tot[kCntN];
    if (!jb.ran) {
        HIP_TRY(launch_pack(L, (uint64_t*)jb.d_packed, (uint64_t*)jb.d_packed_off, nullptr));
        HIP_TRY(hipStreamSynchronize(st));
        if (int rc = job_status(jb)) return rc;
    }
    for (uint32_t k = 0; k < kCntN; ++k) h_tot[k] = ((const volatile uint64_t*)jb.h_io)[k];
    timers_collect_lazy(c);
    c->blocks[kTimePairTest] += h_tot[kCntBlocks];
    c->bytes[kTimePairTest] += h_tot[kCntBytes];
    c->useful[kTimePairTest] += h_tot[kCntUseful];
    c->slots[kTimePairTest] += h_tot[kCntSlots];
    *total_pairs = h_tot[kCntPairs];
    *d_packed = (uint64_t*)jb.d_packed;
    *d_packed_off = (uint64_t*)jb.d_packed_off;
    if (g_host_profile) {
        jb.hp[3] = host_us();
        fprintf(stderr, "host_profile R=%u stage=%.1f enqueue=%.1f wait=%.1f total=%.1f\n", jb.R, jb.hp[1] - jb.hp[0],
                jb.hp[2] ? jb.hp[2] - jb.hp[1] : 0.0, jb.hp_wait, jb.hp[3] - jb.hp[0]);
    }
    // DSY_BULK_AUDIT (diagnostic): the split windows' sort state must be zero once a call's windows are done
    // (k_compact clears what each window used); one stderr line per call that leaves counts behind
    static const bool bulk_audit = getenv("DSY_BULK_AUDIT") != nullptr;
    if (bulk_audit && jb.R) {
        const size_t n = (size_t)jb.R * 1024;
        std::vector<uint32_t> h(2 * n);
        HIP_TRY(hipMemcpyAsync(h.data(), L.bulk_hist, n * 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(h.data() + n, L.bulk_cur, n * 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        std::string msg;
        size_t dirty = 0;
        for (size_t part = 0; part < 2; ++part)
            for (uint32_t a = 0; a < jb.R; ++a) {
                uint64_t sum = 0, nz = 0;
                for (uint32_t i = 0; i < 1024; ++i) {
                    sum += h[part * n + (size_t)a * 1024 + i];
                    nz += h[part * n + (size_t)a * 1024 + i] != 0;
                }
                if (!nz) continue;
                if (++dirty <= 16)
                    msg += std::string(part ? " cur" : " hist") + "[" + std::to_string(a) + "]=" + std::to_string(sum) +
                           "/" + std::to_string(nz);
            }
        if (dirty)
            fprintf(stderr, "bulk_audit R=%u J=%u W_last=%llu dirty_rows=%zu:%s\n", jb.R, jb.J,
                    (unsigned long long)L.window, dirty, msg.c_str());
    }
    return DSY_OK;
}

static RespondSlot& sync_slot(dsy_ctx* c) { return c->rs[0]; }

static int respond_core(dsy_ctx* c, const dsy_store* s, const Claims& cl, uint32_t R, const uint8_t* d_filters,
                        uint64_t filters_len, const dsy_meta* metas, uint32_t J, uint64_t responder_gt,
                        int include_inactive, int64_t byte_limit, uint64_t seed, uint64_t** d_packed,
                        uint64_t** d_packed_off, uint64_t* total_pairs) {
    if (c->inflight()) return fail(DSY_EINVAL, "submitted responder batches are in flight: dsy_sync_respond_wait them first");
    RespondSlot& sl = sync_slot(c);
    sl.last_use = ++c->use_clock;
    int rc = job_start(c, sl, s, cl, R, d_filters, filters_len, metas, J, responder_gt, include_inactive, byte_limit,
                       seed);
    if (rc) return rc;
    return job_finish(c, sl, d_packed, d_packed_off, total_pairs);
}

// the device step of a host-buffer call and its result download, the filters in the "filters" workspace (or, with
// jb.gather set by the caller, gathered there behind the first window's selection)
static int respond_to_host(dsy_ctx* c, const dsy_store* s, const Claims& cl, uint32_t R, const void* d_f,
                           uint64_t filters_len, const dsy_meta* metas, uint32_t nmeta, uint64_t responder_global_time,
                           int include_inactive, int64_t byte_limit, uint64_t random_seed, uint64_t* out_idx,
                           uint64_t out_cap, uint64_t* out_req_offsets) {
    int rc;
    uint64_t *d_packed, *d_off, pairs;
    c->host_out = true;
    rc = respond_core(c, s, cl, R, (const uint8_t*)d_f, filters_len + 64, metas, nmeta, responder_global_time,
                      include_inactive, byte_limit, random_seed, &d_packed, &d_off, &pairs);
    c->host_out = false;
    if (rc) return rc;
    if ((uint8_t*)d_off == c->out_pin) {  // written by the pack kernel into pinned memory; the step has completed
        HIP_TRY(hipStreamSynchronize(c->stream));
        std::memcpy(out_req_offsets, d_off, ((size_t)R + 1) * 8);
        const uint64_t total = out_req_offsets[R];
        if (total > out_cap) return fail(DSY_ECAPACITY, "out_cap %llu < %llu rows", (unsigned long long)out_cap, (unsigned long long)total);
        std::memcpy(out_idx, d_packed, total * 8);
        return DSY_OK;
    }
    HIP_TRY(hipMemcpyAsync(out_req_offsets, d_off, ((size_t)R + 1) * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    const uint64_t total = out_req_offsets[R];
    if (total > out_cap) return fail(DSY_ECAPACITY, "out_cap %llu < %llu rows", (unsigned long long)out_cap, (unsigned long long)total);
    if (total) HIP_TRY(hipMemcpyAsync(out_idx, d_packed, total * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return DSY_OK;
}

int dsy_sync_respond(dsy_ctx* c, const dsy_store* s, const dsy_request* reqs, uint32_t R, const uint8_t* filters,
                     uint64_t filters_len, const dsy_meta* metas, uint32_t nmeta, uint64_t responder_global_time,
                     int include_inactive, int64_t byte_limit, uint64_t random_seed, uint64_t* out_idx,
                     uint64_t out_cap, uint64_t* out_req_offsets) {
    if (!c || !s || (R && (!reqs || !filters)) || (nmeta && !metas) || !out_req_offsets)
        return fail(DSY_EINVAL, "NULL argument");
    Guard g(c);
    void* d_f;
    int rc;
    if ((rc = ws_get(c, "filters", filters_len + 64, &d_f))) return rc;
    if (filters_len) HIP_TRY(hipMemcpyAsync(d_f, filters, filters_len, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemsetAsync((uint8_t*)d_f + filters_len, 0, 64, c->stream));
    Claims cl;
    cl.reqs = reqs;
    return respond_to_host(c, s, cl, R, d_f, filters_len, metas, nmeta, responder_global_time, include_inactive,
                           byte_limit, random_seed, out_idx, out_cap, out_req_offsets);
}

int dsy_sync_respond_refs(dsy_ctx* c, const dsy_store* s, const uint64_t* ranges, const uint64_t* refs, uint32_t R,
                          const dsy_meta* metas, uint32_t nmeta, uint64_t responder_global_time, int include_inactive,
                          int64_t byte_limit, uint64_t random_seed, uint64_t* out_idx, uint64_t out_cap,
                          uint64_t* out_req_offsets) {
    if (!c || !s || (R && (!ranges || !refs)) || (nmeta && !metas) || !out_req_offsets)
        return fail(DSY_EINVAL, "NULL argument");
    Guard g(c);
    // the library lays the filters out: claim r's at foff[r], 4-byte aligned
    std::vector<uint64_t> foff(std::max<uint32_t>(R, 1));
    uint64_t total = 0;
    for (uint32_t r = 0; r < R; ++r) {
        if (!refs[2 * (size_t)r] || !refs[2 * (size_t)r + 1]) return fail(DSY_EINVAL, "claim %u: NULL record or filter", r);
        const uint64_t m = ((const dsy_request*)(uintptr_t)refs[2 * (size_t)r])->m_bits;
        if (m == 0 || m % 8) return fail(DSY_EINVAL, "claim %u: m_bits %llu is not a positive multiple of 8", r, (unsigned long long)m);
        foff[r] = total;
        total += (m / 8 + 3) & ~uint64_t(3);
    }
    void* d_f;
    int rc;
    if ((rc = ws_get(c, "filters", total + 64, &d_f))) return rc;
    Claims cl;
    cl.ranges = ranges;
    cl.refs = refs;
    cl.foff = foff.data();
    RespondSlot& sl = sync_slot(c);
    // the filters are gathered into pinned staging and uploaded once the first window's selection is enqueued: the
    // host copies them while the GPU selects (job_window, jb.gather)
    sl.gather = FilterGather{refs, foff.data(), R, total, (uint8_t*)d_f};
    rc = respond_to_host(c, s, cl, R, d_f, total, metas, nmeta, responder_global_time, include_inactive, byte_limit,
                         random_seed, out_idx, out_cap, out_req_offsets);
    sl.gather = FilterGather{};
    return rc;
}

int dsy_sync_respond_dev(dsy_ctx* c, const dsy_store* s, const dsy_request* reqs, uint32_t R,
                         const uint8_t* d_filters, const dsy_meta* metas, uint32_t nmeta,
                         uint64_t responder_global_time, int include_inactive, int64_t byte_limit,
                         uint64_t random_seed, const uint64_t** d_out_idx, const uint64_t** d_out_offsets,
                         uint64_t* out_total_pairs) {
    if (!c || !s || (R && (!reqs || !d_filters)) || (nmeta && !metas)) return fail(DSY_EINVAL, "NULL argument");
    Guard g(c);
    uint64_t *d_packed, *d_off, pairs = 0;
    Claims cl;
    cl.reqs = reqs;
    int rc = respond_core(c, s, cl, R, d_filters, 0, metas, nmeta, responder_global_time, include_inactive,
                          byte_limit, random_seed, &d_packed, &d_off, &pairs);
    if (rc) return rc;
    if (d_out_idx) *d_out_idx = d_packed;
    if (d_out_offsets) *d_out_offsets = d_off;
    if (out_total_pairs) *out_total_pairs = pairs;
    return DSY_OK;
}

int dsy_sync_respond_submit(dsy_ctx* c, const dsy_store* s, const dsy_request* reqs, uint32_t R,
                            const uint8_t* d_filters, const dsy_meta* metas, uint32_t nmeta,
                            uint64_t responder_global_time, int include_inactive, int64_t byte_limit,
                            uint64_t random_seed, uint64_t* out_ticket) {
    if (!c || !s || (R && (!reqs || !d_filters)) || (nmeta && !metas) || !out_ticket)
        return fail(DSY_EINVAL, "NULL argument");
    Guard g(c);
    // the least recently used free slot: a waited-for batch's output stays valid until two more submits at least
    int k = -1;
    for (int i = 0; i < dsy_ctx::kSlots; ++i)
        if (!c->rs[i].busy && (k < 0 || c->rs[i].last_use < c->rs[k].last_use)) k = i;
    if (k < 0) return fail(DSY_EINVAL, "%d responder batches are in flight: dsy_sync_respond_wait one first", dsy_ctx::kSlots);
    RespondSlot& sl = c->rs[k];
    sl.last_use = ++c->use_clock;
    Claims cl;
    cl.reqs = reqs;
    int rc = job_start(c, sl, s, cl, R, d_filters, 0, metas, nmeta, responder_global_time, include_inactive,
                       byte_limit, random_seed);
    if (rc) {
        hipStreamSynchronize(c->stream);  // whatever was enqueued before the failure
        return rc;
    }
    sl.busy = true;
    sl.ticket = c->next_ticket++;
    *out_ticket = sl.ticket;
    return DSY_OK;
}

int dsy_sync_respond_wait(dsy_ctx* c, uint64_t ticket, const uint64_t** d_out_idx, const uint64_t** d_out_offsets,
                          uint64_t* out_total_pairs) {
    if (!c) return fail(DSY_EINVAL, "NULL argument");
    Guard g(c);
    RespondSlot* sl = nullptr;
    for (auto& x : c->rs)
        if (x.busy && x.ticket == ticket) sl = &x;
    if (!sl) return fail(DSY_EINVAL, "ticket %llu is not in flight", (unsigned long long)ticket);
    uint64_t *d_packed, *d_off, pairs = 0;
    int rc = job_finish(c, *sl, &d_packed, &d_off, &pairs);
    sl->busy = false;
    if (rc) {
        hipStreamSynchronize(c->stream);
        return rc;
    }
    if (d_out_idx) *d_out_idx = d_packed;
    if (d_out_offsets) *d_out_offsets = d_off;
    if (out_total_pairs) *out_total_pairs = pairs;
    return DSY_OK;
}

// ------------------------------------------------------------------------------------------- simulator
static int sim_check(const dsy_sim_config* c) {
    if (!c) return fail(DSY_EINVAL, "cfg is NULL");
    if (c->n_peers < 2 || c->peer_begin > c->peer_end || c->peer_end > c->n_peers || c->peers_per_rank == 0)
        return fail(DSY_EINVAL, "bad peer partition");
    if (c->universe == 0 || c->universe > 65536) return fail(DSY_EINVAL, "universe must be 1..65536 packets");
    if (c->m_bits > 32ull * kSimFilterWordsMax) return fail(DSY_EINVAL, "sim filters are limited to %u bits", 32 * kSimFilterWordsMax);
    int32_t kind;
    uint32_t chunk;
    int rc = check_family(c->m_bits, c->k, &kind, &chunk);
    if (rc) return rc;
    if (kind != c->hash_kind || chunk != c->chunk_bytes || kind > DSY_SHA256)
        return fail(DSY_EINVAL, "sim filter family must match bloomfilter.py and be MD5/SHA-1/SHA-256");
    if (c->capacity == 0 || c->capacity > 2048) return fail(DSY_EINVAL, "capacity must be 1..2048");
    return DSY_OK;
}

static SimLaunch sim_launch(dsy_ctx* c, const dsy_sim_config* cfg) {
    SimLaunch L{};
    L.cfg = *cfg;
    L.stream = c->stream;
    L.or_mode = c->or_mode;
    return L;
}

int dsy_sim_setup(dsy_sim_config* c) {
    if (!c) return fail(DSY_EINVAL, "cfg is NULL");
    c->words = (c->universe + 31) / 32;
    c->claim_bytes = (uint32_t)((sizeof(dsy_sim_claim_header) + filter_words(c->m_bits) * 4 + 15) / 16 * 16);
    c->resp_bytes = (uint32_t)((sizeof(dsy_sim_resp_header) + 2 * DSY_SIM_RESP_MAX + 15) / 16 * 16);
    return sim_check(c);
}

int dsy_sim_seed(dsy_ctx* c, const dsy_sim_config* cfg, uint32_t* d_bits, uint32_t initial) {
    if (!c || !d_bits) return fail(DSY_EINVAL, "NULL argument");
    int rc = sim_check(cfg);
    if (rc) return rc;
    Guard g(c);
    SimLaunch L = sim_launch(c, cfg);
    L.bits = d_bits;
    L.initial = initial;
    HIP_TRY(launch_sim(kSimSeed, L));
    return DSY_OK;
}

static int sim_counts(dsy_ctx* c, SimLaunch& L, int op, uint32_t* h_counts, uint32_t n_ranks) {
    void* d;
    int rc;
    if ((rc = ws_get(c, "sim_counts", 4 * std::max<uint32_t>(n_ranks, 1), &d))) return rc;
    HIP_TRY(hipMemsetAsync(d, 0, 4 * n_ranks, c->stream));
    L.counts = (uint32_t*)d;
    HIP_TRY(launch_sim(op, L));
    HIP_TRY(hipMemcpyAsync(h_counts, d, 4 * n_ranks, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return DSY_OK;
}

int dsy_sim_claim_counts(dsy_ctx* c, const dsy_sim_config* cfg, uint32_t round, uint32_t* h_counts, uint32_t n_ranks) {
    if (!c || !h_counts || !n_ranks) return fail(DSY_EINVAL, "NULL argument");
    int rc = sim_check(cfg);
    if (rc) return rc;
    if ((cfg->n_peers + cfg->peers_per_rank - 1) / cfg->peers_per_rank > n_ranks) return fail(DSY_EINVAL, "n_ranks too small");
    Guard g(c);
    SimLaunch L = sim_launch(c, cfg);
    L.round = round;
    return sim_counts(c, L, kSimClaimCounts, h_counts, n_ranks);
}

// the per-destination record cursors start at h_offsets[]: passed to a one-workgroup kernel by value (the host array
// is pageable: a copy from it would wait for the stream)
static int sim_cursor(dsy_ctx* c, const SimLaunch& base, const uint32_t* h_offsets, uint32_t n_ranks, uint32_t** out) {
    void* d;
    int rc;
    if ((rc = ws_get(c, "sim_cursor", 4 * std::max<uint32_t>(n_ranks, 1), &d))) return rc;
    if (n_ranks > kSimMaxRanks) {  // beyond one launch's argument: a staged copy (synchronous)
        HIP_TRY(hipStreamSynchronize(c->stream));
        HIP_TRY(hipMemcpy(d, h_offsets, 4 * n_ranks, hipMemcpyHostToDevice));
    } else {
        SimLaunch L = base;
        L.cursor_init.n = n_ranks;
        for (uint32_t i = 0; i < n_ranks; ++i) L.cursor_init.start[i] = h_offsets[i];
        L.cursor = (uint32_t*)d;
        HIP_TRY(launch_sim(kSimCursorInit, L));
    }
    *out = (uint32_t*)d;
    return DSY_OK;
}

int dsy_sim_claim_matrix(dsy_ctx* c, const dsy_sim_config* cfg, uint32_t round0, uint32_t n_rounds, uint32_t* h_matrix,
                         uint32_t n_ranks) {
    if (!c || !h_matrix || !n_ranks || !n_rounds) return fail(DSY_EINVAL, "NULL argument");
    int rc = sim_check(cfg);
    if (rc) return rc;
    if ((cfg->n_peers + cfg->peers_per_rank - 1) / cfg->peers_per_rank > n_ranks) return fail(DSY_EINVAL, "n_ranks too small");
    if (n_rounds > 65535) return fail(DSY_EINVAL, "at most 65535 rounds per call");
    Guard g(c);
    if (!c->aux) HIP_TRY(hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
    const size_t bytes = 4ull * n_rounds * n_ranks * n_ranks;
    void* d;
    if ((rc = ws_get(c, "sim_matrix", bytes, &d))) return rc;
    HIP_TRY(hipMemsetAsync(d, 0, bytes, c->aux));
    SimLaunch L = sim_launch(c, cfg);
    L.stream = c->aux;
    L.round = round0;
    L.n_rounds = n_rounds;
    L.n_ranks = n_ranks;
    L.counts = (uint32_t*)d;
    HIP_TRY(launch_sim(kSimClaimMatrix, L));
    HIP_TRY(hipMemcpyAsync(h_matrix, d, bytes, hipMemcpyDeviceToHost, c->aux));
    HIP_TRY(hipStreamSynchronize(c->aux));
    return DSY_OK;
}

int dsy_sim_build_claims(dsy_ctx* c, const dsy_sim_config* cfg, uint32_t round, const uint8_t* d_ublob,
                         const uint64_t* d_uoff, const uint32_t* d_bits, uint8_t* d_out, const uint32_t* h_offsets,
                         uint32_t n_ranks) {
    if (!c || !d_ublob || !d_uoff || !d_bits || !h_offsets) return fail(DSY_EINVAL, "NULL argument");
    int rc = sim_check(cfg);
    if (rc) return rc;
    Guard g(c);
    SimLaunch L = sim_launch(c, cfg);
    L.round = round;
    L.ublob = d_ublob;
    L.uoff = d_uoff;
    L.bits = (uint32_t*)d_bits;
    L.out = d_out;
    if ((rc = sim_cursor(c, L, h_offsets, n_ranks, &L.cursor))) return rc;
    void* ds;
    if ((rc = ws_get(c, "sim_slots", 4 * std::max<uint64_t>(cfg->peer_end - cfg->peer_begin, 1), &ds))) return rc;
    L.slots = (uint32_t*)ds;
    HIP_TRY(launch_sim(kSimClaimSlots, L));
    uint8_t* acc;
    if ((rc = sim_acc_get(c, &acc))) return rc;
    L.work = (unsigned long long*)acc;
    PendingTimer t;
    timer_begin(c, &t, kTimeSimBuild);
    HIP_TRY(launch_sim(kSimBuild, L));
    timer_end(c, &t);
    timers_collect_lazy(c);
    return DSY_OK;
}

int dsy_sim_resp_counts(dsy_ctx* c, const dsy_sim_config* cfg, const uint8_t* d_claims, uint64_t n_claims,
                        uint32_t* h_counts, uint32_t n_ranks) {
    if (!c || !h_counts || !n_ranks || (n_claims && !d_claims)) return fail(DSY_EINVAL, "NULL argument");
    int rc = sim_check(cfg);
    if (rc) return rc;
    Guard g(c);
    SimLaunch L = sim_launch(c, cfg);
    L.in = d_claims;
    L.n_in = n_claims;
    return sim_counts(c, L, kSimRespCounts, h_counts, n_ranks);
}

int dsy_sim_respond(dsy_ctx* c, const dsy_sim_config* cfg, const uint8_t* d_ublob, const uint64_t* d_uoff,
                    const uint32_t* d_bits, const uint8_t* d_claims, uint64_t n_claims, uint8_t* d_out,
                    const uint32_t* h_offsets, uint32_t n_ranks, uint64_t* out_tested) {
    if (!c || !d_ublob || !d_uoff || !d_bits || !h_offsets || (n_claims && (!d_claims || !d_out)))
        return fail(DSY_EINVAL, "NULL argument");
    int rc = sim_check(cfg);
    if (rc) return rc;
    Guard g(c);
    if (out_tested) {  // fold earlier calls first, so the count below is this call's alone
        HIP_TRY(hipStreamSynchronize(c->stream));
        if ((rc = sim_collect(c))) return rc;
    }
    SimLaunch L = sim_launch(c, cfg);
    L.ublob = d_ublob;
    L.uoff = d_uoff;
    L.bits = (uint32_t*)d_bits;
    L.in = d_claims;
    L.n_in = n_claims;
    L.out = d_out;
    if ((rc = sim_cursor(c, L, h_offsets, n_ranks, &L.cursor))) return rc;
    void* ds;
    if ((rc = ws_get(c, "sim_slots", 4 * std::max<uint64_t>(n_claims, 1), &ds))) return rc;
    L.slots = (uint32_t*)ds;
    HIP_TRY(launch_sim(kSimRespSlots, L));
    uint8_t* acc;
    if ((rc = sim_acc_get(c, &acc))) return rc;
    L.work = (unsigned long long*)acc;
    L.tested = (unsigned long long*)(acc + kSimAccWork);
    PendingTimer t;
    timer_begin(c, &t, kTimeSimRespond);
    HIP_TRY(launch_sim(kSimRespond, L));
    timer_end(c, &t);
    timers_collect_lazy(c);
    if (out_tested) {  // the caller wants this call's count now: wait for it
        const uint64_t before = c->useful[kTimeSimRespond];
        HIP_TRY(hipStreamSynchronize(c->stream));
        if ((rc = sim_collect(c))) return rc;
        *out_tested = c->useful[kTimeSimRespond] - before;
    }
    return DSY_OK;
}

int dsy_sim_merge(dsy_ctx* c, const dsy_sim_config* cfg, uint32_t* d_bits, const uint8_t* d_resps, uint64_t n_resps) {
    if (!c || !d_bits || (n_resps && !d_resps)) return fail(DSY_EINVAL, "NULL argument");
    int rc = sim_check(cfg);
    if (rc) return rc;
    Guard g(c);
    SimLaunch L = sim_launch(c, cfg);
    L.bits = d_bits;
    L.in = d_resps;
    L.n_in = n_resps;
    uint8_t* acc;
    if ((rc = sim_acc_get(c, &acc))) return rc;
    L.counts = (uint32_t*)(acc + kSimAccWork + kSimAccTested);  // sticky overflow flag, reported by dsy_sim_stats
    HIP_TRY(launch_sim(kSimMerge, L));
    return DSY_OK;
}

int dsy_sim_stats(dsy_ctx* c, const dsy_sim_config* cfg, const uint32_t* d_bits, uint64_t* out) {
    if (!c || !d_bits || !out) return fail(DSY_EINVAL, "NULL argument");
    int rc = sim_check(cfg);
    if (rc) return rc;
    Guard g(c);
    SimLaunch L = sim_launch(c, cfg);
    L.bits = (uint32_t*)d_bits;
    void* d;
    if ((rc = ws_get(c, "sim_stats", 16, &d))) return rc;
    HIP_TRY(hipMemsetAsync(d, 0, 16, c->stream));
    L.stats = (unsigned long long*)d;
    HIP_TRY(launch_sim(kSimStats, L));
    HIP_TRY(hipMemcpyAsync(out, d, 16, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if ((rc = sim_collect(c))) return rc;
    if (c->sim_overflow) {
        c->sim_overflow = false;
        return fail(DSY_ECAPACITY, "a response exceeded DSY_SIM_RESP_MAX packets (byte_limit / shortest packet too large)");
    }
    return DSY_OK;
}

}  // extern "C"

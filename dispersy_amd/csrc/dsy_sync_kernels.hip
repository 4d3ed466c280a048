// dsy_sync_kernels.hip -- the batched responder (community.py:2746-2811 + :2555-2567) on gfx950.
//
// Work is windowed per claim, mirroring the reference's lazy cursor + lazy not_filter: each window selects at
// most W (claim, packet) pairs per claim in send order, hashes and tests them, and emits missing packets until
// the claim's byte budget is spent.  A claim whose budget is spent after its first window never selects more,
// exactly as the reference stops pulling rows from SQLite.  Only the claims still active take part in a window
// (L.act: window slot a serves claim act[a]); the host grows W as claims finish, so the few claims that walk huge
// ranges (a filter that covers everything, a global time shared by 10^5 rows) take big windows instead of
// hundreds of small ones.
//
//   k_setup       copies the call's staged claims from pinned host memory to the device and zeroes the status
//                 counters (no copy-engine or fill dispatch), then one lane per (claim, meta): binary-search the
//                 live-row span of [time_low', time_high] in the meta's global_time-sorted segment; choose scan
//                 (every row) or enumerate (every global time g = g0 + i*modulo, each found by binary search) by
//                 which touches fewer bytes.  The last workgroup to finish sums the per-claim spans and, when
//                 the output bound is small, scans the per-claim capacities (no separate launch).
//   k_fill        one 256-lane workgroup per claim: the next <= W rows in send order (ASC / DESC / Feistel-
//                 permuted RANDOM), block prefix-sum placement, resumable (meta, candidate, sub-row) cursor.
//   k_pair_test   one lane per pair, a wave per 64 pairs of one claim (filter/prefix/m/k wave-uniform): digest
//                 of prefix || packet, k probes -> missing flag.
//   k_compact     one wave per claim: ballot + prefix-sum compaction of missing pairs in send order with the
//                 byte-limit rule of community.py:2559-2567 (the crossing packet is sent).
//   k_pack        exclusive scan of per-claim counts and a copy into the packed output (one launch for up to
//                 kPackFusedMax claims: each workgroup sums the counts before its claim itself).
#include "dsy_kernels.h"

namespace dsy {

static constexpr uint64_t kMaxGt = 0x7fffffffffffffffull;  // 2^63 - 1 (community.py:2547-2548, :2806)
static constexpr uint32_t kBulkBins = 1024;  // == kSortBins: bulk_hist / bulk_cur entries per window slot

__device__ __forceinline__ uint64_t lower_bound_gt(const uint64_t* gt, uint64_t a, uint64_t b, uint64_t v) {
    while (a < b) {
        const uint64_t mid = a + ((b - a) >> 1);
        if (gt[mid] < v) a = mid + 1; else b = mid;
    }
    return a;
}

__device__ __forceinline__ uint64_t upper_bound_gt(const uint64_t* gt, uint64_t a, uint64_t b, uint64_t v) {
    while (a < b) {
        const uint64_t mid = a + ((b - a) >> 1);
        if (gt[mid] <= v) a = mid + 1; else b = mid;
    }
    return a;
}

// lower_bound over a sorted global-time column, interpolation first: each round probes gt[p-1], gt[p] at the
// position the span's end values predict (one round-trip of independent loads), so dense or roughly uniform
// global times resolve in one or two round-trips instead of ~log2(N) dependent loads; at most three rounds,
// then plain binary search on what is left (skewed data stays O(log N)).
__device__ __forceinline__ uint64_t lower_bound_interp(const uint64_t* gt, uint64_t lo, uint64_t hi, uint64_t v) {
    // invariant: the answer lies in [lo, hi]
#pragma unroll 1
    for (int round = 0; round < 3 && hi - lo > 8; ++round) {
        const uint64_t g0 = gt[lo], g1 = gt[hi - 1];
        if (v <= g0) return lo;
        if (v > g1) return hi;
        // g0 < v <= g1: the answer is in [lo + 1, hi - 1]
        const double f = (double)(v - g0) / (double)(g1 - g0);
        uint64_t p = lo + 1 + (uint64_t)(f * (double)(hi - 2 - lo));
        if (p > hi - 1) p = hi - 1;
        const uint64_t gp = gt[p], gq = gt[p - 1];
        if (gq < v && v <= gp) return p;
        if (gp < v) lo = p + 1;
        else hi = p - 1;
    }
    return lower_bound_gt(gt, lo, hi, v);
}

__device__ __forceinline__ uint32_t mix32(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return (uint32_t)x;
}

// Bijection of [0, n) by a 4-round Feistel network on 2*bits bits with cycle walking (RANDOM direction).
__device__ __forceinline__ uint64_t permute(uint64_t x, uint64_t n, uint32_t bits, uint64_t key) {
    const uint64_t mask = (1ull << bits) - 1;
    do {
        uint64_t l = x >> bits, r = x & mask;
#pragma unroll
        for (int round = 0; round < 4; ++round) {
            const uint64_t f = mix32(r ^ (key + 0x9e3779b97f4a7c15ull * (round + 1))) & mask;
            const uint64_t t = l ^ f;
            l = r;
            r = t;
        }
        x = (l << bits) | r;
    } while (x >= n);
    return x;
}

__device__ __forceinline__ uint64_t plan_one(const RespondLaunch& L, const DevRequest& q, const SegMeta& mt,
                                             uint32_t idx, uint32_t r, uint32_t j, Plan* copy = nullptr) {
    uint64_t lo = q.time_low, hi = q.time_high;
    if (!L.include_inactive && mt.has_pruning) {
        // time_low' = min(max(time_low, global_time - inactive + 1), 2^63-1)   (community.py:2806)
        if (L.responder_gt + 1 > mt.inactive) {
            const uint64_t act = L.responder_gt + 1 - mt.inactive;
            if (act > lo) lo = act;
        }
        if (lo > kMaxGt) lo = kMaxGt;
    }
    Plan p{};
    p.dir = mt.dir;
    p.a = p.b = mt.seg_a;
    bool have_ends = false;  // p.g_lo / p.g_hi known from the searches' probes
    if (lo <= hi && mt.seg_a < mt.seg_b) {
        // Both ends of the span in two dependent rounds of loads when the segment's global times are dense or evenly
        // spread: the segment's end values (shared by both searches), then both interpolated positions and their
        // predecessors together -- whose values are also g_lo and g_hi.  Anything else falls back to
        // lower_bound_interp's rounds and binary search.
        const uint64_t* gt = L.st.live_gt;
        const uint64_t a = mt.seg_a, b = mt.seg_b;
        const uint64_t g0 = gt[a], g1 = gt[b - 1];
        const bool open_hi = hi >= kMaxGt;
        const uint64_t v0 = lo, v1 = open_hi ? 0 : hi + 1;
        auto guess = [&](uint64_t v) -> uint64_t {  // a position in [a + 1, b - 1] for g0 < v <= g1 (b - a >= 2)
            const double f = (double)(v - g0) / (double)(g1 - g0);
            uint64_t q = a + 1 + (uint64_t)(f * (double)(b - 2 - a));
            return q > b - 1 ? b - 1 : q;
        };
        // search 0: lower_bound(lo); search 1: lower_bound(hi + 1) (open_hi: the segment's end)
        bool done0 = false, done1 = open_hi;
        uint64_t r0 = 0, r1 = b, q0 = 0, q1 = 0;
        if (v0 <= g0) { r0 = a; done0 = true; }
        else if (v0 > g1) { r0 = b; done0 = true; }
        else q0 = guess(v0);
        if (!done1) {
            if (v1 <= g0) { r1 = a; done1 = true; }
            else if (v1 > g1) { r1 = b; done1 = true; }
            else q1 = guess(v1);
        }
        uint64_t gp0 = 0, gq0 = 0, gp1 = 0, gq1 = 0;
        if (!done0) { gp0 = gt[q0]; gq0 = gt[q0 - 1]; }
        if (!done1) { gp1 = gt[q1]; gq1 = gt[q1 - 1]; }
        if (!done0 && gq0 < v0 && v0 <= gp0) { r0 = q0; done0 = true; }
        if (!done1 && gq1 < v1 && v1 <= gp1) { r1 = q1; done1 = true; }
        if (!done0) r0 = lower_bound_interp(gt, a, b, v0);
        if (!done1) r1 = lower_bound_interp(gt, r0, b, v1);
        p.a = r0;
        p.b = r1 < r0 ? r0 : r1;
        if (p.b > p.a) {
            // g_lo = gt[p.a]: the found position's value, or the segment's first; g_hi = gt[p.b - 1] likewise
            const bool lo_known = p.a == a || (p.a == q0 && gq0 < v0 && v0 <= gp0);
            const bool hi_known = p.b == b || (!open_hi && p.b == q1 && gq1 < v1 && v1 <= gp1);
            if (lo_known && hi_known) {
                p.g_lo = p.a == a ? g0 : gp0;
                p.g_hi = p.b == b ? g1 : gq1;
                have_ends = true;
            }
        }
    }
    const uint64_t span = p.b - p.a;
    if (span) {
        if (!have_ends) {
            p.g_lo = L.st.live_gt[p.a];
            p.g_hi = L.st.live_gt[p.b - 1];
        }
        p.dense = p.g_hi - p.g_lo == span - 1;
    }
    const uint64_t mod = q.modulo;
    p.mode = 0;
    p.ncand = span;
    if (mod > 1 && span > 0) {
        const uint64_t rem = (lo + q.offset) % mod;
        const uint64_t g0 = rem ? lo + (mod - rem) : lo;
        const uint64_t nenum = g0 > hi ? 0 : (hi - g0) / mod + 1;
        uint32_t lg = 1;
        while ((1ull << lg) < span && lg < 63) ++lg;
        // enumerate when ~2*log2(span) random 64-byte probes per global time beat streaming 8 bytes per row
        if (nenum * (uint64_t)(2 * lg + 2) * 8 < span) {
            p.mode = 1;
            p.g0 = g0;
            p.ncand = nenum;
        }
    }
    if (p.dir == DSY_RANDOM && p.ncand > 1) {
        uint32_t bits = 1;
        while ((1ull << (2 * bits)) < p.ncand) ++bits;
        p.perm_bits = bits;
        p.perm_key = (uint64_t)mix32(L.seed ^ ((uint64_t)r << 32) ^ j) << 32 | mix32(L.seed * 31 + r * 131 + j);
    }
    L.plans[idx] = p;
    if (copy) *copy = p;
    return span;
}

__device__ __forceinline__ uint64_t block_sum_256(uint64_t v, uint64_t* lds4) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    if (lane == 0) lds4[wv] = v;
    __syncthreads();
    const uint64_t t = lds4[0] + lds4[1] + lds4[2] + lds4[3];
    __syncthreads();
    return t;
}

// src: the staged upload region in pinned host memory ([DevRequest R | SegMeta J | ...], respond_core's layout),
// copied to dst (= L.reqs) in 16-byte words; zero: the status counters.  per_claim_cap == 0: upper bounds only
// (the host derives the capacities).
__global__ void __launch_bounds__(256) k_setup(RespondLaunch L, const uint4* __restrict__ src, uint4* __restrict__ dst,
                                               uint32_t in_words, uint4* __restrict__ zero, uint32_t zero_words,
                                               uint64_t per_claim_cap) {
    __shared__ uint64_t red[4];
    __shared__ uint32_t last;
    const uint32_t tid = blockIdx.x * 256 + threadIdx.x, nthr = gridDim.x * 256;
    const bool planner = tid < L.R * L.J;
    const uint32_t r = planner ? tid / L.J : 0, j = planner ? tid % L.J : 0;
    // every host read of the thread is issued before the first wait: each is a PCIe round trip
    static_assert(sizeof(DevRequest) % 16 == 0 && sizeof(SegMeta) % 16 == 0, "16-byte staged records");
    const uint4* hq = src + (size_t)r * (sizeof(DevRequest) / 16);
    const uint4* hm = src + (size_t)L.R * (sizeof(DevRequest) / 16) + (size_t)j * (sizeof(SegMeta) / 16);
    uint4 qw[sizeof(DevRequest) / 16], mw[sizeof(SegMeta) / 16], cw = make_uint4(0, 0, 0, 0);
    if (planner) {
#pragma unroll
        for (int i = 0; i < (int)(sizeof(DevRequest) / 16); ++i) qw[i] = hq[i];
#pragma unroll
        for (int i = 0; i < (int)(sizeof(SegMeta) / 16); ++i) mw[i] = hm[i];
    }
    if (tid < in_words) cw = src[tid];
    if (tid < in_words) dst[tid] = cw;
    for (uint32_t i = tid + nthr; i < in_words; i += nthr) dst[i] = src[i];
    for (uint32_t i = tid; i < zero_words; i += nthr) zero[i] = make_uint4(0, 0, 0, 0);
    // the split windows' sort state starts every call at zero in this call's layout (k_compact keeps it zero between
    // windows; a call that ended early, or one with another R, may have left counts where this call's slots are)
    if (L.bulk_zero)
        for (uint64_t i = tid; i < (uint64_t)L.R * kBulkBins; i += nthr) L.bulk_hist[i] = L.bulk_cur[i] = 0;
    if (planner) {
        DevRequest q;
        SegMeta mt;
        __builtin_memcpy(&q, qw, sizeof q);
        __builtin_memcpy(&mt, mw, sizeof mt);
        const uint64_t span = plan_one(L, q, mt, tid, r, j);
        if (L.J == 1 && per_claim_cap) {
            // one meta: the claim's bound is its span; output slots at r * per_claim_cap (the buffer holds
            // R * per_claim_cap rows), so no scan is needed
            L.upper[r] = span;
            ReqState st{};
            st.cap = min(span, per_claim_cap);
            st.out_base = (uint64_t)r * per_claim_cap;
            st.done = span == 0;
            L.state[r] = st;
        }
    }
    if (L.J == 1 && per_claim_cap) return;
    // the last workgroup to finish: upper[r] = sum of the claim's spans, then the capacities
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(L.ticket, 1u) == gridDim.x - 1;
    __syncthreads();
    if (!last) return;
    __threadfence();
    const uint32_t per = (L.R + 255) / 256;  // thread t owns claims [t*per, t*per + per)
    uint64_t sum = 0;
    for (uint32_t i = 0; i < per; ++i) {
        const uint32_t r = threadIdx.x * per + i;
        if (r >= L.R) break;
        uint64_t u = 0;
        for (uint32_t j = 0; j < L.J; ++j) {
            const Plan& p = L.plans[(size_t)r * L.J + j];
            u += p.b - p.a;
        }
        L.upper[r] = u;
        sum += min(u, per_claim_cap);
    }
    if (per_claim_cap) {
        // exclusive scan of the capacities over the owners (wave scan + one LDS round)
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        uint64_t incl = sum;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t o = __shfl_up(incl, d, 64);
            if (lane >= d) incl += o;
        }
        if (lane == 63) red[wv] = incl;
        __syncthreads();
        uint64_t run = incl - sum;
        for (int w = 0; w < wv; ++w) run += red[w];
        for (uint32_t i = 0; i < per; ++i) {
            const uint32_t r = threadIdx.x * per + i;
            if (r >= L.R) break;
            ReqState st{};
            st.cap = min(L.upper[r], per_claim_cap);
            st.out_base = run;
            st.done = L.upper[r] == 0;
            L.state[r] = st;
            run += st.cap;
        }
    }
    if (threadIdx.x == 0) *L.ticket = 0;  // ready for the next call
}

// ------------------------------------------------------------------------------------------- k_fill
static constexpr int kFillThreads = 256;
static constexpr int kFillWaves = kFillThreads / 64;

// Live-row range [x, y) of global time g inside the plan's span.  One round of three independent loads when the
// span's global times are dense or evenly spread (the position interpolated from the span's end values is exact);
// otherwise the interpolation / binary search of lower_bound_interp.
__device__ __forceinline__ void enum_range(const uint64_t* __restrict__ gt, const Plan& p, uint64_t g, uint64_t* x,
                                           uint64_t* y) {
    if (p.a >= p.b || g < p.g_lo || g > p.g_hi) {
        *x = *y = g < p.g_lo ? p.a : p.b;
        return;
    }
    const uint64_t span = p.b - p.a;
    uint64_t guess = p.a;
    if (p.g_hi > p.g_lo)
        guess = p.a + (uint64_t)((double)(g - p.g_lo) / (double)(p.g_hi - p.g_lo) * (double)(span - 1) + 0.5);
    if (guess >= p.b) guess = p.b - 1;
    const uint64_t gp = gt[guess];
    const uint64_t gq = guess > p.a ? gt[guess - 1] : 0;
    const uint64_t gn = guess + 1 < p.b ? gt[guess + 1] : ~0ull;
    if (gp == g && (guess == p.a || gq < g)) {
        *x = guess;
        *y = gn != g ? guess + 1 : upper_bound_gt(gt, guess + 1, p.b, g);
        return;
    }
    const uint64_t lx = lower_bound_interp(gt, p.a, p.b, g);
    uint64_t ly = lx;
    if (lx < p.b && gt[lx] == g) ly = (lx + 1 < p.b && gt[lx + 1] == g) ? upper_bound_gt(gt, lx + 1, p.b, g) : lx + 1;
    *x = lx;
    *y = ly;
}
static constexpr uint32_t kSortBins = kBulkBins;
// k_fill: a window one workgroup selected with more pairs than this is sorted by k_fill_sort's workgroups
static constexpr uint64_t kSplitSortMin = 8192;
static_assert(kSortBins == kPoolBins, "a pooled family's histogram has k_fill's bins");

// exclusive scan of kSortBins LDS counters in place, by the first wave of the workgroup (the others idle); the sum
// of the counters goes to *total when given
__device__ __forceinline__ void bins_exclusive_scan(uint32_t* bins, uint32_t* total = nullptr) {
    if (threadIdx.x >= 64) return;
    const uint32_t per = kSortBins / 64, lane = threadIdx.x;
    uint32_t sum = 0;
    for (uint32_t i = 0; i < per; ++i) sum += bins[lane * per + i];
    uint32_t incl = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d, 64);
        if ((int)lane >= d) incl += o;
    }
    uint32_t run = incl - sum;
    for (uint32_t i = 0; i < per; ++i) {
        const uint32_t h = bins[lane * per + i];
        bins[lane * per + i] = run;
        run += h;
    }
    if (total && lane == 63) *total = incl;
}

__device__ __forceinline__ uint64_t block_exclusive_scan(uint64_t v, uint64_t* lds, uint64_t* total) {
    // lds: kFillWaves + 1 words.  Wave-level inclusive scans (no barrier), one LDS round for the wave totals.
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    uint64_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = __shfl_up(incl, d, 64);
        if (lane >= d) incl += o;
    }
    if (lane == 63) lds[wv] = incl;
    __syncthreads();
    uint64_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kFillWaves; ++w) {
        const uint64_t x = lds[w];
        before += w < wv ? x : 0;
        all += x;
    }
    *total = all;
    __syncthreads();  // lds is reused by the next call
    return before + incl - v;
}

// The next window of claim r (window slot a_slot) from its cursor (meta j, candidate c, rows s of c already sent):
// selection in send order, then the block-count sort into task records; thread 0 stores the new cursor in *S.
// plan_at(j): the claim's plan for meta j.
template <class PlanAt>
__device__ __forceinline__ void fill_claim(const RespondLaunch& L, uint32_t a_slot, uint32_t r, const DevRequest& q,
                                           ReqState* S, uint32_t j, uint64_t c, uint64_t s, PlanAt plan_at,
                                           uint64_t clk_start, uint64_t clk0, bool may_split = false,
                                           bool slice = false, uint64_t s0 = 0, uint64_t s1 = 0) {
    __shared__ uint64_t scan[kFillWaves + 2];
    __shared__ uint32_t first_cross;
    constexpr int kCandRuns = kFillThreads * 2;  // kBatch below: a round's candidates
    __shared__ uint32_t run_pos[kCandRuns];       // a round's candidates: first output position (round-relative)
    __shared__ uint64_t run_x[kCandRuns];         // and first live row
    const uint64_t W = L.window;
    // slice: this workgroup is one of the window's parts -- every part selects alike (the same candidates, counts
    // and cursor) and writes only the pairs at window positions [s0, s1); part 0 (s0 == 0) files the cursor, the
    // parts' histograms go to bulk_hist and k_fill_sort places the pairs
    if (!slice) { s0 = 0; s1 = W; }
    if (s1 > W) s1 = W;
    // this window's missing-pair bits of the claim start clear (k_pair_test sets them)
    for (uint64_t w = s0 / 64 + threadIdx.x; w < s1 / 64; w += kFillThreads)
        L.miss_mask[(uint64_t)a_slot * (W / 64) + w] = 0;
    uint64_t* out = L.pair_row + (uint64_t)a_slot * W;
    uint64_t* out_off = L.pair_off + (uint64_t)a_slot * W;
    uint32_t* out_len = L.pair_len + (uint64_t)a_slot * W;
    uint64_t filled = 0;
    const uint64_t mod = q.modulo, off = q.offset;
    // the sort's registers (below); a window that is one dense run of <= kFillThreads * kSortReg rows fills them
    // during the selection itself (pair t = thread t % 256, register t / 256), so the sort reads nothing back
    constexpr int kSortReg = 8;
    uint32_t reg_off[kSortReg];  // line index: a pair's packet starts kLineBias bytes into a 128-byte line
    uint32_t reg_len[kSortReg];
    uint64_t regs_rows = 0;  // pairs t < regs_rows are in the registers already (their pair_off is not written)
    // each thread takes kCand consecutive candidates, so one round of independent lookups covers
    // kFillThreads * kCand candidates (the fill is latency-bound: fewer, wider rounds)
    constexpr int kCand = 2;
    constexpr uint64_t kBatch = (uint64_t)kFillThreads * kCand;
    static_assert(kBatch == kCandRuns, "one LDS run slot per candidate of a round");
    while (j < L.J && filled < W) {
        const Plan p = plan_at(j);
        if (c >= p.ncand) { ++j; c = 0; s = 0; continue; }
        if (p.dir != DSY_RANDOM && ((p.dense && p.mode == 1) || (p.mode == 0 && mod <= 1))) {
            // Candidate -> row is arithmetic, no lookup and no scan: a scan that keeps every live row of the span
            // (candidate i is live row a + i), or an enumeration over a span with one row per global time,
            // consecutive.  Candidates (ascending) whose global time lies in [g_lo, g_hi] are [i0, i1); the others
            // have no row.
            uint64_t i0 = 0, i1 = p.ncand;
            if (p.mode == 1) {
                i0 = p.g_lo > p.g0 ? (p.g_lo - p.g0 + mod - 1) / mod : 0;
                i1 = p.g_hi >= p.g0 ? (p.g_hi - p.g0) / mod + 1 : 0;
                if (i1 > p.ncand) i1 = p.ncand;
                if (i0 > i1) i0 = i1;
            }
            // iteration order: ASC visits candidates i0..i1-1, DESC i1-1..i0
            const uint64_t it0 = p.dir == DSY_DESC ? p.ncand - i1 : i0, it1 = p.dir == DSY_DESC ? p.ncand - i0 : i1;
            const uint64_t cs = c > it0 ? c : it0;
            const uint64_t avail = cs < it1 ? it1 - cs : 0;
            const uint64_t take = avail < W - filled ? avail : W - filled;
            const RowRec* __restrict__ rec = L.st.rec;
            // kDenseU rows per thread per round, every load of the round issued before the first is consumed
            constexpr int kDenseU = kSortReg;
            const bool to_regs = !slice && filled == 0 && take <= (uint64_t)kFillThreads * kDenseU;
            // the positions this workgroup writes: i in [ib, ie)
            const uint64_t ib = s0 > filled ? s0 - filled : 0;
            const uint64_t ie = s1 > filled ? (take < s1 - filled ? take : s1 - filled) : 0;
            for (uint64_t i0 = ib; i0 < ie; i0 += (uint64_t)kFillThreads * kDenseU) {
                uint64_t row[kDenseU];
                RowRec rr[kDenseU];
#pragma unroll
                for (int u = 0; u < kDenseU; ++u) {
                    const uint64_t i = i0 + threadIdx.x + (uint64_t)kFillThreads * u;
                    const uint64_t ci = cs + (i < ie ? i : ib);
                    const uint64_t cd = p.dir == DSY_DESC ? p.ncand - 1 - ci : ci;
                    const uint64_t lr = p.a + (p.mode == 1 ? p.g0 + cd * mod - p.g_lo : cd);
                    row[u] = (L.st.live_row && i < ie) ? L.st.live_row[lr] : lr;
                }
#pragma unroll
                for (int u = 0; u < kDenseU; ++u) {
                    const bool in = i0 + threadIdx.x + (uint64_t)kFillThreads * u < ie;
                    rr[u] = in ? rec[row[u]] : RowRec{};
                }
#pragma unroll
                for (int u = 0; u < kDenseU; ++u) {
                    const uint64_t i = i0 + threadIdx.x + (uint64_t)kFillThreads * u;
                    if (i < ie) {
                        out[filled + i] = row[u];
                        if (!to_regs) out_off[filled + i] = rr[u].off;  // read back only by the sort
                        out_len[filled + i] = rr[u].len;
                    }
                    if (to_regs) {
                        reg_off[u] = (uint32_t)(rr[u].off >> 7);  // line index (off = line * 128 + kLineBias)
                        reg_len[u] = rr[u].len;
                    }
                }
            }
            if (to_regs) regs_rows = take;
            filled += take;
            c = cs + take;
            if (c >= it1) c = p.ncand;  // the remaining candidates have no row
            s = 0;
            continue;
        }
        uint64_t xs[kCand], cnts[kCand], sks[kCand];
        uint64_t tcnt = 0;
        const uint64_t* __restrict__ gt = L.st.live_gt;
        // phase A: every candidate's probe addresses, and ALL the loads issued before any is consumed (a branch
        // between them would serialise kCand memory round-trips)
        uint64_t cand[kCand], pa[kCand], ga[kCand], gb[kCand], gc[kCand];
        bool ok[kCand];
#pragma unroll
        for (int u = 0; u < kCand; ++u) {
            const uint64_t ci = c + (uint64_t)threadIdx.x * kCand + u;
            ok[u] = ci < p.ncand;
            uint64_t cd = ci;
            if (p.dir == DSY_DESC) cd = p.ncand - 1 - ci;
            else if (p.dir == DSY_RANDOM && p.ncand > 1 && ok[u]) cd = permute(ci, p.ncand, p.perm_bits, p.perm_key);
            cand[u] = cd;
            if (p.mode == 0) {
                pa[u] = p.a + cd;
            } else {
                const uint64_t g = p.g0 + cd * mod;
                uint64_t guess = p.a;
                if (p.g_hi > p.g_lo && g > p.g_lo)
                    guess = p.a + (uint64_t)((double)(g - p.g_lo) / (double)(p.g_hi - p.g_lo) * (double)(p.b - p.a - 1) + 0.5);
                pa[u] = guess < p.b ? guess : p.b - 1;
            }
        }
#pragma unroll
        for (int u = 0; u < kCand; ++u) {
            const bool need = ok[u] && p.b > p.a && (p.mode == 1 || mod > 1);
            ga[u] = need ? gt[pa[u]] : 0;
            gb[u] = (need && p.mode == 1 && pa[u] > p.a) ? gt[pa[u] - 1] : 0;
            gc[u] = (need && p.mode == 1 && pa[u] + 1 < p.b) ? gt[pa[u] + 1] : ~0ull;
        }
        // phase B: ranges (the enumerate fallback -- a guess that missed -- is rare on dense or even global times)
#pragma unroll
        for (int u = 0; u < kCand; ++u) {
            uint64_t x = 0, y = 0;  // live-row range of this candidate
            if (ok[u]) {
                if (p.mode == 0) {
                    x = pa[u];
                    y = (mod <= 1 || ((ga[u] + off) % mod) == 0) ? x + 1 : x;
                } else {
                    const uint64_t g = p.g0 + cand[u] * mod;
                    if (p.a >= p.b || g < p.g_lo || g > p.g_hi) {
                        x = y = g < p.g_lo ? p.a : p.b;
                    } else if (ga[u] == g && (pa[u] == p.a || gb[u] < g)) {
                        x = pa[u];
                        y = gc[u] != g ? x + 1 : upper_bound_gt(gt, x + 1, p.b, g);
                    } else {
                        enum_range(gt, p, g, &x, &y);
                    }
                }
            }
            const uint64_t sk = (threadIdx.x == 0 && u == 0) ? s : 0;  // rows of a resumed candidate already sent
            uint64_t n = y - x;
            n = n > sk ? n - sk : 0;
            // DESC walks the range from its top: the first row emitted is y - 1 - sk
            xs[u] = p.dir == DSY_DESC ? y - 1 - sk : x + sk;
            cnts[u] = n;
            sks[u] = sk;
            tcnt += n;
        }
        uint64_t total;
        const uint64_t pos = block_exclusive_scan(tcnt, scan, &total);
        // emit the rows of these candidates that still fit in the window, in candidate order: first every
        // candidate's first row with all loads issued together, then the rare extra rows of shared global times
        const RowRec* __restrict__ rec = L.st.rec;
        uint64_t row0[kCand];
        RowRec r0[kCand];
#pragma unroll
        for (int u = 0; u < kCand; ++u) {
            const uint64_t lr = xs[u];
            row0[u] = (cnts[u] && L.st.live_row) ? L.st.live_row[lr] : lr;
        }
#pragma unroll
        for (int u = 0; u < kCand; ++u) r0[u] = cnts[u] ? rec[row0[u]] : RowRec{};
        uint64_t at = pos;
#pragma unroll
        for (int u = 0; u < kCand; ++u) {
            const uint64_t dst = filled + at;
            if (cnts[u] && dst >= s0 && dst < s1) {
                out[dst] = row0[u];
                out_off[dst] = r0[u].off;
                out_len[dst] = r0[u].len;
            }
            at += cnts[u];
        }
        // the extra rows of shared global times: when a candidate of this round holds more than one row, the
        // workgroup emits them together -- thread i takes the round's output positions i, i + 256, ..., its
        // candidate found by binary search over the candidates' starts in LDS -- so a global time shared by 10^5
        // rows (config 5's Zipf global times) is not walked by one thread
        bool many = false;
#pragma unroll
        for (int u = 0; u < kCand; ++u) many |= cnts[u] > 1;
        if (__syncthreads_or(many)) {
            at = pos;
#pragma unroll
            for (int u = 0; u < kCand; ++u) {
                run_pos[threadIdx.x * kCand + u] = (uint32_t)(at < W ? at : W);
                run_x[threadIdx.x * kCand + u] = xs[u];
                at += cnts[u];
            }
            __syncthreads();
            uint64_t lim = total < W - filled ? total : W - filled;  // positions j of this round: [jb, lim)
            const uint64_t lim_s = s1 > filled ? s1 - filled : 0;
            if (lim_s < lim) lim = lim_s;
            const uint64_t jb = s0 > filled ? s0 - filled : 0;
            // kRowU positions per thread per pass, their record loads issued together; a thread's positions only
            // grow, so its candidate index is kept and searched forward only when the position leaves it (a global
            // time of 10^5 rows is one candidate for every position)
            constexpr int kRowU = 4;
            uint32_t cur = 0;
            for (uint64_t j0 = jb + threadIdx.x; j0 < lim; j0 += (uint64_t)kFillThreads * kRowU) {
                uint64_t lr[kRowU];
                bool take[kRowU];
#pragma unroll
                for (int u = 0; u < kRowU; ++u) {
                    const uint64_t jj = j0 + (uint64_t)kFillThreads * u;
                    const uint32_t j = (uint32_t)jj;
                    take[u] = false;
                    lr[u] = 0;
                    if (jj < lim) {
                        if (cur + 1 < (uint32_t)kBatch && run_pos[cur + 1] <= j) {
                            uint32_t lo = cur + 1, hi = (uint32_t)kBatch;  // the last candidate starting <= j
                            while (hi - lo > 1) {
                                const uint32_t mid = (lo + hi) >> 1;
                                if (run_pos[mid] <= j) lo = mid;
                                else hi = mid;
                            }
                            cur = lo;
                        }
                        const uint64_t e = j - run_pos[cur];
                        take[u] = e != 0;  // a candidate's first row was emitted above
                        lr[u] = p.dir == DSY_DESC ? run_x[cur] - e : run_x[cur] + e;
                    }
                }
                uint64_t row[kRowU];
#pragma unroll
                for (int u = 0; u < kRowU; ++u) row[u] = (take[u] && L.st.live_row) ? L.st.live_row[lr[u]] : lr[u];
                RowRec rw[kRowU];
#pragma unroll
                for (int u = 0; u < kRowU; ++u) rw[u] = take[u] ? rec[row[u]] : RowRec{};
#pragma unroll
                for (int u = 0; u < kRowU; ++u) {
                    if (take[u]) {
                        const uint64_t dst = filled + j0 + (uint64_t)kFillThreads * u;
                        out[dst] = row[u];
                        out_off[dst] = rw[u].off;
                        out_len[dst] = rw[u].len;
                    }
                }
            }
            __syncthreads();  // run_pos / run_x are rewritten by the next round
        }
        const uint64_t batch = (p.ncand - c) < kBatch ? (p.ncand - c) : kBatch;
        if (filled + total <= W) {
            filled += total;
            c += batch;
            s = 0;
        } else {
            // the window ends inside candidate `key`: resume there next window with its rows already sent
            if (threadIdx.x == 0) first_cross = 0xffffffffu;
            __syncthreads();
            uint64_t acc = pos, acc_mine = 0;
            int mine = -1;
#pragma unroll
            for (int u = 0; u < kCand; ++u) {
                if (mine < 0 && cnts[u] > 0 && filled + acc + cnts[u] > W) {
                    mine = u;
                    acc_mine = acc;
                }
                acc += cnts[u];
            }
            if (mine >= 0) atomicMin(&first_cross, threadIdx.x * kCand + (uint32_t)mine);
            __syncthreads();
            const uint32_t key = first_cross;
            if (threadIdx.x == key / kCand) {
                uint64_t skm = 0;
#pragma unroll
                for (int u = 0; u < kCand; ++u)
                    if (u == (int)(key % kCand)) skm = sks[u];
                scan[kFillWaves + 1] = W - filled - acc_mine + skm;
            }
            __syncthreads();
            s = scan[kFillWaves + 1];
            c = c + key;
            filled = W;
            __syncthreads();
        }
    }
    if (threadIdx.x == 0 && s0 == 0) {
        S->meta = j;
        S->cand = c;
        S->sub = s;
        S->n_window = filled;
        if (j >= L.J) S->exhausted = 1;
        // the window's longest claim, in 64-pair chunks: k_pair_test visits no chunk beyond it
        if (filled) atomicMax(&L.flags[kFlagChunks], (uint32_t)((filled + 63) / 64));
    }
    const uint64_t clk1 = L.fill_clock ? __builtin_amdgcn_s_memtime() : 0;
    if (slice) {
        // this part's pairs into the claim's histogram (and its pooled family's); k_fill_sort places them
        __shared__ uint32_t sh[kSortBins];
        for (uint32_t i = threadIdx.x; i < kSortBins; i += kFillThreads) sh[i] = 0;
        __syncthreads();  // every thread's writes of this part's pairs are complete, sh cleared
        const uint64_t e = filled < s1 ? filled : s1;
        const uint32_t blk_s = q.hash_kind >= DSY_SHA384 ? 128u : 64u, lenb_s = q.hash_kind >= DSY_SHA384 ? 16u : 8u;
        for (uint64_t t = s0 + threadIdx.x; t < e; t += kFillThreads)
            atomicAdd(&sh[kSortBins - 1u - min(n_blocks(q.prefix_len + out_len[t], blk_s, lenb_s), kSortBins - 1)], 1u);
        __syncthreads();
        uint32_t* gh = L.bulk_hist + (uint64_t)a_slot * kSortBins;
        const uint32_t fam_s = family_id(q.hash_kind, q.chunk_bytes, q.prefix_len);
        uint32_t* ph = ((L.pool_mask >> fam_s) & 1u) ? L.pool_counts->hist[fam_s] : nullptr;
        for (uint32_t i = threadIdx.x; i < kSortBins; i += kFillThreads)
            if (sh[i]) {
                atomicAdd(&gh[i], sh[i]);
                if (ph) atomicAdd(&ph[i], sh[i]);
            }
        if (threadIdx.x == 0 && s0 == 0) S->sort_later = 1;
        if (ph && threadIdx.x == 0) L.pool_counts->split[fam_s] = 1;  // no pool_tab rows: the scatter's atomics
        if (L.fill_clock && threadIdx.x == 0 && s0 == 0) {
            uint64_t* fc = L.fill_clock + (uint64_t)a_slot * 4;
            fc[0] = clk0;
            fc[1] = clk1;
            fc[2] = __builtin_amdgcn_s_memtime();
            fc[3] = clk_start;
        }
        return;
    }
    // Load balance: order this window's pairs by compression-block count (counting sort in LDS) so the 64
    // lanes of a hashing wave run the same number of blocks.  task[i] = the pair hashed by lane-slot i (blob
    // offset, length, window slot), so the hashing kernel reads 16 contiguous bytes per lane and then the packet;
    // the send order (slot order) is untouched.
    // Bins run from the most blocks down, so the longest packets start first (they set the window's tail).
    __shared__ uint32_t hist[kSortBins];
    const uint32_t blk = q.hash_kind >= DSY_SHA384 ? 128u : 64u, lenb = q.hash_kind >= DSY_SHA384 ? 16u : 8u;
    auto bin_of = [&](uint64_t len) {
        return (uint32_t)kSortBins - 1u - min(n_blocks(q.prefix_len + (uint32_t)len, blk, lenb), (uint32_t)kSortBins - 1);
    };
    for (uint32_t i = threadIdx.x; i < kSortBins; i += kFillThreads) hist[i] = 0;
    // small windows (the common case): every pair's (offset, length) loaded once, in one round, into registers
    const bool in_regs = filled <= (uint64_t)kFillThreads * kSortReg;
    __syncthreads();  // the selection's placements (other threads' writes) are complete
    if (!in_regs && regs_rows) {
        // the window outgrew the registers: their pairs' offsets go to pair_off like every other pair's
#pragma unroll
        for (int u = 0; u < kSortReg; ++u) {
            const uint64_t t = threadIdx.x + (uint64_t)kFillThreads * u;
            if (t < regs_rows) out_off[t] = ((uint64_t)reg_off[u] << 7) + kLineBias;
        }
    }
    if (in_regs && regs_rows < filled) {
#pragma unroll
        for (int u = 0; u < kSortReg; ++u) {
            const uint64_t t = threadIdx.x + (uint64_t)kFillThreads * u;
            if (t >= regs_rows) {
                reg_off[u] = t < filled ? (uint32_t)(out_off[t] >> 7) : 0u;
                reg_len[u] = t < filled ? out_len[t] : 0;
            }
        }
    }
    __syncthreads();
    if (in_regs) {
#pragma unroll
        for (int u = 0; u < kSortReg; ++u)
            if (threadIdx.x + (uint64_t)kFillThreads * u < filled) atomicAdd(&hist[bin_of(reg_len[u])], 1u);
    } else {
        for (uint64_t t = threadIdx.x; t < filled; t += kFillThreads) atomicAdd(&hist[bin_of(out_len[t])], 1u);
    }
    __syncthreads();
    const uint32_t fam = family_id(q.hash_kind, q.chunk_bytes, q.prefix_len);
    const bool pooled = (L.pool_mask >> fam) & 1u;
    if (pooled) {  // a pooled family: the window's counts go into the family's histogram too
        uint32_t* ph = L.pool_counts->hist[fam];
        uint32_t* tc = L.pool_tab + (uint64_t)a_slot * kSortBins;  // (pool_scan) the claim's counts, every bin
        for (uint32_t i = threadIdx.x; i < kSortBins; i += kFillThreads) {
            if (hist[i]) atomicAdd(&ph[i], hist[i]);
            if (L.pool_scan) tc[i] = hist[i];
        }
        __syncthreads();
    }
    if (may_split && filled > kSplitSortMin) {
        if (pooled && threadIdx.x == 0) L.pool_counts->split[fam] = 1;
        // a big window this one workgroup selected (a claim whose global times hold 10^4-10^5 rows each, config
        // 5's Zipf): its pairs are placed by k_fill_sort's workgroups, kBulkChunk each, from this histogram
        uint32_t* gh = L.bulk_hist + (uint64_t)a_slot * kSortBins;
        for (uint32_t i = threadIdx.x; i < kSortBins; i += kFillThreads) gh[i] = hist[i];
        if (threadIdx.x == 0) S->sort_later = 1;
        if (L.fill_clock && threadIdx.x == 0) {
            uint64_t* fc = L.fill_clock + (uint64_t)a_slot * 4;
            fc[0] = clk0;
            fc[1] = clk1;
            fc[2] = __builtin_amdgcn_s_memtime();
            fc[3] = clk_start;
        }
        return;
    }
    if (threadIdx.x < 64) {  // exclusive scan of the kSortBins counters by one wave
        const uint32_t per = kSortBins / 64, lane = threadIdx.x;
        uint32_t sum = 0;
        for (uint32_t i = 0; i < per; ++i) sum += hist[lane * per + i];
        uint32_t incl = sum;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(incl, d, 64);
            if ((int)lane >= d) incl += o;
        }
        uint32_t run = incl - sum;
        for (uint32_t i = 0; i < per; ++i) {
            const uint32_t h = hist[lane * per + i];
            hist[lane * per + i] = run;
            run += h;
        }
    }
    __syncthreads();
    if (pooled && L.pool_scan) {  // the claim's bin starts in its task order (k_pool_scan makes them offsets)
        uint32_t* ts = L.pool_tab + ((uint64_t)L.R + a_slot) * kSortBins;
        for (uint32_t i = threadIdx.x; i < kSortBins; i += kFillThreads) ts[i] = hist[i];
    }
    PairTask* task = L.task + (uint64_t)a_slot * W;
    if (in_regs) {
#pragma unroll
        for (int u = 0; u < kSortReg; ++u) {
            const uint64_t t = threadIdx.x + (uint64_t)kFillThreads * u;
            if (t < filled) {
                PairTask tk;
                tk.off = ((uint64_t)reg_off[u] << 7) + kLineBias;
                tk.len = reg_len[u];
                tk.slot = (uint32_t)t;
                task[atomicAdd(&hist[bin_of(tk.len)], 1u)] = tk;
            }
        }
    } else {
        for (uint64_t t = threadIdx.x; t < filled; t += kFillThreads) {
            PairTask tk;
            tk.off = out_off[t];
            tk.len = out_len[t];
            tk.slot = (uint32_t)t;
            task[atomicAdd(&hist[bin_of(tk.len)], 1u)] = tk;
        }
    }
    if (L.fill_clock && threadIdx.x == 0) {
        uint64_t* fc = L.fill_clock + (uint64_t)a_slot * 4;
        fc[0] = clk0;
        fc[1] = clk1;
        fc[2] = __builtin_amdgcn_s_memtime();
        fc[3] = clk_start;  // k_fill_first: before the claim's host reads and plan (k_fill: == clk0)
    }
}

// a pooled claim without a window this round: its pool_tab counts row reads zero in k_pool_scan
__device__ __forceinline__ void pool_row_zero(const RespondLaunch& L, uint32_t a_slot, const DevRequest& q) {
    if (!L.pool_scan || !((L.pool_mask >> family_id(q.hash_kind, q.chunk_bytes, q.prefix_len)) & 1u)) return;
    for (uint32_t i = threadIdx.x; i < kSortBins; i += blockDim.x) L.pool_tab[(uint64_t)a_slot * kSortBins + i] = 0;
}

// A split window: a claim that keeps every live row of a span (a scan with modulo 1, ASC or DESC) and has at least W
// candidates left in its current meta fills its window with gridDim.y workgroups, part p taking pairs
// [p * kBulkChunk, (p + 1) * kBulkChunk) -- candidate -> row is arithmetic, so every part knows its pairs' slots without
// the others.  The block-count sort stays one sort over the whole window (a heavy-tailed window sorted part by part
// spreads its few 64 KB packets over many hashing waves): the parts add their histograms into the claim's
// bulk_hist, and k_fill_sort places every part's pairs from the scanned totals.  Part 0 files the window; the cursor
// is committed by k_compact, since the other parts read it while this launch runs.  (A config 5 claim whose filter
// covers its 10^5-10^6 rows walks them in 2^18-pair windows: one workgroup per claim left the chip idle, 1-2 ms per
// window.)
#ifndef DSY_BULK_UNROLL
#define DSY_BULK_UNROLL 16  // pairs per thread of a split window's part (8: 2048-pair parts)
#endif
static constexpr uint64_t kBulkChunk = (uint64_t)kFillThreads * DSY_BULK_UNROLL;
// k_fill: an enumerating claim with at most this many candidates left fills a window of >= 2 parts part by part
static constexpr uint64_t kSliceCands = 2048;

__device__ __forceinline__ bool bulk_window(const RespondLaunch& L, const DevRequest& q, const ReqState& S,
                                            const Plan& p) {
    // (a claim's last, partial window of such a span splits too: one workgroup walking 2^18 rows took ~0.4 ms)
    return S.meta < L.J && S.sub == 0 && p.mode == 0 && q.modulo <= 1 && p.dir != DSY_RANDOM && S.cand < p.ncand &&
           p.ncand - S.cand >= 2 * kBulkChunk;
}

// A split window's pair t is candidate win_cand + t of the plan's span: its store row is arithmetic (the span's
// candidates are consecutive live rows), so the fill writes no per-pair row / offset / length for it -- k_fill_sort
// and k_compact recompute them from the row records.
__device__ __forceinline__ uint64_t bulk_row(const RespondLaunch& L, const Plan& p, uint64_t c0, uint64_t t) {
    const uint64_t ci = c0 + t;
    const uint64_t lr = p.a + (p.dir == DSY_DESC ? p.ncand - 1 - ci : ci);
    return L.st.live_row ? L.st.live_row[lr] : lr;
}

__device__ __forceinline__ uint32_t sort_bin(const DevRequest& q, uint32_t len) {
    const uint32_t blk = q.hash_kind >= DSY_SHA384 ? 128u : 64u, lenb = q.hash_kind >= DSY_SHA384 ? 16u : 8u;
    return (uint32_t)kSortBins - 1u - min(n_blocks(q.prefix_len + len, blk, lenb), (uint32_t)kSortBins - 1);
}

__device__ __forceinline__ void fill_bulk_part(const RespondLaunch& L, uint32_t a_slot, uint32_t part,
                                               const DevRequest& q, ReqState* S, const Plan& p, uint64_t c) {
    __shared__ uint32_t hist[kSortBins];
    const uint64_t W = L.window;
    const uint64_t nw = p.ncand - c < W ? p.ncand - c : W;  // this window's pairs: the span's rest, at most W
    const uint64_t base = (uint64_t)part * kBulkChunk;
    if (base >= nw) return;
    const uint64_t n = nw - base < kBulkChunk ? nw - base : kBulkChunk;
    uint64_t* mask = L.miss_mask + (uint64_t)a_slot * (W / 64) + base / 64;
    for (uint64_t w = threadIdx.x; w < (n + 63) / 64; w += kFillThreads) mask[w] = 0;
    for (uint32_t i = threadIdx.x; i < kSortBins; i += kFillThreads) hist[i] = 0;
    const RowRec* __restrict__ rec = L.st.rec;
    constexpr int kU = (int)(kBulkChunk / kFillThreads);
    uint32_t len[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const uint64_t t = threadIdx.x + (uint64_t)kFillThreads * u;
        len[u] = t < n ? rec[bulk_row(L, p, c, base + t)].len : 0u;  // (only the histogram: bulk_row)
    }
    __syncthreads();  // hist cleared
#pragma unroll
    for (int u = 0; u < kU; ++u)
        if (threadIdx.x + (uint64_t)kFillThreads * u < n) atomicAdd(&hist[sort_bin(q, len[u])], 1u);
    __syncthreads();
    uint32_t* gh = L.bulk_hist + (uint64_t)a_slot * kSortBins;
    const uint32_t fam = family_id(q.hash_kind, q.chunk_bytes, q.prefix_len);
    uint32_t* ph = ((L.pool_mask >> fam) & 1u) ? L.pool_counts->hist[fam] : nullptr;
    for (uint32_t i = threadIdx.x; i < kSortBins; i += kFillThreads)
        if (hist[i]) {
            atomicAdd(&gh[i], hist[i]);
            if (ph) atomicAdd(&ph[i], hist[i]);
        }
    if (part == 0 && threadIdx.x == 0) {
        if (ph) L.pool_counts->split[fam] = 1;  // no pool_tab rows: the scatter's atomics
        S->n_window = nw;
        S->cand_next = c + nw;
        S->commit = 1;
        // the span's rest in the last meta: every candidate visited (the next meta, if any, starts next window)
        if (c + nw >= p.ncand && S->win_meta + 1 >= L.J) S->exhausted = 1;
        atomicMax(&L.flags[kFlagChunks], (uint32_t)((nw + 63) / 64));
    }
}

// The split windows' sort: every part places its pairs at the claim's bin starts (scan of bulk_hist) plus the ranges
// it reserves per bin in bulk_cur (one atomic per part and bin); slots inside a bin come in no particular order.
__global__ void __launch_bounds__(kFillThreads) k_fill_sort(RespondLaunch L) {
    __shared__ uint32_t start[kSortBins];
    __shared__ uint32_t hist[kSortBins];
    const uint32_t a_slot = blockIdx.x, part = blockIdx.y;
    const uint32_t r = L.act[a_slot];
    const ReqState* S = &L.state[r];
    if (S->done || !(S->commit || S->sort_later)) return;  // k_fill sorted it whole
    const uint64_t W = L.window;
    const uint64_t nw = S->n_window;  // (W for a split window)
    if (nw > W) {  // (cannot happen: the fill never places more than W pairs)
        if (threadIdx.x == 0) guard_trip(L.h_status, kGuardWindow);
        return;
    }
    const uint64_t base = (uint64_t)part * kBulkChunk;
    if (base >= nw) return;
    const uint64_t n = nw - base < kBulkChunk ? nw - base : kBulkChunk;
    const DevRequest& q = L.reqs[r];
    const uint32_t* gh = L.bulk_hist + (uint64_t)a_slot * kSortBins;
    for (uint32_t i = threadIdx.x; i < kSortBins; i += kFillThreads) {
        start[i] = gh[i];
        hist[i] = 0;
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // exclusive scan of the claim's totals by one wave
        const uint32_t per = kSortBins / 64, lane = threadIdx.x;
        uint32_t sum = 0;
        for (uint32_t i = 0; i < per; ++i) sum += start[lane * per + i];
        uint32_t incl = sum;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(incl, d, 64);
            if ((int)lane >= d) incl += o;
        }
        uint32_t run = incl - sum;
        for (uint32_t i = 0; i < per; ++i) {
            const uint32_t h = start[lane * per + i];
            start[lane * per + i] = run;
            run += h;
        }
    }
    const uint32_t* len_w = L.pair_len + (uint64_t)a_slot * W + base;
    const uint64_t* off_w = L.pair_off + (uint64_t)a_slot * W + base;
    constexpr int kU = (int)(kBulkChunk / kFillThreads);
    uint32_t len[kU];
    uint64_t off[kU];
    // a split window (fill_bulk_part): the pairs' rows are arithmetic and their records are re-read, once
    const bool bulk = S->commit;
    const Plan bp = bulk ? L.plans[(uint64_t)r * L.J + S->win_meta] : Plan{};
    const uint64_t c0 = S->win_cand;
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const uint64_t t = threadIdx.x + (uint64_t)kFillThreads * u;
        RowRec rr{};
        if (t < n) {
            if (bulk) rr = L.st.rec[bulk_row(L, bp, c0, base + t)];
            else rr = RowRec{off_w[t], len_w[t], 0u};
        }
        len[u] = rr.len;
        off[u] = rr.off;
    }
    __syncthreads();  // starts scanned
#pragma unroll
    for (int u = 0; u < kU; ++u)
        if (threadIdx.x + (uint64_t)kFillThreads * u < n) atomicAdd(&hist[sort_bin(q, len[u])], 1u);
    __syncthreads();
    uint32_t* gc = L.bulk_cur + (uint64_t)a_slot * kSortBins;
    for (uint32_t i = threadIdx.x; i < kSortBins; i += kFillThreads)
        if (hist[i]) hist[i] = start[i] + atomicAdd(&gc[i], hist[i]);  // this part's range in bin i
    __syncthreads();
    PairTask* task = L.task + (uint64_t)a_slot * W;
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const uint64_t t = threadIdx.x + (uint64_t)kFillThreads * u;
        if (t < n) {
            PairTask tk;
            tk.off = off[u];
            tk.len = len[u];
            tk.slot = (uint32_t)(base + t);
            // the position lies in [0, nw) when bulk_hist holds exactly this window's counts; a stale count (state a
            // window left behind) would place past the claim's slot: refuse the write and fail the call loudly
            const uint32_t pos = atomicAdd(&hist[sort_bin(q, len[u])], 1u);
            if (pos < nw) task[pos] = tk;
            else guard_trip(L.h_status, kGuardSortPos);
        }
    }
}

// ------------------------------------------------------------------------------------ k_pool_scatter
// A pooled family's window pairs -- its listed claims' task records, each claim's sorted by block count on its own --
// into one block-count order over all of them, L.pool[0 .. total), longest first.  With ~300 pairs per claim
// (the SHA-1 test filters of node.py:617 hold 284 keys) a claim's 64-pair chunks each span several block counts, and
// a claim's last chunk is partly empty; pooled, every hashing wave but the last runs 64 lanes of one block count.
// Workgroup (x, y) takes parts y, y + gridDim.y, ... (kPoolPart pairs each) of claim list[x]'s window: the family's
// histogram (k_fill) scanned in LDS gives every bin's start, one atomic per (workgroup, part, bin) its range in the
// bin.  Workgroup (0, 0) also publishes the total and resets the wave-task queue.
static constexpr uint64_t kPoolPart = 1024;

// The per-(claim, bin) exclusive scan (L.pool_scan): k_fill left every listed claim's block-count histogram (counts
// row) and its bins' starts in its own task order (starts row) in L.pool_tab; here bin b's column of counts is
// scanned over the list's claims, and every nonzero entry's starts-row word becomes (offset of the claim's first pair
// of bin b among the family's pairs of bin b) - (its start in the claim's task order).  k_pool_scatter then places
// task[j] at bin_start[b] + that word + j: no atomics, no cursor contention.  Workgroup g takes bins 64 g .. 64 g + 63
// (lane = bin, coalesced 256-byte row pieces); its 16 waves take consecutive ranges of the list.  A family with a
// split window (k_fill_sort's order, no rows) keeps the scatter's atomics: both kernels read the same flag.
__global__ void __launch_bounds__(1024) k_pool_scan(RespondLaunch L, const uint32_t* __restrict__ list, uint32_t n_list,
                                                    uint32_t fam) {
    __shared__ uint32_t part[16][64];
    if (L.pool_counts->split[fam]) return;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t bin = blockIdx.x * 64 + lane;
    const uint32_t per = (n_list + 15) / 16;
    const uint32_t x0 = min(wv * per, n_list), x1 = min(x0 + per, n_list);
    const uint32_t* tc = L.pool_tab + bin;
    uint32_t* ts = L.pool_tab + (uint64_t)L.R * kSortBins + bin;
    // 64 rows at a time: lane i holds row c0 + i's window slot, every row's count is one load at a wave-uniform row
    // address, all 64 in flight together (a claim without a window this round has a zero counts row: k_fill)
    auto load = [&](uint32_t c0, uint32_t* cnt) -> uint32_t {
        const uint32_t my = c0 + lane < x1 ? list[c0 + lane] : ~0u;
#pragma unroll
        for (int k = 0; k < 64; ++k) {
            const uint32_t a = __builtin_amdgcn_readlane(my, k);
            cnt[k] = a != ~0u ? tc[(uint64_t)a * kSortBins] : 0u;
        }
        return my;
    };
    uint32_t cnt[64], my = ~0u, sum = 0;
    const bool one = x1 - x0 <= 64;  // (the common case, <= 1024 claims: the counts stay in registers)
    for (uint32_t c0 = x0; c0 < x1; c0 += 64) {
        my = load(c0, cnt);
#pragma unroll
        for (int k = 0; k < 64; ++k) sum += cnt[k];
    }
    part[wv][lane] = sum;
    __syncthreads();
    uint32_t off = 0;
    for (uint32_t v = 0; v < wv; ++v) off += part[v][lane];
    for (uint32_t c0 = x0; c0 < x1; c0 += 64) {
        if (!one) my = load(c0, cnt);
#pragma unroll
        for (int h = 0; h < 64; h += 32) {  // 32 starts loaded, then their offsets stored: no store between loads
            uint32_t st[32];
#pragma unroll
            for (int k = 0; k < 32; ++k)
                st[k] = cnt[h + k] ? ts[(uint64_t)__builtin_amdgcn_readlane(my, h + k) * kSortBins] : 0u;
#pragma unroll
            for (int k = 0; k < 32; ++k)
                if (cnt[h + k]) {
                    ts[(uint64_t)__builtin_amdgcn_readlane(my, h + k) * kSortBins] = off - st[k];
                    off += cnt[h + k];
                }
        }
    }
}

__global__ void __launch_bounds__(256) k_pool_scatter(RespondLaunch L, const uint32_t* __restrict__ list, uint32_t fam) {
    __shared__ uint32_t start[kSortBins];
    __shared__ uint32_t lh[kSortBins];
    const uint32_t a_slot = list[blockIdx.x];
    const uint32_t r = L.act[a_slot];
    const uint64_t W = L.window;
    const uint64_t n = L.state[r].n_window;
    PoolCounts* pc = L.pool_counts;
    const bool first = blockIdx.x == 0 && blockIdx.y == 0;
    const uint64_t base0 = (uint64_t)blockIdx.y * kPoolPart;
    if (base0 >= n && !first) return;
    for (uint32_t i = threadIdx.x; i < kSortBins; i += 256) {
        start[i] = pc->hist[fam][i];
        lh[i] = 0;
    }
    __syncthreads();
    bins_exclusive_scan(start, first ? &pc->total[fam] : nullptr);
    if (first && threadIdx.x == 0) pc->next[fam] = 0;
    __syncthreads();
    const DevRequest& q = L.reqs[r];
    const PairTask* task = L.task + (uint64_t)a_slot * W;
    if (L.pool_scan && !pc->split[fam]) {  // k_pool_scan's offsets: pair j of bin b goes to start[b] + delta[b] + j
        const uint32_t* delta = L.pool_tab + ((uint64_t)L.R + a_slot) * kSortBins;
        const uint64_t cap = (uint64_t)L.n_act * W;
        for (uint64_t base = base0; base < n; base += (uint64_t)gridDim.y * kPoolPart)
            for (uint64_t j = base + threadIdx.x; j < n && j < base + kPoolPart; j += 256) {
                const PairTask tk = task[j];
                const uint32_t b = sort_bin(q, tk.len);
                PoolTask p;
                p.line = (uint32_t)(tk.off >> 7);  // off = line * 128 + kLineBias
                p.len = tk.len;
                p.a_slot = a_slot;
                p.slot = tk.slot;
                const uint32_t pos = start[b] + delta[b] + (uint32_t)j;
                if (pos < cap) L.pool[pos] = p;  // (always: the counts are this window's pairs)
            }
        return;
    }
    for (uint64_t base = base0; base < n; base += (uint64_t)gridDim.y * kPoolPart) {
        const uint64_t cnt = n - base < kPoolPart ? n - base : kPoolPart;
        constexpr int kU = (int)(kPoolPart / 256);
        PairTask tk[kU];
        uint32_t bin[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const uint64_t t = threadIdx.x + 256ull * u;
            if (t < cnt) {
                tk[u] = task[base + t];
                bin[u] = sort_bin(q, tk[u].len);
            }
        }
#pragma unroll
        for (int u = 0; u < kU; ++u)
            if (threadIdx.x + 256ull * u < cnt) atomicAdd(&lh[bin[u]], 1u);
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < kSortBins; i += 256)
            if (lh[i]) lh[i] = start[i] + atomicAdd(&pc->cur[fam][i], lh[i]);
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            if (threadIdx.x + 256ull * u < cnt) {
                PoolTask p;
                p.line = (uint32_t)(tk[u].off >> 7);  // off = line * 128 + kLineBias
                p.len = tk[u].len;
                p.a_slot = a_slot;
                p.slot = tk[u].slot;
                const uint32_t pos = atomicAdd(&lh[bin[u]], 1u);
                if (pos < (uint64_t)L.n_act * W) L.pool[pos] = p;  // (always: the counts are this window's pairs)
            }
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < kSortBins; i += 256) lh[i] = 0;
        __syncthreads();
    }
}

__device__ uint32_t g_fill_skew = 0;  // set_fill_skew (diagnostics)

hipError_t set_fill_skew(uint32_t sleeps) { return hipMemcpyToSymbol(HIP_SYMBOL(g_fill_skew), &sleeps, sizeof sleeps); }

__global__ void __launch_bounds__(kFillThreads) __attribute__((amdgpu_waves_per_eu(4, 8))) k_fill(RespondLaunch L) {
    const uint32_t a_slot = blockIdx.x, part = blockIdx.y;
    const uint64_t clk0 = L.fill_clock ? __builtin_amdgcn_s_memtime() : 0;
    const uint32_t r = L.act[a_slot];
    ReqState* S = &L.state[r];
    if (S->done) {
        if (part == 0 && threadIdx.x == 0) S->n_window = 0;
        if (part == 0) pool_row_zero(L, a_slot, L.reqs[r]);
        return;
    }
    const Plan* plans = L.plans + (uint64_t)r * L.J;
    if (gridDim.y > 1) {  // a split window when the claim allows one: every part decides from the window's start cursor
        ReqState st = *S;
        st.meta = S->win_meta;
        st.cand = S->win_cand;
        st.sub = S->win_sub;
        if (st.meta < L.J) {
            const Plan p = plans[st.meta];
            if (bulk_window(L, L.reqs[r], st, p)) {
                fill_bulk_part(L, a_slot, part, L.reqs[r], S, p, st.cand);
                return;
            }
            // an enumeration with few candidates left, each global time possibly holding 10^4-10^5 rows (config 5's
            // Zipf global times): every part selects alike from the window-start cursor and writes its slice
            if (p.mode == 1 && st.cand <= p.ncand && p.ncand - st.cand <= kSliceCands) {
                const uint64_t s0 = (uint64_t)part * kBulkChunk;
                if (s0 >= L.window) return;
                fill_claim(L, a_slot, r, L.reqs[r], S, st.meta, st.cand, st.sub, [&](uint32_t j) { return plans[j]; },
                           clk0, clk0, false, true, s0, s0 + kBulkChunk);
                return;
            }
        }
        if (part > 0) return;
    }
    // (k_fill_sort runs after this launch whenever it has parts: a big window may leave its placement to it)
    // The window's start cursor, read once for the workgroup: fill_claim's thread 0 writes the next cursor into S when
    // its selection ends, and a wave that read S only after that (waves of a workgroup start at different times; one
    // scheduled late under a busy GPU did) would select nothing -- its pairs then missing from the window's sort,
    // their task records left from an earlier window (k_pair_test's kGuardTask check caught it; tools/r6_cfg5_audit.sh)
    __shared__ uint32_t c_meta;
    __shared__ uint64_t c_cand, c_sub;
    if (const uint32_t skew = g_fill_skew; skew && threadIdx.x >= 64)
        for (uint32_t i = 0; i < skew; ++i) __builtin_amdgcn_s_sleep(127);
    if (threadIdx.x == 0) {
        c_meta = S->meta;
        c_cand = S->cand;
        c_sub = S->sub;
    }
    __syncthreads();
    fill_claim(L, a_slot, r, L.reqs[r], S, c_meta, c_cand, c_sub, [&](uint32_t j) { return plans[j]; }, clk0, clk0,
               gridDim.y > 1);
}

// First window of a call whose claims all serve one meta with device-side output capacities (respond_core's common
// case): k_setup's work fused into k_fill -- one launch and one dependent chain per claim instead of two kernels.
// Every workgroup copies its share of the staged upload (pinned host memory -> the device copy later kernels read);
// workgroup a_slot reads its own claim and meta straight from the host copy, plans the claim (one lane), initialises
// its state and fills its first window.  The status counters are zeroed by workgroup 0 (flags[kFlagChunks], which
// the workgroups raise, is zero between calls: k_compact resets it).  identity_act: window slot a serves claim a.
__global__ void __launch_bounds__(kFillThreads) __attribute__((amdgpu_waves_per_eu(4, 8))) k_fill_first(RespondLaunch L, const uint4* __restrict__ src,
                                                             uint4* __restrict__ dst, uint32_t in_words,
                                                             uint4* __restrict__ counters, uint32_t counter_words,
                                                             uint64_t per_claim_cap, const uint32_t* __restrict__ h_act) {
    __shared__ DevRequest sq;
    __shared__ Plan sp;
    __shared__ ReqState sst;
    const uint32_t a_slot = blockIdx.x;
    const uint64_t clk0 = L.fill_clock ? __builtin_amdgcn_s_memtime() : 0;
    const uint32_t tid = blockIdx.x * kFillThreads + threadIdx.x, nthr = gridDim.x * kFillThreads;
    // the host reads of this thread are all issued before the first is consumed (each is a PCIe round trip)
    constexpr uint32_t kQw = sizeof(DevRequest) / 16, kMw = sizeof(SegMeta) / 16;
    const uint32_t r = h_act ? h_act[a_slot] : a_slot;
    uint4 w = make_uint4(0, 0, 0, 0);
    if (threadIdx.x < kQw) w = src[(size_t)r * kQw + threadIdx.x];
    else if (threadIdx.x < kQw + kMw) w = src[(size_t)L.R * kQw + (threadIdx.x - kQw)];
    uint4 cw = make_uint4(0, 0, 0, 0);
    if (tid < in_words) cw = src[tid];
    if (tid < in_words) dst[tid] = cw;
    for (uint32_t i = tid + nthr; i < in_words; i += nthr) dst[i] = src[i];
    if (blockIdx.x == 0)
        for (uint32_t i = threadIdx.x; i < counter_words; i += kFillThreads) counters[i] = make_uint4(0, 0, 0, 0);
    // this window slot's split-window sort state starts the call at zero (as k_setup's loop does)
    if (L.bulk_zero)
        for (uint32_t i = threadIdx.x; i < kSortBins; i += kFillThreads)
            L.bulk_hist[(uint64_t)a_slot * kSortBins + i] = L.bulk_cur[(uint64_t)a_slot * kSortBins + i] = 0;
    if (threadIdx.x < kQw) ((uint4*)&sq)[threadIdx.x] = w;
    else if (threadIdx.x < kQw + kMw) ((uint4*)&sp)[threadIdx.x - kQw] = w;  // the SegMeta, parked in sp
    __syncthreads();
    if (threadIdx.x == 0) {
        SegMeta mt;
        __builtin_memcpy(&mt, &sp, sizeof mt);
        const uint64_t span = plan_one(L, sq, mt, r, r, 0, &sp);  // and in L.plans[r] for later windows
        L.upper[r] = span;
        ReqState st{};
        st.cap = min(span, per_claim_cap);
        st.out_base = (uint64_t)r * per_claim_cap;
        st.done = span == 0;
        sst = st;
    }
    __syncthreads();
    ReqState* S = &L.state[r];
    if (sst.done) {
        if (threadIdx.x == 0) S[0] = sst;  // n_window = 0
        pool_row_zero(L, a_slot, sq);
        return;
    }
    if (threadIdx.x == 0) S[0] = sst;  // the cursor fields are rewritten by fill_claim's thread 0 below
    fill_claim(L, a_slot, r, sq, S, 0u, 0ull, 0ull, [&](uint32_t) { return sp; }, clk0,
               L.fill_clock ? __builtin_amdgcn_s_memtime() : 0);
}

// -------------------------------------------------------------------------------------- k_pair_test
// DIAG (DMA, 2-byte chunks; DSY_PAIR_DIAG): 0 the product kernel, 1 no packet loads (compute ceiling), 2 packet
// loads without the compression (gather ceiling) -- diagnostics only, their answers are meaningless
// Registers: 128 VGPRs (4 waves per SIMD, as the 8 KiB-per-wave LDS allows 5).  Forcing 5 waves (96 VGPRs) spills
// per task and measured 234 -> 338 us per headline launch.
// Measured and dropped: half-line staging (two 4 KiB buffers, one block's words live, 95 VGPRs, 5 waves per SIMD)
// ran the headline launch in the same 234 us (compute ceiling 175 us, gather ceiling 191 us vs 176 for full lines).
// POOL: the wave-tasks are 64 consecutive pairs of the family's pooled order (k_pool_scatter): the claim -- filter,
// prefix, m, k -- is per lane.  pool_queue: waves take wave-tasks from a queue (longest first) instead of the grid
// stride.
static constexpr uint32_t kPairRedBytes = 32;  // a wave's end-of-launch sums in LDS (direct-load kernels)
// DSY_PAIR_WAVES5=1 builds the padded line-staged kernel for 5 waves per SIMD (<= 96 VGPRs; 5 workgroups x 4 x 8 KiB
// fill the CU's LDS). Measured and dropped (profiles/waves5_ab_r5.json): at 96 VGPRs the task setup spills and the
// launch ran 207-209 vs 202 us (headline), 108 vs 99 us (SHA-1 leg), 1064 vs 1050 us (config 5).
#ifndef DSY_PAIR_WAVES5
#define DSY_PAIR_WAVES5 0
#endif
static constexpr bool kPairWaves5 = DSY_PAIR_WAVES5;
template <class H, int CHUNK, bool DMA, int DIAG = 0, bool POOL = false, bool PADDED = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kPairWaves5 && DMA && PADDED ? 5 : 4, 8))) k_pair_test(RespondLaunch L, const uint32_t* __restrict__ req_list,
                                                   uint32_t n_list, uint32_t fam) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dma_lds[];
    const uint64_t W = L.window;
    uint64_t total_waves;
    uint32_t n_pool = 0;
    if constexpr (POOL) {
        n_pool = (uint32_t)min((uint64_t)L.pool_counts->total[fam], (uint64_t)L.n_act * W);
        total_waves = (n_pool + 63) / 64;
        if (blockIdx.x == 0) {  // the family's histogram and cursors start the next window at zero (k_fill adds)
            for (uint32_t i = threadIdx.x; i < kSortBins; i += blockDim.x)
                L.pool_counts->hist[fam][i] = L.pool_counts->cur[fam][i] = 0;
            if (threadIdx.x == 0) L.pool_counts->split[fam] = 0;
        }
    } else {
        // chunks per claim: the window's longest claim (k_fill), not W / 64 -- a claim of ~1000 pairs in a 4096-pair
        // window would otherwise leave 3/4 of the wave-tasks empty, each costing a dependent load chain to skip
        const uint64_t waves_per_req = min((uint64_t)L.flags[kFlagChunks], W / 64);
        total_waves = (uint64_t)n_list * waves_per_req;
    }
    const uint32_t lane = threadIdx.x & 63;
    // (wave-uniform in SGPRs: readfirstlane tells the compiler, so the task decode and the claim's state loads below
    // are scalar instructions, not 64-bit VALU arithmetic on every wave-task)
    const uint64_t wave0 = (uint64_t)blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t wstride = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const bool queue = POOL && L.pool_queue;
    auto next_task = [&]() -> uint64_t {
        uint32_t v = 0;
        if (lane == 0) v = atomicAdd(&L.pool_counts->next[fam], 1u);
        return (uint64_t)__builtin_amdgcn_readfirstlane(__shfl((int)v, 0, 64));
    };
    uint8_t* my_lds = dma_lds + (threadIdx.x >> 6) * DmaGeometry<2, 1>::kWaveBytes;
    unsigned long long acc_blocks = 0, acc_bytes = 0, acc_slots = 0;  // this lane's work, reduced once per block
    // deal: the resident grid (4 workgroups per CU) visits whole rounds of its waves, the wave-tasks permuted within
    // a round.  Workgroups i, i + G/4, i + G/2, i + 3G/4 share a CU (observed: tools/trace_summary.py over
    // DSY_PAIR_TRACE), and each SIMD holds one wave of each, in no fixed order.  A workgroup's four waves take four
    // consecutive wave-tasks (about equal), and the workgroups of a CU take positions c, G/2 - 1 - c, G/2 + c,
    // G - 1 - c of the G workgroup positions (snaking over the quarters), so every SIMD's four waves sum to about the
    // mean when the wave-tasks come longest first.  Later rounds snake back.
    const uint32_t nl_recip = n_list > 1 ? mod_recip(n_list) : 0u;  // ceil(2^32 / n_list): the task -> claim split
    const bool deal = L.pool_deal && gridDim.x % 4 == 0;
    const uint64_t wend = deal ? (total_waves + wstride - 1) / wstride * wstride : total_waves;
    for (uint64_t wv = queue ? next_task() : wave0; wv < wend; wv = queue ? next_task() : wv + wstride) {
        uint32_t a_slot, r, t = 0;
        bool active;
        const uint8_t* key = L.st.lines + DSY_BLOB_GUARD;  // idle lanes: an empty key past the guard
        uint32_t len = 0;
        uint64_t v = wv;
        if (deal) {
            const uint64_t R = wstride, G = gridDim.x, k = wv / R, x = wv % R;
            const uint64_t i = x / 4, q = i / (G / 4), c = i % (G / 4);
            const uint64_t pos = q * (G / 4) + ((q & 1) ? G / 4 - 1 - c : c);
            const uint64_t rank = 4 * pos + x % 4;
            v = k * R + ((k & 1) ? R - 1 - rank : rank);
            if (v >= total_waves) continue;  // wave-uniform
        }
        if constexpr (POOL) {
            const uint64_t i = v * 64 + lane;
            active = i < n_pool;
            const PoolTask pt = L.pool[active ? i : n_pool - 1];
            a_slot = pt.a_slot;
            r = L.act[a_slot];
            if (active) {
                const uint64_t off = ((uint64_t)pt.line << 7) + kLineBias;
                if (!packet_in_lines(off, pt.len, L.st.lines_bytes) || pt.slot >= W) {
                    guard_trip(L.h_status, kGuardTask);
                    active = false;
                } else {
                    t = pt.slot;
                    key = L.st.lines + off;
                    len = pt.len;
                }
            }
        } else {
            // chunk-major task order: wave-task v hashes 64-pair chunk (v / n_list) of claim (v % n_list), so the
            // non-empty chunks of every claim come first (the longest packets of each) and spread over the grid
            // (v < 2^32 on every real launch: one multiply-high instead of a 64-bit division per wave-task)
            uint64_t chunk, slot_i;
            if (v < (1ull << 32) && (n_list == 1 || nl_recip)) {
                uint32_t q = n_list > 1 ? __umulhi((uint32_t)v, nl_recip) : (uint32_t)v;  // floor(v / n) or one more
                int64_t rem = (int64_t)(uint32_t)v - (int64_t)q * n_list;
                if (rem < 0) { --q; rem += n_list; }
                chunk = q;
                slot_i = (uint64_t)rem;
            } else {
                chunk = v / n_list;
                slot_i = v % n_list;
            }
            a_slot = req_list[slot_i];
            r = L.act[a_slot];
            const uint64_t i0 = chunk * 64;
            const uint64_t n = L.state[r].n_window;
            if (i0 >= n) continue;  // wave-uniform: past this claim's window
            if (n > W) {  // wave-uniform (cannot happen: the fill never places more than W pairs)
                if (lane == 0) guard_trip(L.h_status, kGuardWindow);
                continue;
            }
            const uint64_t i = i0 + lane;
            active = i < n;
            if (active) {
                const PairTask tk = L.task[(uint64_t)a_slot * W + i];
                // bounds check of the packet the record names (a record the fill did not write this window would
                // address another store's line copy): skipped and reported, never dereferenced
                if (!packet_in_lines(tk.off, tk.len, L.st.lines_bytes) ||
                    tk.slot >= n) {
                    guard_trip(L.h_status, kGuardTask);
                    active = false;
                } else {
                    t = tk.slot;
                    key = L.st.lines + tk.off;
                    len = tk.len;
                }
            }
        }
        const DevRequest& q = L.reqs[r];
        KeyView kv{key, len, q.prefix, q.prefix_len};
        const uint64_t trace_t0 = L.trace ? __builtin_amdgcn_s_memrealtime() : 0;
        const uint32_t nb = active ? n_blocks(kv.plen + kv.len, H::block_bytes, H::len_bytes) : 0u;
        // lane-block slots this wave-task occupies: 64 x the longest lane (load-balance denominator)
        const uint32_t nbmax = wave_max_uniform(nb);
        // the SIMD's arbiter issues for the longest wave-tasks first: a heavy-tailed window's few 64 KB packets (1024
        // blocks of serial digest) set its end.  pair_prio 1 (default): tasks of >= 32 blocks (2 KB packets; config
        // 5: k_pair_test -4 %, the headline's packets never qualify); 2: every task by length (packets of 100-1500 B
        // too: headline and SHA-1 leg +1-4 %)
        const uint32_t prio_b = L.pair_prio == 2 ? nbmax * 16 : L.pair_prio == 1 ? nbmax : 0u;
        const bool raised = prio_b >= 32;  // wave-uniform
        if (raised) {
            if (prio_b >= 256) __builtin_amdgcn_s_setprio(3);
            else if (prio_b >= 64) __builtin_amdgcn_s_setprio(2);
            else __builtin_amdgcn_s_setprio(1);
        }
        H st;
        if constexpr (DMA) {
            // prefixes of 0 or > 4 bytes go to DMA = false
            // (the idle lanes' empty keys hash one block: a wave with no active lane still walks one stage)
            hash_key_dma_lines<H, DIAG, PADDED>(kv, st, my_lds, q.prefix_word, L.st.lines, max(nbmax, 1u));
        } else {
            hash_key<H>(kv, st);
        }
        if (raised) __builtin_amdgcn_s_setprio(0);
        const uint32_t* filt = (const uint32_t*)(L.filters + q.filter_offset);
        const uint64_t m = q.m_bits;
        const uint32_t ok = filter_has_all<H, CHUNK>(filt, st, q.k, m, q.m_recip);
        if (active) {
            // misses are rare (the requester holds most of its range): one atomic bit per missing pair
            if (!ok && DIAG == 0)  // (the diagnostics' digests are garbage: their misses would be mostly atomics)
                atomicOr((unsigned long long*)&L.miss_mask[(uint64_t)a_slot * (W / 64) + t / 64], 1ull << (t % 64));
            acc_blocks += nb;
            acc_bytes += kv.len;
        }
        if (lane == 0) acc_slots += 64ull * nbmax;
        if (L.trace && lane == 0) {  // diagnostics: the wave-task's place and time
            const uint32_t at = atomicAdd(L.trace_n, 1u);
            if (at < L.trace_cap) {
                WaveTrace w;
                w.hw_id = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
                w.xcc_id = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
                w.t0 = trace_t0;
                w.t1 = __builtin_amdgcn_s_memrealtime();
                w.blocks = nbmax;
                w.task = (uint32_t)wv;
                L.trace[at] = w;
            }
        }
    }
    // one set of atomics per workgroup (a contended atomic per wave-task would stall the next vmcnt wait of
    // every wave behind it); each wave's sums go through its own LDS stage buffer, free once its walk is done (no
    // static LDS: five workgroups of 4 x 8 KiB fill a CU's 160 KiB exactly)
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        acc_blocks += __shfl_xor(acc_blocks, d, 64);
        acc_bytes += __shfl_xor(acc_bytes, d, 64);
        acc_slots += __shfl_xor(acc_slots, d, 64);
    }
    // (the direct-load kernels launch with kPairRedBytes of LDS per wave for this)
    constexpr uint32_t kWaveLds = DMA ? DmaGeometry<2, 1>::kWaveBytes : kPairRedBytes;
    if (lane == 0) {
        unsigned long long* red = (unsigned long long*)(dma_lds + (threadIdx.x >> 6) * kWaveLds);
        red[0] = acc_blocks;
        red[1] = acc_bytes;
        red[2] = acc_slots;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long b = 0, y = 0, z = 0;
        for (uint32_t wv = 0; wv < blockDim.x / 64; ++wv) {
            const unsigned long long* red = (const unsigned long long*)(dma_lds + wv * kWaveLds);
            b += red[0], y += red[1], z += red[2];
        }
        if (b) atomicAdd(counter(L.counters, kCntBlocks), b);
        if (y) atomicAdd(counter(L.counters, kCntBytes), y);
        if (z) atomicAdd(counter(L.counters, kCntSlots), z);
    }
}

// pooled (fam: the family id): k_pool_scatter orders the listed claims' pairs into L.pool first; MD5, SHA-1 and
// SHA-256 only (the larger SHA-2 families take the per-claim order)
template <class H, int CHUNK>
static hipError_t pair_test_family(const RespondLaunch& L, bool long_prefix, const uint32_t* list, uint32_t n_list,
                                   bool pooled = false, uint32_t fam = 0, bool padded = false) {
    const uint64_t waves = (uint64_t)n_list * (L.window / 64);
    uint64_t blocks = (waves + 3) / 4;
    // 8 workgroups per CU (respond_core: the ctx's max_grid, DSY_PAIR_GRID overrides): the grid-stride then deals
    // each wave 2-3 wave-tasks round-robin; same-box A/B on the headline, 4096 / 2048 / 1280 / 1024 workgroups:
    // 227-229 / 224-226 / 230-233 / 230-234 us
    const uint64_t cap = L.grid_cap ? L.grid_cap : 2048;
    if (blocks > cap) blocks = cap;
    if (blocks == 0) return hipSuccess;
    if (L.pool_deal) blocks = cap / 2 / 4 * 4;  // the resident grid: 4 workgroups per CU (128 VGPRs)
    constexpr bool poolable = H::kind == DSY_MD5 || H::kind == DSY_SHA1 || H::kind == DSY_SHA256;
    if constexpr (poolable) {
        if (pooled) {
            // one workgroup per claim for windows of <= 16 parts (the common 4096-pair window: 1024 claims, 1024
            // workgroups), more for the big windows of a few long claims
            const uint32_t parts = (uint32_t)std::max<uint64_t>(1, L.window / (16 * kPoolPart));
            if (L.pool_scan)
                hipLaunchKernelGGL(k_pool_scan, dim3(kPoolBins / 64), dim3(1024), 0, L.stream, L, list, n_list, fam);
            hipLaunchKernelGGL(k_pool_scatter, dim3(n_list, parts), dim3(256), 0, L.stream, L, list, fam);
        }
    } else {
        pooled = false;
    }
    // MD5 and SHA-1 stage their 64-byte blocks through LDS with DMA (8 keys x 128 contiguous bytes per wave
    // instruction, single LDS buffer, next stage in flight while the current one is compressed from registers:
    // tools/hashbench, profiles/hashbench_r1_dmareg.txt); SHA-2 is compute-bound enough that direct loads match it
    constexpr bool dma = H::kind == DSY_MD5 || H::kind == DSY_SHA1;
    if constexpr (dma) {
        // (the line-staged pieces address the line copy in 16-byte units from a 32-bit index: under 64 GiB)
        // (and every packet short enough for the pieces' 16-bit limits: kLinePathMaxLen)
        if (!long_prefix && !((L.direct_kinds >> H::kind) & 1u) && L.st.lines_bytes < (1ull << 36) &&
            L.st.max_len <= kLinePathMaxLen) {
            const size_t lds = 4 * DmaGeometry<2, 1>::kWaveBytes;
            // (padded: every listed claim has a 1-byte prefix)
            auto kern = pooled ? (padded ? k_pair_test<H, CHUNK, true, 0, true, true> : k_pair_test<H, CHUNK, true, 0, true>)
                               : padded ? k_pair_test<H, CHUNK, true, 0, false, true> : k_pair_test<H, CHUNK, true>;
            if constexpr (CHUNK == 2) {  // (respond_core pools no family while a diagnostic build is asked for)
                if (L.diag == 1) kern = padded ? k_pair_test<H, CHUNK, true, 1, false, true> : k_pair_test<H, CHUNK, true, 1>;
                if (L.diag == 2) kern = padded ? k_pair_test<H, CHUNK, true, 2, false, true> : k_pair_test<H, CHUNK, true, 2>;
            }
            launch_timed(kern, dim3((uint32_t)blocks), dim3(256), lds, L.stream, L.ev_start, L.ev_stop, L, list, n_list,
                         fam);
            return hipGetLastError();
        }
    }
    auto kern = k_pair_test<H, CHUNK, false>;
    if constexpr (poolable)
        if (pooled) kern = k_pair_test<H, CHUNK, false, 0, true>;
    launch_timed(kern, dim3((uint32_t)blocks), dim3(256), 4 * kPairRedBytes, L.stream, L.ev_start, L.ev_stop, L, list,
                 n_list, fam);
    return hipGetLastError();
}

template <class H>
static hipError_t pair_test_chunk(const RespondLaunch& L, uint32_t chunk, bool lp, const uint32_t* list, uint32_t n,
                                  bool pooled, uint32_t fam, bool padded) {
    switch (chunk) {
        case 2: return pair_test_family<H, 2>(L, lp, list, n, pooled, fam, padded);
        case 4: return pair_test_family<H, 4>(L, lp, list, n, pooled, fam, padded);
        default: return pair_test_family<H, 8>(L, lp, list, n, pooled, fam, padded);
    }
}

static hipError_t pair_test_kind(const RespondLaunch& L, int kind, uint32_t chunk, bool long_prefix, const uint32_t* list,
                                 uint32_t n, bool pooled, uint32_t fam, bool padded) {
    switch (kind) {
        case DSY_MD5: return pair_test_chunk<Md5>(L, chunk, long_prefix, list, n, pooled, fam, padded);
        case DSY_SHA1:
            return chunk == 2 ? pair_test_family<Sha1, 2>(L, long_prefix, list, n, pooled, fam, padded)
                              : pair_test_family<Sha1, 4>(L, long_prefix, list, n, pooled, fam, padded);
        case DSY_SHA256: return pair_test_chunk<Sha256>(L, chunk, long_prefix, list, n, pooled, fam, false);
        case DSY_SHA384: return pair_test_chunk<Sha384>(L, chunk, long_prefix, list, n, false, fam, false);
        default: return pair_test_chunk<Sha512>(L, chunk, long_prefix, list, n, false, fam, false);
    }
}

hipError_t launch_pair_test_list(const RespondLaunch& L, int kind, uint32_t chunk, bool long_prefix, bool padded,
                                 const uint32_t* list, uint32_t n) {
    return pair_test_kind(L, kind, chunk, long_prefix, list, n, false, 0, padded && !long_prefix);
}

hipError_t launch_pair_test_pooled(const RespondLaunch& L, int kind, uint32_t chunk, bool long_prefix, bool padded,
                                   uint32_t fam, const uint32_t* list, uint32_t n) {
    return pair_test_kind(L, kind, chunk, long_prefix, list, n, true, fam, padded && !long_prefix);
}

// ----------------------------------------------------------------------------------------- k_compact
__device__ __forceinline__ int64_t wave_inclusive_scan(int64_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int64_t o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}

// Fold the kCntSpread counter copies into the host-mapped status (wave 0 of the calling workgroup).  Called by
// the pack kernels, which run after the window's k_compact: the kernel boundary orders the counters' atomics.
__device__ __forceinline__ void fold_status(const RespondLaunch& L) {
    if (threadIdx.x >= 64) return;
    const uint32_t lane = threadIdx.x;
    static_assert(kCntSpread == 64, "one lane per counter copy");
#pragma unroll
    for (int k = 0; k < kCntN; ++k) {
        uint64_t v = L.counters[lane * kCntN + k];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
        if (lane == 0) L.h_status[k] = v;
    }
    if (lane == 0) {  // this window's number (copy 0's spare counter slot), after its totals
        const uint64_t seq = L.counters[kCntSeq] + 1;
        L.counters[kCntSeq] = seq;
        L.h_status[kStatusSeq] = seq;
    }
}

// position of the k-th set bit of w (k < popcount(w))
__device__ __forceinline__ uint32_t select_bit(uint64_t w, uint32_t k) {
    uint32_t pos = 0;
#pragma unroll
    for (int h = 32; h >= 1; h >>= 1) {
        const uint32_t c = __popcll(w & ((1ull << h) - 1));
        if (k >= c) {
            k -= c;
            w >>= h;
            pos += h;
        }
    }
    return pos;
}

// One wave per claim.  The window's missing pairs are the set bits of the claim's miss_mask words (bit t: window
// slot t, i.e. send order); each round loads 256 words (16 K slots), ranks their set bits, and takes the misses in
// batches of 64: lane i fetches the i-th miss's length and row, a prefix sum applies the byte-limit rule of
// community.py:2559-2567 (send while the budget before the packet is positive; the crossing packet is sent).
__global__ void __launch_bounds__(64) k_compact(RespondLaunch L) {
    const uint32_t a_slot = blockIdx.x;
    if (a_slot == 0 && threadIdx.x == 0) L.flags[kFlagChunks] = 0;  // every k_pair_test of this window has run
    const uint32_t r = L.act[a_slot];
    ReqState* S = &L.state[r];
    if (S->done) {
        if (threadIdx.x == 0) {
            L.act_done[a_slot] = 1;
            L.emitted_n[r] = S->emitted;
        }
        return;
    }
    const uint64_t W = L.window;
    const uint64_t n = S->n_window;
    const uint32_t lane = threadIdx.x;
    uint64_t emitted = S->emitted;
    int64_t spent = S->spent;
    uint32_t done = 0, overflow = S->overflow;
    uint64_t useful = n;  // pairs the reference hashes in this window: up to the packet that spends the budget
    const int64_t limit = L.byte_limit;
    const uint64_t cap = S->cap, out_base = S->out_base;
    const uint64_t* mask_w = L.miss_mask + (uint64_t)a_slot * (W / 64);
    const uint32_t* len_w = L.pair_len + (uint64_t)a_slot * W;
    const uint64_t* row_w = L.pair_row + (uint64_t)a_slot * W;
    const bool bulk = S->commit;
    const Plan bp = bulk ? L.plans[(uint64_t)r * L.J + S->win_meta] : Plan{};
    const uint64_t nw = (n + 63) / 64;
    constexpr uint32_t kPer = 4;  // words per lane per round
    for (uint64_t wb = 0; wb < nw && !done; wb += 64 * kPer) {
        uint64_t w[kPer];
        uint32_t c[kPer], cnt = 0;
#pragma unroll
        for (uint32_t u = 0; u < kPer; ++u) {
            const uint64_t x = wb + kPer * lane + u;
            w[u] = x < nw ? mask_w[x] : 0ull;
        }
#pragma unroll
        for (uint32_t u = 0; u < kPer; ++u) {
            c[u] = __popcll(w[u]);
            cnt += c[u];
        }
        uint32_t incl = cnt;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(incl, d, 64);
            if ((int)lane >= d) incl += o;
        }
        const uint32_t pos = incl - cnt;                  // misses before this lane's words
        const uint32_t total = __shfl(incl, 63, 64);      // misses in this round
        for (uint32_t kb = 0; kb < total && !done; kb += 64) {
            const uint32_t k = kb + lane;
            const bool miss = k < total;
            // owner lane: the last lane whose first miss index is <= k (binary search over the monotone pos)
            uint32_t lo = 0;
#pragma unroll
            for (int step = 32; step >= 1; step >>= 1) {
                const uint32_t cand = lo + step;
                const uint32_t pc = (uint32_t)__shfl((int)pos, (int)min(cand, 63u), 64);
                if (cand < 64 && pc <= k) lo = cand;
            }
            uint32_t kk = k - (uint32_t)__shfl((int)pos, (int)lo, 64);
            uint64_t t = 0;
            {
                uint64_t ww[kPer];
                uint32_t cc[kPer];
#pragma unroll
                for (uint32_t u = 0; u < kPer; ++u) {
                    ww[u] = __shfl(w[u], (int)lo, 64);
                    cc[u] = (uint32_t)__shfl((int)c[u], (int)lo, 64);
                }
                uint32_t u_sel = 0;
                uint64_t wsel = ww[0];
#pragma unroll
                for (uint32_t u = 0; u < kPer - 1; ++u) {
                    if (u_sel == u && kk >= cc[u]) {
                        kk -= cc[u];
                        u_sel = u + 1;
                        wsel = ww[u + 1];
                    }
                }
                t = (wb + kPer * lo + u_sel) * 64 + (miss ? select_bit(wsel, kk) : 0u);
            }
            int64_t len = 0;
            uint64_t row = 0;
            if (miss) {
                if (bulk) {  // a split window: the row is arithmetic (fill_bulk_part wrote no pair arrays)
                    row = bulk_row(L, bp, S->win_cand, t);
                    len = (int64_t)L.st.rec[row].len;
                } else {
                    len = (int64_t)len_w[t];
                    row = row_w[t];
                }
            }
            int64_t inc_sum = len;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int64_t o = __shfl_up(inc_sum, d, 64);
                if ((int)lane >= d) inc_sum += o;
            }
            const int64_t excl = inc_sum - len;
            // send while the budget before this packet is positive; the first packet is always sent
            const bool inc = miss && ((emitted + lane == 0) || (spent + excl < limit));
            const uint64_t imask = __ballot(inc);
            const uint32_t nin = __popcll(imask);
            if (inc) {
                const uint64_t slot = emitted + lane;
                if (slot < cap) L.out[out_base + slot] = row;
                else overflow = 1;
            }
            int64_t sum_in = 0;
            int last = -1;
            if (nin) {
                last = 63 - __builtin_clzll(imask);
                sum_in = __shfl(inc_sum, last, 64);
            }
            emitted += nin;
            spent += sum_in;
            if (emitted > 0 && spent >= limit) {
                done = 1;
                useful = (uint64_t)__shfl((long long)t, last, 64) + 1;
            }
        }
    }
    overflow = __any(overflow) ? 1u : 0u;
    if (S->commit || S->sort_later) {  // a split window or sort: its sort state cleared
        uint32_t* gh = L.bulk_hist + (uint64_t)a_slot * kSortBins;
        uint32_t* gc = L.bulk_cur + (uint64_t)a_slot * kSortBins;
        for (uint32_t i = lane; i < kSortBins; i += 64) gh[i] = gc[i] = 0;
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {
            if (S->commit) S->cand = S->cand_next;  // the split window's cursor (k_fill's parts read the old one)
            S->commit = 0;
            S->sort_later = 0;
        }
    }
    if (lane == 0) {
        S->win_meta = S->meta;  // the next window's start (after a split window's commit above)
        S->win_cand = S->cand;
        S->win_sub = S->sub;
        S->emitted = emitted;
        L.emitted_n[r] = emitted;
        S->spent = spent;
        S->overflow = overflow;
        if (overflow) L.h_status[kStatusOverflow] = 1;  // host-mapped: read after the window's sync
        if (done || S->exhausted) S->done = 1;
        L.act_done[a_slot] = (uint8_t)S->done;
        atomicAdd(counter(L.counters, kCntPairs), (unsigned long long)n);
        atomicAdd(counter(L.counters, kCntUseful), (unsigned long long)useful);
    }
}

// -------------------------------------------------------------------------------------------- k_pack
__global__ void __launch_bounds__(1024) k_scan_counts(RespondLaunch L, uint64_t* packed_offsets) {
    // single workgroup: exclusive scan of state[r].emitted over R claims
    __shared__ uint64_t part[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (L.R + 1023) / 1024;
    uint64_t sum = 0;
    for (uint32_t i = 0; i < per; ++i) {
        const uint32_t r = t * per + i;
        if (r < L.R) sum += L.state[r].emitted;
    }
    part[t] = sum;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const uint64_t add = t >= (uint32_t)d ? part[t - d] : 0;
        __syncthreads();
        part[t] += add;
        __syncthreads();
    }
    uint64_t run = part[t] - sum;
    for (uint32_t i = 0; i < per; ++i) {
        const uint32_t r = t * per + i;
        if (r < L.R) {
            packed_offsets[r] = run;
            run += L.state[r].emitted;
        }
    }
    if (t == 1023) packed_offsets[L.R] = part[1023];
    fold_status(L);
}

__global__ void __launch_bounds__(256) k_copy_out(RespondLaunch L, const uint64_t* packed_offsets, uint64_t* packed) {
    const uint32_t r = blockIdx.x;
    const ReqState& S = L.state[r];
    const uint64_t n = S.emitted < S.cap ? S.emitted : S.cap;
    if (packed_offsets[r] + n > L.packed_cap) {
        if (threadIdx.x == 0) guard_trip(L.h_status, kGuardPack);
        return;
    }
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) packed[packed_offsets[r] + i] = L.out[S.out_base + i];
}

// one workgroup per claim: its output offset is the sum of the counts before it (read from the compact emitted_n
// array: R * 8 bytes per workgroup at most), then its rows are copied
__global__ void __launch_bounds__(256) k_pack_fused(RespondLaunch L, uint64_t* packed_offsets, uint64_t* packed) {
    __shared__ uint64_t red[4];
    const uint32_t r = blockIdx.x;
    uint64_t s = 0;
    for (uint32_t i = threadIdx.x; i < r; i += 256) s += L.emitted_n[i];
    const uint64_t off = block_sum_256(s, red);
    const ReqState& S = L.state[r];
    const uint64_t n = S.emitted < S.cap ? S.emitted : S.cap;
    const bool fits = off + n <= L.packed_cap;  // (an overflowed claim's emitted exceeds its cap: k_compact flags it)
    if (!fits && threadIdx.x == 0) guard_trip(L.h_status, kGuardPack);
    if (fits)
        for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) packed[off + i] = L.out[S.out_base + i];
    if (threadIdx.x == 0) {
        packed_offsets[r] = off;
        if (r + 1 == L.R) packed_offsets[L.R] = off + S.emitted;
    }
    if (r == 0) fold_status(L);
}

// one wave per row: bytes of the packet to its line-aligned place (coalesced 64-byte stretches), then the padded
// message's terminator after it (the line copy is zeroed: the padding's zeros are there already; line_bytes_for)
__global__ void __launch_bounds__(256) k_store_lines(const uint8_t* __restrict__ blob, const uint64_t* __restrict__ offsets,
                                                     const RowRec* __restrict__ rec, uint64_t n, uint8_t* __restrict__ lines) {
    const uint64_t row = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    if (row >= n) return;
    const uint8_t* src = blob + offsets[row];
    uint8_t* dst = lines + rec[row].off;
    const uint32_t len = rec[row].len;
    for (uint32_t k = lane; k < len; k += 64) dst[k] = src[k];
    if (lane == 0) dst[len] = 0x80;
}

hipError_t launch_store_lines(const uint8_t* blob, const uint64_t* offsets, const RowRec* rec, uint64_t n,
                              uint8_t* lines, hipStream_t stream) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_store_lines, dim3((uint32_t)((n * 64 + 255) / 256)), dim3(256), 0, stream, blob, offsets, rec,
                       n, lines);
    return hipGetLastError();
}

hipError_t launch_setup(const RespondLaunch& L, const void* h_src, void* d_dst, size_t in_bytes, void* d_zero,
                        size_t zero_bytes, uint64_t per_claim_cap) {
    const uint32_t in_words = (uint32_t)(in_bytes / 16), zero_words = (uint32_t)(zero_bytes / 16);
    // one 16-byte word per lane where possible: the host reads are PCIe round trips
    const uint64_t lanes = std::max<uint64_t>(std::max<uint64_t>((uint64_t)L.R * L.J, in_words), 1);
    const uint32_t blocks = (uint32_t)((lanes + 255) / 256);
    hipLaunchKernelGGL(k_setup, dim3(blocks), dim3(256), 0, L.stream, L, (const uint4*)h_src, (uint4*)d_dst,
                       in_words, (uint4*)d_zero, zero_words, per_claim_cap);
    return hipGetLastError();
}

hipError_t launch_fill(const RespondLaunch& L) {
    if (!L.n_act) return hipSuccess;
    // windows of >= 2 bulk chunks may split over workgroups (k_fill's parts, then k_fill_sort)
    const uint32_t parts = L.window >= 2 * kBulkChunk ? (uint32_t)((L.window + kBulkChunk - 1) / kBulkChunk) : 1u;
    hipLaunchKernelGGL(k_fill, dim3(L.n_act, parts), dim3(kFillThreads), 0, L.stream, L);
    if (parts > 1) hipLaunchKernelGGL(k_fill_sort, dim3(L.n_act, parts), dim3(kFillThreads), 0, L.stream, L);
    return hipGetLastError();
}

hipError_t launch_fill_first(const RespondLaunch& L, const void* h_src, void* d_dst, size_t in_bytes, void* d_counters,
                             size_t counter_bytes, uint64_t per_claim_cap, const uint32_t* h_act) {
    if (!L.n_act) return hipSuccess;
    hipLaunchKernelGGL(k_fill_first, dim3(L.n_act), dim3(kFillThreads), 0, L.stream, L, (const uint4*)h_src,
                       (uint4*)d_dst, (uint32_t)(in_bytes / 16), (uint4*)d_counters, (uint32_t)(counter_bytes / 16),
                       per_claim_cap, h_act);
    return hipGetLastError();
}

// Diagnostics, run only after a window whose k_pair_test tripped kGuardTask: every listed claim's task records
// [0, n_window) checked as k_pair_test checks them.  out[0]: bad records; out[1..8]: one of them (a_slot, claim, index,
// n_window, off, len, slot, W); out[9]: claims with a bad record.
__global__ void __launch_bounds__(256) k_task_audit(RespondLaunch L, unsigned long long* __restrict__ out) {
    __shared__ uint32_t bad_here;
    const uint32_t a_slot = blockIdx.x;
    const uint32_t r = L.act[a_slot];
    const uint64_t n = L.state[r].n_window, W = L.window;
    if (threadIdx.x == 0) bad_here = 0;
    __syncthreads();
    for (uint64_t i = threadIdx.x; i < n && i < W; i += blockDim.x) {
        const PairTask tk = L.task[(uint64_t)a_slot * W + i];
        if (!packet_in_lines(tk.off, tk.len, L.st.lines_bytes) || tk.slot >= n) {
            atomicAdd(&bad_here, 1u);
            if (atomicAdd(&out[0], 1ull) == 0) {
                out[1] = a_slot;
                out[2] = r;
                out[3] = i;
                out[4] = n;
                out[5] = tk.off;
                out[6] = tk.len;
                out[7] = tk.slot;
                out[8] = W;
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0 && bad_here) atomicAdd(&out[9], 1ull);
}

hipError_t launch_task_audit(const RespondLaunch& L, unsigned long long* out) {
    if (!L.n_act) return hipSuccess;
    hipLaunchKernelGGL(k_task_audit, dim3(L.n_act), dim3(256), 0, L.stream, L, out);
    return hipGetLastError();
}

hipError_t launch_compact(const RespondLaunch& L) {
    if (!L.n_act) return hipSuccess;
    hipLaunchKernelGGL(k_compact, dim3(L.n_act), dim3(64), 0, L.stream, L);
    return hipGetLastError();
}

hipError_t launch_pack(const RespondLaunch& L, uint64_t* packed, uint64_t* packed_offsets, uint64_t*, hipEvent_t done) {
    // done: recorded by the last kernel's own dispatch (an event record between two dispatches leaves a ~6 us gap on
    // the queue, in front of the next batch's selection)
    if (L.R && L.R <= kPackFusedMax) {
        if (done) hipExtLaunchKernelGGL(k_pack_fused, dim3(L.R), dim3(256), 0, L.stream, nullptr, done, 0, L,
                                        packed_offsets, packed);
        else hipLaunchKernelGGL(k_pack_fused, dim3(L.R), dim3(256), 0, L.stream, L, packed_offsets, packed);
        return hipGetLastError();
    }
    if (!L.R) {
        if (done) hipExtLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, L.stream, nullptr, done, 0, L,
                                        packed_offsets);
        else hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, L.stream, L, packed_offsets);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, L.stream, L, packed_offsets);
    if (done) hipExtLaunchKernelGGL(k_copy_out, dim3(L.R), dim3(256), 0, L.stream, nullptr, done, 0, L, packed_offsets,
                                    packed);
    else hipLaunchKernelGGL(k_copy_out, dim3(L.R), dim3(256), 0, L.stream, L, packed_offsets, packed);
    return hipGetLastError();
}

}  // namespace dsy

// Requester-side ingest into the packed store: `Dispersy._store` INSERTs every received sync
// packet into the `sync` table (dispersy.py:1475-1612); the responder serves it from then on through the
// `sync_meta_message_undone_global_time_index` (dispersydatabase.py:63).  Here the new rows take the next row
// positions and the store's live index -- live_gt/live_row in (meta_message, global_time, rowid) order -- is merged
// on the device:
//   k_ingest_rank       one lane per new row (in index order): upper bound of its global time in its meta's live
//                       segment = how many old live rows precede it (equal global times: the old row first, it has
//                       the smaller rowid).
//   k_ingest_merge_old  one lane per old live row: shift by the number of new rows ranked at or before it.  Each
//                       workgroup bounds its tile's shifts with two searches, so most lanes search an empty range.
//   k_ingest_merge_new  one lane per new row: its place is rank + index.
// Every output slot is written exactly once; reads and writes of the old index stream (16 B in, 16 B out per row).
#include "dsy_kernels.h"

#include <algorithm>
#include <rocprim/device/device_radix_sort.hpp>

namespace dsy {

static constexpr uint32_t kIngestThreads = 256;
static constexpr uint32_t kIngestPerThread = 4;
static constexpr uint64_t kIngestTile = (uint64_t)kIngestThreads * kIngestPerThread;

__global__ void __launch_bounds__(kIngestThreads) k_ingest_rank(const uint64_t* __restrict__ live_gt,
                                                                 const uint64_t* __restrict__ live_row,
                                                                 const IngestRow* __restrict__ rows, uint64_t a,
                                                                 uint64_t* __restrict__ rank,
                                                                 unsigned int* __restrict__ present) {
    const uint64_t j = (uint64_t)blockIdx.x * kIngestThreads + threadIdx.x;
    if (j >= a) return;
    const IngestRow r = rows[j];
    // the first index entry of the segment at or after (gt, row) in (global_time, row) order: for an appended row
    // (a row position past every stored one) the upper bound of its global time, for a redone row its place among
    // the rows of equal global time
    uint64_t lo = r.seg_a, hi = r.seg_b;
    while (lo < hi) {
        const uint64_t mid = lo + ((hi - lo) >> 1);
        const uint64_t g = live_gt[mid], w = live_row ? live_row[mid] : mid;
        if (g < r.gt || (g == r.gt && w < r.row)) lo = mid + 1; else hi = mid;
    }
    rank[j] = lo;
    if (present && lo < r.seg_b && live_gt[lo] == r.gt && (live_row ? live_row[lo] : lo) == r.row) atomicOr(present, 1u);
}

// number of j in [lo, hi) with rank[j] <= i (rank is non-decreasing)
__device__ __forceinline__ uint64_t ranks_at_or_before(const uint64_t* __restrict__ rank, uint64_t lo, uint64_t hi,
                                                       uint64_t i) {
    while (lo < hi) {
        const uint64_t mid = lo + ((hi - lo) >> 1);
        if (rank[mid] <= i) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(kIngestThreads) k_ingest_merge_old(const uint64_t* __restrict__ live_gt,
                                                                      const uint64_t* __restrict__ live_row,
                                                                      uint64_t n_live, const uint64_t* __restrict__ rank,
                                                                      uint64_t a, uint64_t* __restrict__ out_gt,
                                                                      uint64_t* __restrict__ out_row) {
    __shared__ uint64_t bound[2];
    for (uint64_t t0 = (uint64_t)blockIdx.x * kIngestTile; t0 < n_live; t0 += (uint64_t)gridDim.x * kIngestTile) {
        const uint64_t t1 = t0 + kIngestTile < n_live ? t0 + kIngestTile : n_live;
        __syncthreads();  // the previous tile's bounds are consumed
        if (threadIdx.x < 2) bound[threadIdx.x] = ranks_at_or_before(rank, 0, a, threadIdx.x ? t1 - 1 : t0);
        __syncthreads();
        const uint64_t s0 = bound[0], s1 = bound[1];
#pragma unroll
        for (uint32_t u = 0; u < kIngestPerThread; ++u) {
            const uint64_t i = t0 + (uint64_t)u * kIngestThreads + threadIdx.x;
            if (i < t1) {
                const uint64_t shift = s0 == s1 ? s0 : ranks_at_or_before(rank, s0, s1, i);
                out_gt[i + shift] = live_gt[i];
                out_row[i + shift] = live_row ? live_row[i] : i;
            }
        }
    }
}

__global__ void __launch_bounds__(kIngestThreads) k_ingest_merge_new(const IngestRow* __restrict__ rows, uint64_t a,
                                                                      const uint64_t* __restrict__ rank,
                                                                      uint64_t* __restrict__ out_gt,
                                                                      uint64_t* __restrict__ out_row) {
    const uint64_t j = (uint64_t)blockIdx.x * kIngestThreads + threadIdx.x;
    if (j >= a) return;
    const IngestRow r = rows[j];
    out_gt[rank[j] + j] = r.gt;
    out_row[rank[j] + j] = r.row;
}

// DELETE FROM sync WHERE meta_message = ? AND global_time <= ? (community.py:1092-1096, GlobalTimePruning): the rows
// form a prefix [a, a + k) of the meta's live segment.  k_prune_count finds k (one upper bound by one lane);
// k_live_cut copies the index without that range (16 B in, 16 B out per indexed row).
__global__ void k_prune_count(const uint64_t* __restrict__ live_gt, uint64_t a, uint64_t b, uint64_t max_gt,
                              uint64_t* __restrict__ out_k) {
    if (threadIdx.x) return;
    uint64_t lo = a, hi = b;
    while (lo < hi) {
        const uint64_t mid = lo + ((hi - lo) >> 1);
        if (live_gt[mid] <= max_gt) lo = mid + 1; else hi = mid;
    }
    *out_k = lo - a;
}

__global__ void __launch_bounds__(kIngestThreads) k_live_cut(const uint64_t* __restrict__ live_gt,
                                                              const uint64_t* __restrict__ live_row, uint64_t n_out,
                                                              uint64_t a, uint64_t k, uint64_t* __restrict__ out_gt,
                                                              uint64_t* __restrict__ out_row) {
    for (uint64_t i = (uint64_t)blockIdx.x * kIngestThreads + threadIdx.x; i < n_out;
         i += (uint64_t)gridDim.x * kIngestThreads) {
        const uint64_t src = i < a ? i : i + k;
        out_gt[i] = live_gt[src];
        out_row[i] = live_row ? live_row[src] : src;
    }
}

hipError_t launch_prune_count(const uint64_t* live_gt, uint64_t a, uint64_t b, uint64_t max_gt, uint64_t* out_k,
                              hipStream_t stream) {
    hipLaunchKernelGGL(k_prune_count, dim3(1), dim3(64), 0, stream, live_gt, a, b, max_gt, out_k);
    return hipGetLastError();
}

hipError_t launch_live_cut(const uint64_t* live_gt, const uint64_t* live_row, uint64_t n_out, uint64_t a, uint64_t k,
                           uint64_t* out_gt, uint64_t* out_row, uint32_t max_grid, hipStream_t stream) {
    if (!n_out) return hipSuccess;
    uint64_t g = (n_out + kIngestThreads - 1) / kIngestThreads;
    if (g > (uint64_t)max_grid * 4) g = (uint64_t)max_grid * 4;
    hipLaunchKernelGGL(k_live_cut, dim3((uint32_t)g), dim3(kIngestThreads), 0, stream, live_gt, live_row, n_out, a, k,
                       out_gt, out_row);
    return hipGetLastError();
}

// ---- pending entries (rows appended since the index was last read) in index order, on the device: two stable radix
// sorts of the entry numbers j, by global time and then by the meta's rank among the pending metas, leave equal
// (meta, global_time) entries in j order = row order (row = base + j).  The host sorted them before (~6 ms for
// 110 k entries on one core, the whole cost of the deferred merge).
__global__ void __launch_bounds__(kIngestThreads) k_pend_key_gt(const uint64_t* __restrict__ gt, uint64_t P,
                                                                 uint64_t glo, uint64_t* __restrict__ key,
                                                                 uint32_t* __restrict__ idx) {
    const uint64_t j = (uint64_t)blockIdx.x * kIngestThreads + threadIdx.x;
    if (j >= P) return;
    key[j] = gt[j] - glo;
    idx[j] = (uint32_t)j;
}

// rank of a meta in the sorted table of the pending metas (it is there: the table holds every pending meta)
__device__ __forceinline__ uint32_t meta_rank(const uint32_t* __restrict__ metas, uint32_t nm, uint32_t m) {
    uint32_t lo = 0, hi = nm;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (metas[mid] < m) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(kIngestThreads) k_pend_key_meta(const uint32_t* __restrict__ meta, uint64_t P,
                                                                   const uint32_t* __restrict__ order,
                                                                   const uint32_t* __restrict__ metas, uint32_t nm,
                                                                   uint64_t* __restrict__ key) {
    const uint64_t t = (uint64_t)blockIdx.x * kIngestThreads + threadIdx.x;
    if (t >= P) return;
    key[t] = meta_rank(metas, nm, meta[order[t]]);
}

// gap_before (optional): slack entries placed before meta rank r's rows (after each smaller meta's own rows)
__global__ void __launch_bounds__(kIngestThreads) k_pend_rows(const uint32_t* __restrict__ meta,
                                                               const uint64_t* __restrict__ gt, uint64_t P,
                                                               const uint32_t* __restrict__ order,
                                                               const uint32_t* __restrict__ metas, uint32_t nm,
                                                               const uint64_t* __restrict__ segs,
                                                               const uint64_t* __restrict__ gap_before, uint64_t base,
                                                               IngestRow* __restrict__ out) {
    const uint64_t t = (uint64_t)blockIdx.x * kIngestThreads + threadIdx.x;
    if (t >= P) return;
    const uint32_t j = order[t];
    const uint32_t r = meta_rank(metas, nm, meta[j]);
    out[t + (gap_before ? gap_before[r] : 0)] = IngestRow{gt[j], segs[2 * r], segs[2 * r + 1], base + j};
}

// slack entries of one meta's region: ranked at the region's end (rank = seg_a = seg_b = end), row kGapRow
__global__ void __launch_bounds__(kIngestThreads) k_gap_rows(IngestRow* __restrict__ out, uint64_t k, uint64_t end) {
    const uint64_t t = (uint64_t)blockIdx.x * kIngestThreads + threadIdx.x;
    if (t < k) out[t] = IngestRow{0, end, end, kGapRow};
}

// per meta r with pending entries: the position of its first (smallest) new entry in its live segment -- where the
// in-place merge of the segment's tail starts (starts[r]: its first row in the ordered pending rows)
__global__ void k_first_rank(const uint64_t* __restrict__ live_gt, const uint64_t* __restrict__ live_row,
                             const IngestRow* __restrict__ rows, const uint64_t* __restrict__ starts,
                             const uint64_t* __restrict__ counts, uint32_t nm, uint64_t* __restrict__ out) {
    const uint32_t r = blockIdx.x * 64 + threadIdx.x;
    if (r >= nm) return;
    if (!counts[r]) { out[r] = 0; return; }
    const IngestRow q = rows[starts[r]];
    uint64_t lo = q.seg_a, hi = q.seg_b;
    while (lo < hi) {
        const uint64_t mid = lo + ((hi - lo) >> 1);
        const uint64_t g = live_gt[mid], w = live_row[mid];
        if (g < q.gt || (g == q.gt && w < q.row)) lo = mid + 1; else hi = mid;
    }
    out[r] = lo;
}

// rebase k ordered rows onto a segment [sa, sb) of a copied tail
__global__ void __launch_bounds__(kIngestThreads) k_rows_seg(IngestRow* __restrict__ rows, uint64_t k, uint64_t sa,
                                                              uint64_t sb) {
    const uint64_t t = (uint64_t)blockIdx.x * kIngestThreads + threadIdx.x;
    if (t < k) {
        rows[t].seg_a = sa;
        rows[t].seg_b = sb;
    }
}

static int bit_width(uint64_t x) {
    int b = 0;
    while (b < 64 && (x >> b)) ++b;
    return b;
}

// scratch: keys 2 x P u64, order 2 x P u32, then the radix sort's temporary storage
size_t pend_order_scratch(uint64_t P) {
    size_t tmp = 0;
    rocprim::radix_sort_pairs(nullptr, tmp, (const uint64_t*)nullptr, (uint64_t*)nullptr, (const uint32_t*)nullptr,
                              (uint32_t*)nullptr, (size_t)P, 0u, 64u, nullptr);
    return (size_t)P * 24 + 256 + tmp;
}

hipError_t launch_pend_order(const uint32_t* meta, const uint64_t* gt, uint64_t P, uint64_t glo, uint64_t ghi,
                             const uint32_t* metas, const uint64_t* segs, const uint64_t* gap_before, uint32_t nm,
                             uint64_t base, void* scratch, size_t scratch_bytes, IngestRow* out, hipStream_t stream) {
    if (!P) return hipSuccess;
    uint64_t* key_a = (uint64_t*)scratch;
    uint64_t* key_b = key_a + P;
    uint32_t* ord_a = (uint32_t*)(key_b + P);
    uint32_t* ord_b = ord_a + P;
    void* tmp = (uint8_t*)scratch + (((size_t)P * 24 + 255) & ~(size_t)255);
    size_t tmp_bytes = scratch_bytes - (((size_t)P * 24 + 255) & ~(size_t)255);
    const uint32_t g = (uint32_t)((P + kIngestThreads - 1) / kIngestThreads);
    hipLaunchKernelGGL(k_pend_key_gt, dim3(g), dim3(kIngestThreads), 0, stream, gt, P, glo, key_a, ord_a);
    hipError_t e = rocprim::radix_sort_pairs(tmp, tmp_bytes, key_a, key_b, ord_a, ord_b, (size_t)P, 0u,
                                             (unsigned)std::max(1, bit_width(ghi - glo)), stream);
    if (e != hipSuccess) return e;
    const uint32_t* order = ord_b;
    if (nm > 1) {
        hipLaunchKernelGGL(k_pend_key_meta, dim3(g), dim3(kIngestThreads), 0, stream, meta, P, ord_b, metas, nm,
                           key_a);
        e = rocprim::radix_sort_pairs(tmp, tmp_bytes, key_a, key_b, ord_b, ord_a, (size_t)P, 0u,
                                      (unsigned)bit_width(nm - 1), stream);
        if (e != hipSuccess) return e;
        order = ord_a;
    }
    hipLaunchKernelGGL(k_pend_rows, dim3(g), dim3(kIngestThreads), 0, stream, meta, gt, P, order, metas, nm, segs,
                       gap_before, base, out);
    return hipGetLastError();
}

hipError_t launch_gap_rows(IngestRow* out, uint64_t k, uint64_t end, hipStream_t stream) {
    if (!k) return hipSuccess;
    hipLaunchKernelGGL(k_gap_rows, dim3((uint32_t)((k + kIngestThreads - 1) / kIngestThreads)), dim3(kIngestThreads), 0,
                       stream, out, k, end);
    return hipGetLastError();
}

hipError_t launch_first_rank(const uint64_t* live_gt, const uint64_t* live_row, const IngestRow* rows,
                             const uint64_t* starts, const uint64_t* counts, uint32_t nm, uint64_t* out,
                             hipStream_t stream) {
    if (!nm) return hipSuccess;
    hipLaunchKernelGGL(k_first_rank, dim3((nm + 63) / 64), dim3(64), 0, stream, live_gt, live_row, rows, starts, counts,
                       nm, out);
    return hipGetLastError();
}

hipError_t launch_rows_seg(IngestRow* rows, uint64_t k, uint64_t sa, uint64_t sb, hipStream_t stream) {
    if (!k) return hipSuccess;
    hipLaunchKernelGGL(k_rows_seg, dim3((uint32_t)((k + kIngestThreads - 1) / kIngestThreads)), dim3(kIngestThreads), 0,
                       stream, rows, k, sa, sb);
    return hipGetLastError();
}

hipError_t launch_ingest_merge(const uint64_t* live_gt, const uint64_t* live_row, uint64_t n_live,
                               const IngestRow* rows, uint64_t a, uint64_t* rank, uint64_t* out_gt, uint64_t* out_row,
                               unsigned int* present, uint32_t max_grid, hipStream_t stream) {
    if (!a) return hipSuccess;
    const uint32_t gnew = (uint32_t)((a + kIngestThreads - 1) / kIngestThreads);
    hipLaunchKernelGGL(k_ingest_rank, dim3(gnew), dim3(kIngestThreads), 0, stream, live_gt, live_row, rows, a, rank,
                       present);
    if (n_live) {
        uint64_t g = (n_live + kIngestTile - 1) / kIngestTile;
        if (g > (uint64_t)max_grid * 4) g = (uint64_t)max_grid * 4;
        hipLaunchKernelGGL(k_ingest_merge_old, dim3((uint32_t)g), dim3(kIngestThreads), 0, stream, live_gt, live_row,
                           n_live, rank, a, out_gt, out_row);
    }
    hipLaunchKernelGGL(k_ingest_merge_new, dim3(gnew), dim3(kIngestThreads), 0, stream, rows, a, rank, out_gt, out_row);
    return hipGetLastError();
}

// Claim side, modulo strategy (community.py:908-933): the rows of one meta's live segment [a, b) whose
// (global_time + offset) % modulo == 0 -- the SELECTs of :918/:922 over the store's index.  One lane per indexed row
// (8 B of live_gt read, 8 B of live_row for the hits); each wave ranks its hits by ballot and takes one slot range
// with a single atomic; the residue comes from a 64-bit Barrett step (a multiply-high and one correction) instead
// of a software 64-bit division.  The output order is not the index order; the filter the rows go into is an OR,
// so the claim's bytes do not depend on it.
__global__ void __launch_bounds__(kIngestThreads) k_claim_modulo(const uint64_t* __restrict__ live_gt,
                                                                  const uint64_t* __restrict__ live_row, uint64_t a,
                                                                  uint64_t b, uint64_t offset, uint64_t modulo,
                                                                  uint64_t recip, uint64_t* __restrict__ out_rows,
                                                                  uint64_t cap, unsigned long long* __restrict__ count) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t stride = (uint64_t)gridDim.x * kIngestTile;
    // each wave covers kIngestPerThread x 64 consecutive rows per step, all loads issued before the first ballot
    for (uint64_t base = a + (uint64_t)blockIdx.x * kIngestTile + (uint64_t)(threadIdx.x >> 6) * 64 * kIngestPerThread;
         base < b; base += stride) {
        uint64_t x[kIngestPerThread];
#pragma unroll
        for (uint32_t u = 0; u < kIngestPerThread; ++u) {
            const uint64_t i = base + u * 64 + lane;
            x[u] = i < b ? live_gt[i] + offset : 0;  // lanes past the segment are masked below
        }
#pragma unroll
        for (uint32_t u = 0; u < kIngestPerThread; ++u) {
            const uint64_t i = base + u * 64 + lane;
            // x % modulo by Barrett: q = floor(x * recip / 2^64) is floor(x / modulo) or one less
            uint64_t r = x[u] - __umul64hi(x[u], recip) * modulo;
            if (r >= modulo) r -= modulo;
            const bool hit = i < b && r == 0;
            const uint64_t mask = __ballot(hit);
            if (!mask) continue;
            unsigned long long at = 0;
            if (lane == 0) at = atomicAdd(count, (unsigned long long)__popcll(mask));
            at = __shfl(at, 0);
            const uint64_t slot = at + __popcll(mask & ((1ull << lane) - 1));
            if (hit && slot < cap) out_rows[slot] = live_row ? live_row[i] : i;
        }
    }
}

hipError_t launch_claim_modulo(const uint64_t* live_gt, const uint64_t* live_row, uint64_t a, uint64_t b,
                               uint64_t offset, uint64_t modulo, uint64_t* out_rows, uint64_t cap,
                               unsigned long long* count, uint32_t max_grid, hipStream_t stream) {
    if (b <= a) return hipSuccess;
    uint64_t g = (b - a + kIngestTile - 1) / kIngestTile;
    if (g > (uint64_t)max_grid * 4) g = (uint64_t)max_grid * 4;
    const uint64_t recip = ~0ull / modulo;  // floor((2^64 - 1) / modulo): one correction step suffices
    hipLaunchKernelGGL(k_claim_modulo, dim3((uint32_t)g), dim3(kIngestThreads), 0, stream, live_gt, live_row, a, b,
                       offset, modulo, recip, out_rows, cap, count);
    return hipGetLastError();
}

// DELETE FROM sync WHERE id = ? for arbitrary rows (dsy_store_delete: the sequence-number conflict DELETE of
// dispersy.py:1006, LastSyncDistribution's history pruning :1560-1591): a stable compaction of the live index without
// the entries whose row is marked in del_bits.  16 B read + 16 B written per indexed row, two passes over a bit per
// entry (the bitmap is n/8 bytes: L2-resident for small deletes).
__global__ void __launch_bounds__(256) k_mark_rows(const uint64_t* __restrict__ rows, uint64_t k, uint64_t n_rows,
                                                   uint32_t* __restrict__ bits) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < k && rows[i] < n_rows) atomicOr(&bits[rows[i] >> 5], 1u << (rows[i] & 31));
}

__device__ __forceinline__ bool entry_kept(const uint64_t* __restrict__ live_row, const uint32_t* __restrict__ bits,
                                           uint64_t i) {
    const uint64_t r = live_row ? live_row[i] : i;
    return r != kGapRow && !((bits[r >> 5] >> (r & 31)) & 1u);  // slack entries go too
}

// kept entries per tile of kDelTile (256 lanes x 4)
__global__ void __launch_bounds__(256) k_del_count(const uint64_t* __restrict__ live_row, uint64_t n_live,
                                                   const uint32_t* __restrict__ bits, uint64_t* __restrict__ tile_cnt) {
    __shared__ uint32_t part[4];
    const uint64_t t0 = (uint64_t)blockIdx.x * kDelTile;
    uint32_t c = 0;
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) {
        const uint64_t i = t0 + u * 256 + threadIdx.x;
        c += (i < n_live && entry_kept(live_row, bits, i)) ? 1u : 0u;
    }
    for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) tile_cnt[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

// exclusive scan of the tile counts, one workgroup (tile_cnt[tiles] receives the total)
__global__ void __launch_bounds__(1024) k_del_scan(uint64_t* __restrict__ tile_cnt, uint64_t tiles) {
    __shared__ uint64_t sums[1024];
    const uint64_t per = (tiles + 1023) / 1024;
    const uint64_t b0 = threadIdx.x * per, b1 = b0 + per < tiles ? b0 + per : tiles;
    uint64_t s = 0;
    for (uint64_t t = b0; t < b1; ++t) s += tile_cnt[t];
    sums[threadIdx.x] = s;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const uint64_t v = threadIdx.x >= d ? sums[threadIdx.x - d] : 0;
        __syncthreads();
        sums[threadIdx.x] += v;
        __syncthreads();
    }
    uint64_t run = sums[threadIdx.x] - s;
    for (uint64_t t = b0; t < b1; ++t) {
        const uint64_t c = tile_cnt[t];
        tile_cnt[t] = run;
        run += c;
    }
    if (threadIdx.x == 1023) tile_cnt[tiles] = sums[1023];
}

// each tile writes its kept entries at its scanned offset, in order (wave ballots + a 4-wave LDS prefix per pass)
__global__ void __launch_bounds__(256) k_del_scatter(const uint64_t* __restrict__ live_gt,
                                                     const uint64_t* __restrict__ live_row, uint64_t n_live,
                                                     const uint32_t* __restrict__ bits,
                                                     const uint64_t* __restrict__ tile_off, uint64_t* __restrict__ out_gt,
                                                     uint64_t* __restrict__ out_row) {
    __shared__ uint32_t wsum[4];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t t0 = (uint64_t)blockIdx.x * kDelTile;
    uint64_t at = tile_off[blockIdx.x];
    for (uint32_t u = 0; u < 4; ++u) {
        const uint64_t i = t0 + u * 256 + threadIdx.x;
        const bool keep = i < n_live && entry_kept(live_row, bits, i);
        const uint64_t m = __ballot(keep);
        if (lane == 0) wsum[wave] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t before = 0, total = 0;
        for (uint32_t w = 0; w < 4; ++w) {
            before += w < wave ? wsum[w] : 0;
            total += wsum[w];
        }
        if (keep) {
            const uint64_t o = at + before + __popcll(m & ((1ull << lane) - 1));
            out_gt[o] = live_gt[i];
            out_row[o] = live_row ? live_row[i] : i;
        }
        at += total;
        __syncthreads();
    }
}

// old index position -> new one (kept entries before it): the tile's offset plus a count inside the tile
__global__ void k_del_bounds(const uint64_t* __restrict__ live_row, uint64_t n_live, const uint32_t* __restrict__ bits,
                             const uint64_t* __restrict__ tile_off, uint64_t* __restrict__ bounds, uint32_t nb) {
    const uint32_t j = blockIdx.x * 64 + threadIdx.x;
    if (j >= nb) return;
    const uint64_t x = bounds[j];
    const uint64_t t = x / kDelTile;
    uint64_t pos = tile_off[t];
    for (uint64_t i = t * kDelTile; i < x && i < n_live; ++i) pos += entry_kept(live_row, bits, i) ? 1 : 0;
    bounds[j] = pos;
}

hipError_t launch_mark_rows(const uint64_t* rows, uint64_t k, uint64_t n_rows, uint32_t* del_bits, hipStream_t stream) {
    if (!k) return hipSuccess;
    hipLaunchKernelGGL(k_mark_rows, dim3((uint32_t)((k + 255) / 256)), dim3(256), 0, stream, rows, k, n_rows, del_bits);
    return hipGetLastError();
}

hipError_t launch_live_delete(const uint64_t* live_gt, const uint64_t* live_row, uint64_t n_live,
                              const uint32_t* del_bits, uint64_t* tile_tmp, uint64_t* out_gt, uint64_t* out_row,
                              uint64_t* bounds, uint32_t nb, hipStream_t stream) {
    const uint64_t tiles = (n_live + kDelTile - 1) / kDelTile;
    if (tiles) {
        hipLaunchKernelGGL(k_del_count, dim3((uint32_t)tiles), dim3(256), 0, stream, live_row, n_live, del_bits, tile_tmp);
    }
    hipLaunchKernelGGL(k_del_scan, dim3(1), dim3(1024), 0, stream, tile_tmp, tiles);
    if (tiles) {
        hipLaunchKernelGGL(k_del_scatter, dim3((uint32_t)tiles), dim3(256), 0, stream, live_gt, live_row, n_live,
                           del_bits, tile_tmp, out_gt, out_row);
    }
    if (nb) {
        hipLaunchKernelGGL(k_del_bounds, dim3((nb + 63) / 64), dim3(64), 0, stream, live_row, n_live, del_bits, tile_tmp,
                           bounds, nb);
    }
    return hipGetLastError();
}

}  // namespace dsy

namespace dsy {

// ---------------------------------------------------------------------------------------------------------
// Claim side, largest strategy: _select_and_fix (community.py:881-903) on the device.  The reference runs
//   SELECT global_time, packet FROM sync WHERE meta_message IN (..) AND undone = 0 AND global_time > ?
//   ORDER BY global_time ASC LIMIT to_select + 1            (or < ? ... DESC)
// and, when it got to_select + 1 rows, drops the last global time's whole group.  The rows it keeps are therefore
// exactly those strictly between the pivot and the (to_select+1)-th candidate's global time g -- a global-time
// interval, whatever order SQLite gives equal global times -- or every candidate when there are at most to_select.
// One workgroup: per-meta bounds by binary search, then g: with one meta it is an index; with several, every
// candidate's rank across the metas (binary searches over the others' first to_select+1 candidates, held in LDS
// when they fit) finds the one of rank to_select+1.
static constexpr uint32_t kSelThreads = 1024;

__device__ __forceinline__ uint64_t lower_bound_gt(const uint64_t* __restrict__ g, uint64_t lo, uint64_t hi, uint64_t v) {
    while (lo < hi) {
        const uint64_t mid = lo + ((hi - lo) >> 1);
        if (g[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ uint64_t upper_bound_gt(const uint64_t* __restrict__ g, uint64_t lo, uint64_t hi, uint64_t v) {
    while (lo < hi) {
        const uint64_t mid = lo + ((hi - lo) >> 1);
        if (g[mid] <= v) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(kSelThreads) k_select_and_fix(const uint64_t* __restrict__ live_gt,
                                                                 const uint64_t* __restrict__ spans, uint32_t J,
                                                                 uint64_t pivot, uint64_t to_select, int higher,
                                                                 uint64_t* __restrict__ cand_global,
                                                                 uint32_t cand_lds, uint64_t* __restrict__ out_spans,
                                                                 SelResult* __restrict__ res) {
    extern __shared__ uint64_t cand_shared[];
    __shared__ unsigned long long s_total, s_cands, s_cut, s_count;
    __shared__ unsigned long long s_first, s_last;
    const uint64_t L = to_select + 1;
    if (threadIdx.x == 0) {
        s_total = 0;
        s_cut = higher ? ~0ull : 0ull;
        s_count = 0;
        s_first = ~0ull;
        s_last = 0;
    }
    __syncthreads();
    // 1. each meta's candidates: higher [s, b) ascending; lower [a, s) (taken from its end)
    for (uint32_t j = threadIdx.x; j < J; j += blockDim.x) {
        const uint64_t a = spans[2 * j], b = spans[2 * j + 1];
        const uint64_t sj = higher ? upper_bound_gt(live_gt, a, b, pivot) : lower_bound_gt(live_gt, a, b, pivot);
        out_spans[2 * j] = sj;
        out_spans[2 * j + 1] = higher ? b - sj : sj - a;  // available candidates
        atomicAdd(&s_total, (unsigned long long)(higher ? b - sj : sj - a));
    }
    __syncthreads();
    const uint64_t total = s_total;
    const bool fixed = total >= L;
    if (fixed) {
        if (J == 1) {
            if (threadIdx.x == 0) s_cut = higher ? live_gt[out_spans[0] + L - 1] : live_gt[out_spans[0] - L];
        } else {
            uint64_t* cand = cand_lds ? cand_shared : cand_global;
            // offsets of each meta's first min(avail, L) candidates (single thread: J is small)
            if (threadIdx.x == 0) {
                uint64_t at = 0;
                for (uint32_t j = 0; j < J; ++j) {
                    const uint64_t m = out_spans[2 * j + 1] < L ? out_spans[2 * j + 1] : L;
                    out_spans[2 * j + 1] = at;  // reuse: the meta's offset into cand
                    at += m;
                }
                s_cands = at;
            }
            __syncthreads();
            const uint64_t C = s_cands;
            for (uint64_t i = threadIdx.x; i < C; i += blockDim.x) {
                uint32_t j = 0;
                while (j + 1 < J && out_spans[2 * (j + 1) + 1] <= i) ++j;
                const uint64_t t = i - out_spans[2 * j + 1];
                const uint64_t sj = out_spans[2 * j];
                const uint64_t mj = (j + 1 < J ? out_spans[2 * (j + 1) + 1] : C) - out_spans[2 * j + 1];
                cand[i] = higher ? live_gt[sj + t] : live_gt[sj - mj + t];  // ascending within the meta
            }
            __syncthreads();
            // rank: higher -> the L-th smallest v: #(< v) < L <= #(<= v); lower -> the L-th largest: #(> v) < L <= #(>= v)
            for (uint64_t i = threadIdx.x; i < C; i += blockDim.x) {
                const uint64_t v = cand[i];
                uint64_t lt = 0, le = 0;
                for (uint32_t j = 0; j < J; ++j) {
                    const uint64_t o = out_spans[2 * j + 1], e = j + 1 < J ? out_spans[2 * (j + 1) + 1] : C;
                    lt += lower_bound_gt(cand, o, e, v) - o;
                    le += upper_bound_gt(cand, o, e, v) - o;
                }
                const bool hit = higher ? (lt < L && L <= le) : (C - le < L && L <= C - lt);
                if (hit) s_cut = v;  // every hit carries the same value
            }
            __syncthreads();
            // restore the search starts
            if (threadIdx.x == 0) {
                for (uint32_t j = 0; j < J; ++j) {
                    const uint64_t a = spans[2 * j], b = spans[2 * j + 1];
                    out_spans[2 * j] = higher ? upper_bound_gt(live_gt, a, b, pivot) : lower_bound_gt(live_gt, a, b, pivot);
                }
            }
        }
    }
    __syncthreads();
    const uint64_t cut = s_cut;
    // 2. the kept rows per meta: strictly between the pivot and the cut (or every candidate when not over-full)
    for (uint32_t j = threadIdx.x; j < J; j += blockDim.x) {
        const uint64_t a = spans[2 * j], b = spans[2 * j + 1], sj = out_spans[2 * j];
        uint64_t x, y;
        if (higher) {
            x = sj;
            y = fixed ? lower_bound_gt(live_gt, sj, b, cut) : b;
        } else {
            x = fixed ? upper_bound_gt(live_gt, a, sj, cut) : a;
            y = sj;
        }
        out_spans[2 * j] = x;
        out_spans[2 * j + 1] = y;
        if (y > x) {
            atomicAdd(&s_count, (unsigned long long)(y - x));
            atomicMin(&s_first, (unsigned long long)live_gt[x]);
            atomicMax(&s_last, (unsigned long long)live_gt[y - 1]);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        res->count = s_count;
        res->first_gt = s_first;
        res->last_gt = s_last;
        res->total = total;
        res->fixed = fixed ? 1u : 0u;
        res->pad = 0;
    }
}

__global__ void __launch_bounds__(256) k_span_rows(const uint64_t* __restrict__ live_row,
                                                   const uint64_t* __restrict__ spans, uint32_t n_spans,
                                                   uint64_t* __restrict__ out_rows) {
    // one workgroup per span; its rows land after the earlier spans' (prefix by a short serial sum)
    const uint32_t j = blockIdx.x;
    uint64_t at = 0;
    for (uint32_t i = 0; i < j; ++i) at += spans[2 * i + 1] - spans[2 * i];
    const uint64_t x = spans[2 * j], y = spans[2 * j + 1];
    for (uint64_t i = x + threadIdx.x; i < y; i += 256) out_rows[at + (i - x)] = live_row ? live_row[i] : i;
}

hipError_t launch_select_and_fix(const uint64_t* live_gt, const uint64_t* spans, uint32_t J, uint64_t pivot,
                                 uint64_t to_select, int higher, uint64_t* cand, uint64_t* out_spans, SelResult* res,
                                 hipStream_t stream) {
    const uint64_t cap = (uint64_t)J * (to_select + 1);
    // dynamic LDS beside the kernel's static __shared__ words (a few hundred bytes): stay under 64 KiB per workgroup so
    // the launch also fits parts with 64 KiB of LDS (gfx950 has 160 KiB)
    const bool lds = J > 1 && cap * 8 <= 64 * 1024 - 1024;
    hipLaunchKernelGGL(k_select_and_fix, dim3(1), dim3(kSelThreads), lds ? (size_t)cap * 8 : 0, stream, live_gt, spans,
                       J, pivot, to_select, higher, cand, lds ? 1u : 0u, out_spans, res);
    return hipGetLastError();
}

hipError_t launch_span_rows(const uint64_t* live_row, const uint64_t* spans, uint32_t n_spans, uint64_t* out_rows,
                            hipStream_t stream) {
    if (!n_spans) return hipSuccess;
    hipLaunchKernelGGL(k_span_rows, dim3(n_spans), dim3(256), 0, stream, live_row, spans, n_spans, out_rows);
    return hipGetLastError();
}

}  // namespace dsy

// dsy_bloom_kernels.hip -- single-filter Bloom kernels for gfx950: build (add), membership test, index dump.
//
// Mapping: one key per lane (Merkle-Damgard is sequential per message), 256-thread workgroups, a grid-stride
// loop over 64-key wave-tasks.  Large batches are first put in length-bucketed order (k_len_* below: a counting
// sort of the keys by compression-block count, longest first) so the 64 lanes of a wave run the same number of
// blocks; the sort writes 16-byte task records (blob offset, length, key index) that the hashing kernel reads
// contiguously.  Small filters (the ~10 Kbit MTU filters of community.py:637-666) live in LDS for the whole
// workgroup: the build ORs bits with ds_or_b32 and merges the LDS filter into HBM once per workgroup; the test
// stages the filter into LDS once and probes it there.  Large filters (m = 2^20..2^24 bits, BASELINE config 4)
// are probed/ORed in place in L2/HBM with global atomics.  MD5 and SHA-1 stage packet bytes through LDS with
// LDS-DMA when the filter is small (dsy_message.h hash_key_dma_reg); SHA-2 loads directly.
#include "dsy_kernels.h"

namespace dsy {

static constexpr uint32_t kLenBins = 1024;
static constexpr int kDmaS = 2;
static constexpr size_t kDmaWaveBytes = DmaGeometry<kDmaS, 1>::kWaveBytes;
static constexpr size_t kLineWaveBytes = LineStaging::kWaveBytes;

// bin of a key in the length sort, longest first: by compression blocks, or (line_mode: the line-staged hashing,
// hash_key_dma_packed) by line stages, which also depend on where the message starts in its first line
__device__ __forceinline__ uint32_t len_bin(uint64_t off, uint64_t len, const LenSort& s) {
    uint32_t units = n_blocks(s.plen + (uint32_t)len, s.blk, s.lenb);
    if (s.line_mode) units = line_stages(units, (s.base_lo + (uint32_t)off - s.plen) & 127u);
    return kLenBins - 1u - min(units, kLenBins - 1u);
}

__device__ __forceinline__ void key_span(const uint64_t* __restrict__ offsets, const uint64_t* __restrict__ rows,
                                         const RowRec* __restrict__ rec, uint64_t i, uint64_t* off, uint32_t* len) {
    const uint64_t row = rows ? rows[i] : i;
    if (rec) {  // store rows: the packet's place in the store's line copy
        const RowRec r = rec[row];
        *off = r.off;
        *len = r.len;
        return;
    }
    const uint64_t a = offsets[row], e = offsets[row + 1];
    *off = a;
    *len = (uint32_t)(e - a);
}

// ---------------------------------------------------------------------------- length-bucketed task order
// pass 1: global histogram of bins (LDS-aggregated)
__global__ void __launch_bounds__(256) k_len_hist(LenSort s, const uint64_t* __restrict__ offsets,
                                                  const uint64_t* __restrict__ rows, const RowRec* __restrict__ rec, uint64_t n,
                                                  uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[kLenBins];
    for (uint32_t i = threadIdx.x; i < kLenBins; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint64_t off;
        uint32_t len;
        key_span(offsets, rows, rec, i, &off, &len);
        atomicAdd(&h[len_bin(off, len, s)], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < kLenBins; i += blockDim.x)
        if (h[i]) atomicAdd(&hist[i], h[i]);
}

// pass 2: exclusive scan of the bins (one workgroup of kLenBins threads)
__global__ void __launch_bounds__(kLenBins) k_len_scan(uint32_t* __restrict__ hist) {
    __shared__ uint32_t part[kLenBins];
    const uint32_t t = threadIdx.x;
    const uint32_t v = hist[t];
    part[t] = v;
    __syncthreads();
    for (uint32_t d = 1; d < kLenBins; d <<= 1) {
        const uint32_t add = t >= d ? part[t - d] : 0u;
        __syncthreads();
        part[t] += add;
        __syncthreads();
    }
    hist[t] = part[t] - v;
}

// pass 3: scatter task records; each workgroup reserves its bins' ranges with one global atomic per bin
static constexpr uint32_t kScatterChunk = 4096;
__global__ void __launch_bounds__(256) k_len_scatter(LenSort s, const uint64_t* __restrict__ offsets,
                                                     const uint64_t* __restrict__ rows, const RowRec* __restrict__ rec, uint64_t n,
                                                     uint32_t* __restrict__ base, PairTask* __restrict__ tasks) {
    __shared__ uint32_t cnt[kLenBins];
    __shared__ uint32_t at[kLenBins];
    for (uint64_t c0 = (uint64_t)blockIdx.x * kScatterChunk; c0 < n; c0 += (uint64_t)gridDim.x * kScatterChunk) {
        const uint64_t c1 = min(n, c0 + kScatterChunk);
        for (uint32_t i = threadIdx.x; i < kLenBins; i += blockDim.x) cnt[i] = 0;
        __syncthreads();
        for (uint64_t i = c0 + threadIdx.x; i < c1; i += blockDim.x) {
            uint64_t off;
            uint32_t len;
            key_span(offsets, rows, rec, i, &off, &len);
            atomicAdd(&cnt[len_bin(off, len, s)], 1u);
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < kLenBins; i += blockDim.x) {
            at[i] = cnt[i] ? atomicAdd(&base[i], cnt[i]) : 0u;
            cnt[i] = 0;
        }
        __syncthreads();
        for (uint64_t i = c0 + threadIdx.x; i < c1; i += blockDim.x) {
            PairTask tk;
            key_span(offsets, rows, rec, i, &tk.off, &tk.len);
            tk.slot = (uint32_t)i;
            const uint32_t b = len_bin(tk.off, tk.len, s);
            tasks[at[b] + atomicAdd(&cnt[b], 1u)] = tk;
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------- hash + probe / set
// DIAG (DMA path, 2-byte chunks only): 0 = the product kernel; 1 = no packet loads (the stage is hashed as left in
// LDS: the compute ceiling); 2 = packet loads without the compression (the gather ceiling).  Diagnostics only, selected
// by the ctx's DSY_BLOOM_DIAG environment knob (tools/hash_sweep.py); results are meaningless for DIAG != 0.
// OP 0: add (filter_set_all, OR_MODE as there), OP 1: test (present[key] = all k bits set).
// DMA 0: direct loads (hash_key); 1: LDS-DMA windows at the key's own alignment (hash_key_dma_reg); 2: line-aligned
// LDS-DMA stages (hash_key_dma_packed: each line of a key moved once).
template <class H, int CHUNK, int OP, int DMA, int DIAG = 0, int OR_MODE = 0>
__global__ void __launch_bounds__(256, 3) k_bloom(const DevParams* __restrict__ prm, const uint8_t* __restrict__ blob,
                                               const uint64_t* __restrict__ offsets, const uint64_t* __restrict__ rows,
                                               const RowRec* __restrict__ rec, const PairTask* __restrict__ tasks, uint64_t n,
                                               uint32_t* __restrict__ filter, uint32_t nwords, int use_lds,
                                               uint8_t* __restrict__ present) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn_lds[];
    constexpr size_t kWaveLds = DMA == 2 ? kLineWaveBytes : DMA == 1 ? kDmaWaveBytes : 0;
    uint8_t* my_dma = dyn_lds + (threadIdx.x >> 6) * kWaveLds;
    uint32_t* lds_filter = (uint32_t*)(dyn_lds + 4 * kWaveLds);
    const uint64_t m = prm->m_bits;
    const uint32_t k = prm->k;
    uint32_t preword = 0;  // the prefix's bytes, little-endian (DMA 2; <= 4 bytes)
    if constexpr (DMA == 2)
        for (uint32_t j = 0; j < min(prm->prefix_len, 4u); ++j) preword |= (uint32_t)prm->prefix[j] << (8 * j);
    if (use_lds) {
        for (uint32_t i = threadIdx.x; i < nwords; i += blockDim.x) lds_filter[i] = OP == 0 ? 0u : filter[i];
        __syncthreads();
    }
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t waves = (n + 63) / 64;
    const uint64_t wstride = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    // (the wave index through readfirstlane: wave-uniform to the compiler, so the loop control is scalar)
    const uint64_t v0 = (uint64_t)blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint64_t v = v0; v < waves; v += wstride) {
        const uint64_t i = v * 64 + lane;
        const bool active = i < n;
        // idle lanes hash an empty key; the LDS-DMA path still reads its stage from key - prefix_len, so the key
        // must sit past readable bytes: a packed blob has DSY_BLOB_GUARD of them before it, a store's line copy
        // (rec) keeps its guard inside the allocation
        KeyView kv{rec ? blob + DSY_BLOB_GUARD : blob, 0u, prm->prefix, prm->prefix_len};
        uint64_t slot = i;
        if (active) {
            if (tasks) {
                const PairTask tk = tasks[i];
                kv.key = blob + tk.off;
                kv.len = tk.len;
                slot = tk.slot;
            } else {
                uint64_t off;
                key_span(offsets, rows, rec, i, &off, &kv.len);
                kv.key = blob + off;
            }
        }
        H st;
        if constexpr (DMA == 2) hash_key_dma_packed<H, DIAG>(kv, st, my_dma, preword);
        else if constexpr (DMA == 1) hash_key_dma_reg<H, kDmaS, DIAG>(kv, st, my_dma);
        else hash_key<H>(kv, st);
        // two call sites, so each sees where its filter lives: ds_or / ds_read on the LDS copy, global atomics /
        // loads on the HBM one (one pointer picked at run time would be a flat pointer: every probe a flat atomic or
        // load behind its own vmcnt(0) wait -- 30 % of the SHA-1 add kernel)
        if constexpr (OP == 0) {
            if (use_lds) filter_set_all<H, CHUNK, OR_MODE>(lds_filter, st, k, m, active);
            else filter_set_all<H, CHUNK, OR_MODE>(filter, st, k, m, active);
        } else if (active) {
            const uint32_t ok = use_lds ? filter_has_all<H, CHUNK>(lds_filter, st, k, m)
                                        : filter_has_all<H, CHUNK>(filter, st, k, m);
            present[slot] = (uint8_t)ok;
        }
    }
    if (OP == 0 && use_lds) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < nwords; i += blockDim.x) {
            const uint32_t val = lds_filter[i];
            if (val) atomicOr(&filter[i], val);
        }
    }
}

template <class H, int CHUNK>
__global__ void __launch_bounds__(256) k_bloom_indices(const DevParams* __restrict__ prm, const uint8_t* __restrict__ blob,
                                                       const uint64_t* __restrict__ offsets, uint64_t n,
                                                       uint64_t* __restrict__ out) {
    const uint64_t m = prm->m_bits;
    const uint32_t k = prm->k;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t a = offsets[i], e = offsets[i + 1];
        KeyView kv{blob + a, (uint32_t)(e - a), prm->prefix, prm->prefix_len};
        H st;
        hash_key<H>(kv, st);
#pragma unroll
        for (int j = 0; j < ChunkLimit<H, CHUNK>::kmax; ++j)
            if (j < (int)k) out[i * k + j] = bit_position<CHUNK>(digest_chunk<H, CHUNK>(st, j), m);
    }
}

// ------------------------------------------------------------------------------ union of partial filters
__global__ void __launch_bounds__(256) k_or_reduce(const uint4* __restrict__ parts, uint32_t n_parts, uint64_t vecs,
                                                   uint64_t stride_vecs, uint4* __restrict__ out) {
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < vecs; i += step) {
        uint4 acc = parts[i];
        for (uint32_t g = 1; g < n_parts; ++g) {
            const uint4 v = parts[g * stride_vecs + i];
            acc.x |= v.x; acc.y |= v.y; acc.z |= v.z; acc.w |= v.w;
        }
        out[i] = acc;
    }
}

__global__ void __launch_bounds__(256) k_or_reduce_tail(const uint32_t* __restrict__ parts, uint32_t n_parts,
                                                        uint64_t first, uint64_t words, uint32_t* __restrict__ out) {
    const uint64_t w = first + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= words) return;
    uint32_t acc = 0;
    for (uint32_t g = 0; g < n_parts; ++g) acc |= parts[g * words + w];
    out[w] = acc;
}

hipError_t launch_or_reduce(const uint32_t* parts, uint32_t n_parts, uint64_t words, uint32_t* out, uint32_t max_grid,
                            hipStream_t stream) {
    // 16-byte vectors when every part starts 16-byte aligned (words % 4 == 0 and aligned base pointers)
    const bool vec = words % 4 == 0 && ((uintptr_t)parts % 16) == 0 && ((uintptr_t)out % 16) == 0;
    uint64_t done = 0;
    if (vec && words) {
        const uint64_t vecs = words / 4;
        const uint64_t want = (vecs + 255) / 256;
        const uint32_t grid = (uint32_t)(want < max_grid ? want : max_grid);
        hipLaunchKernelGGL(k_or_reduce, dim3(grid), dim3(256), 0, stream, (const uint4*)parts, n_parts, vecs, vecs,
                           (uint4*)out);
        done = words;
    }
    if (done < words) {
        const uint64_t rest = words - done;
        hipLaunchKernelGGL(k_or_reduce_tail, dim3((uint32_t)((rest + 255) / 256)), dim3(256), 0, stream, parts, n_parts,
                           done, words, out);
    }
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------ dispatch
hipError_t launch_len_sort(const LenSort& s, const uint64_t* offsets, const uint64_t* rows, const RowRec* rec, uint64_t n,
                           uint32_t* d_bins, PairTask* d_tasks, uint32_t max_grid, hipStream_t stream) {
    hipError_t e = hipMemsetAsync(d_bins, 0, kLenBins * 4, stream);
    if (e != hipSuccess) return e;
    const uint64_t want = (n + 255) / 256;
    const uint32_t grid = (uint32_t)(want < max_grid ? (want ? want : 1) : max_grid);
    hipLaunchKernelGGL(k_len_hist, dim3(grid), dim3(256), 0, stream, s, offsets, rows, rec, n, d_bins);
    hipLaunchKernelGGL(k_len_scan, dim3(1), dim3(kLenBins), 0, stream, d_bins);
    const uint64_t chunks = (n + kScatterChunk - 1) / kScatterChunk;
    const uint32_t sgrid = (uint32_t)(chunks < max_grid ? (chunks ? chunks : 1) : max_grid);
    hipLaunchKernelGGL(k_len_scatter, dim3(sgrid), dim3(256), 0, stream, s, offsets, rows, rec, n, d_bins, d_tasks);
    return hipGetLastError();
}

// Which staging k_bloom uses (bloom_staging): 2 = line-aligned (hash_key_dma_packed), 1 = windows at the key's own
// alignment (hash_key_dma_reg), 0 = direct loads.  LDS-DMA is for MD5 / SHA-1 (64-byte blocks; SHA-2 is
// compute-bound enough that direct loads match it) with prefixes of <= 4 bytes, when the LDS filter leaves room:
// line staging takes 12 KiB per wave, so three 4-wave workgroups per CU (the VGPR limit) fit beside filters of
// <= 5 KiB (the MTU filter is 1.3 KiB); window staging 8 KiB per wave.
int bloom_staging(const BloomLaunch& L) {
    if (!(L.kind == DSY_MD5 || L.kind == DSY_SHA1) || L.prm_prefix_len > 4) return 0;
    const uint64_t fbytes = L.use_lds ? (uint64_t)L.nwords * 4 : 0;
    if (((L.line_kinds >> L.kind) & 1u) && fbytes <= 5 * 1024) return 2;
    return fbytes <= 16 * 1024 ? 1 : 0;
}

template <class H, int CHUNK, int OP, int OR_MODE>
static hipError_t launch_op(const BloomLaunch& L, uint32_t grid) {
    const int dma = bloom_staging(L);
    const size_t lds = (dma == 2 ? 4 * kLineWaveBytes : dma == 1 ? 4 * kDmaWaveBytes : 0) +
                       (L.use_lds ? (size_t)L.nwords * 4 : 0);
    if constexpr (H::block_bytes == 64) {
        if (dma) {
            if constexpr (CHUNK == 2 && OR_MODE == 0) {
                if (L.diag == 1 || L.diag == 2) {
                    auto kern = dma == 2 ? (L.diag == 1 ? k_bloom<H, CHUNK, OP, 2, 1> : k_bloom<H, CHUNK, OP, 2, 2>)
                                         : (L.diag == 1 ? k_bloom<H, CHUNK, OP, 1, 1> : k_bloom<H, CHUNK, OP, 1, 2>);
                    launch_timed(kern, dim3(grid), dim3(256), lds, L.stream, L.ev_start, L.ev_stop, L.prm, L.blob,
                                 L.offsets, L.rows, L.rec, L.tasks, L.n, L.filter, L.nwords, L.use_lds, L.present);
                    return hipGetLastError();
                }
            }
            launch_timed(dma == 2 ? k_bloom<H, CHUNK, OP, 2, 0, OR_MODE> : k_bloom<H, CHUNK, OP, 1, 0, OR_MODE>,
                         dim3(grid), dim3(256), lds, L.stream, L.ev_start, L.ev_stop, L.prm, L.blob, L.offsets, L.rows,
                         L.rec, L.tasks, L.n, L.filter, L.nwords, L.use_lds, L.present);
            return hipGetLastError();
        }
    }
    launch_timed(k_bloom<H, CHUNK, OP, 0, 0, OR_MODE>, dim3(grid), dim3(256), lds, L.stream, L.ev_start, L.ev_stop, L.prm,
                 L.blob, L.offsets, L.rows, L.rec, L.tasks, L.n, L.filter, L.nwords, L.use_lds, L.present);
    return hipGetLastError();
}

template <class H, int CHUNK>
static hipError_t launch_family(const BloomLaunch& L) {
    const uint32_t block = 256;
    const uint64_t want = (L.n + block - 1) / block;
    const uint32_t grid = (uint32_t)(want < L.max_grid ? (want ? want : 1) : L.max_grid);
    switch (L.op) {
        case BloomOp::Add:
            switch (L.or_mode) {
                case 0: return launch_op<H, CHUNK, 0, 0>(L, grid);
                case 2: return launch_op<H, CHUNK, 0, 2>(L, grid);
                default: return launch_op<H, CHUNK, 0, 1>(L, grid);
            }
        case BloomOp::Test: return launch_op<H, CHUNK, 1, 0>(L, grid);
        case BloomOp::Indices:
            hipLaunchKernelGGL((k_bloom_indices<H, CHUNK>), dim3(grid), dim3(block), 0, L.stream, L.prm, L.blob,
                               L.offsets, L.n, L.indices);
            return hipGetLastError();
    }
    return hipErrorInvalidValue;
}

template <class H>
static hipError_t launch_chunk(const BloomLaunch& L) {
    switch (L.chunk) {
        case 2: return launch_family<H, 2>(L);
        case 4: return launch_family<H, 4>(L);
        default: return launch_family<H, 8>(L);
    }
}

hipError_t launch_bloom(const BloomLaunch& L) {
    switch (L.kind) {
        case 0: return launch_chunk<Md5>(L);
        case 1: return L.chunk == 8 ? hipErrorInvalidValue : (L.chunk == 2 ? launch_family<Sha1, 2>(L) : launch_family<Sha1, 4>(L));
        case 2: return launch_chunk<Sha256>(L);
        case 3: return launch_chunk<Sha384>(L);
        default: return launch_chunk<Sha512>(L);
    }
}

}  // namespace dsy

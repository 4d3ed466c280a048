// dsy_bloom_kernels.hip -- single-filter Bloom kernels for gfx950: build (add), membership test, index dump.
//
// Mapping: one key per lane (Merkle-Damgard is sequential per message), 256-thread workgroups, grid-stride
// over keys.  Small filters (the ~10 Kbit MTU filters of community.py:637-666) live in LDS for the whole
// workgroup: the build ORs bits with ds_or_b32 and merges the LDS filter into HBM once per workgroup; the
// test stages the filter into LDS once and probes it there.  Large filters (m = 2^20..2^24 bits, BASELINE
// config 4) are probed/ORed in place in HBM/L2 with global atomics.
#include "dsy_kernels.h"

namespace dsy {

template <class H, int CHUNK>
__global__ void __launch_bounds__(256) k_bloom_add(const DevParams* __restrict__ prm, const uint8_t* __restrict__ blob,
                                                   const uint64_t* __restrict__ offsets, const uint64_t* __restrict__ rows,
                                                   uint64_t n, uint32_t* __restrict__ filter, uint32_t nwords, int use_lds) {
    extern __shared__ uint32_t lds_filter[];
    const uint64_t m = prm->m_bits;
    const uint32_t k = prm->k;
    if (use_lds) {
        for (uint32_t i = threadIdx.x; i < nwords; i += blockDim.x) lds_filter[i] = 0;
        __syncthreads();
    }
    uint32_t* dst = use_lds ? lds_filter : filter;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t row = rows ? rows[i] : i;
        const uint64_t a = offsets[row], e = offsets[row + 1];
        KeyView kv{blob + a, (uint32_t)(e - a), prm->prefix, prm->prefix_len};
        H st;
        hash_key<H>(kv, st);
#pragma unroll
        for (int j = 0; j < ChunkLimit<H, CHUNK>::kmax; ++j) {
            if (j < (int)k) {
                const uint64_t pos = bit_position<CHUNK>(digest_chunk<H, CHUNK>(st, j), m);
                atomicOr(&dst[pos >> 5], 1u << (pos & 31));
            }
        }
    }
    if (use_lds) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < nwords; i += blockDim.x) {
            const uint32_t v = lds_filter[i];
            if (v) atomicOr(&filter[i], v);
        }
    }
}

template <class H, int CHUNK>
__global__ void __launch_bounds__(256) k_bloom_test(const DevParams* __restrict__ prm, const uint8_t* __restrict__ blob,
                                                    const uint64_t* __restrict__ offsets, uint64_t n,
                                                    const uint32_t* __restrict__ filter, uint32_t nwords, int use_lds,
                                                    uint8_t* __restrict__ present) {
    extern __shared__ uint32_t lds_filter[];
    const uint64_t m = prm->m_bits;
    const uint32_t k = prm->k;
    if (use_lds) {
        for (uint32_t i = threadIdx.x; i < nwords; i += blockDim.x) lds_filter[i] = filter[i];
        __syncthreads();
    }
    const uint32_t* src = use_lds ? lds_filter : filter;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t a = offsets[i], e = offsets[i + 1];
        KeyView kv{blob + a, (uint32_t)(e - a), prm->prefix, prm->prefix_len};
        H st;
        hash_key<H>(kv, st);
        uint32_t ok = 1;
#pragma unroll
        for (int j = 0; j < ChunkLimit<H, CHUNK>::kmax; ++j) {
            if (j < (int)k) {
                const uint64_t pos = bit_position<CHUNK>(digest_chunk<H, CHUNK>(st, j), m);
                ok &= (src[pos >> 5] >> (pos & 31)) & 1u;
            }
        }
        present[i] = (uint8_t)ok;
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

// ------------------------------------------------------------------------------------------ dispatch
template <class H, int CHUNK>
static hipError_t launch_family(const BloomLaunch& L) {
    const uint32_t block = 256;
    const uint64_t want = (L.n + block - 1) / block;
    const uint32_t grid = (uint32_t)(want < L.max_grid ? (want ? want : 1) : L.max_grid);
    const size_t lds = L.use_lds ? (size_t)L.nwords * 4 : 0;
    switch (L.op) {
        case BloomOp::Add:
            hipLaunchKernelGGL((k_bloom_add<H, CHUNK>), dim3(grid), dim3(block), lds, L.stream, L.prm, L.blob, L.offsets,
                               L.rows, L.n, L.filter, L.nwords, L.use_lds);
            break;
        case BloomOp::Test:
            hipLaunchKernelGGL((k_bloom_test<H, CHUNK>), dim3(grid), dim3(block), lds, L.stream, L.prm, L.blob,
                               L.offsets, L.n, (const uint32_t*)L.filter, L.nwords, L.use_lds, L.present);
            break;
        case BloomOp::Indices:
            hipLaunchKernelGGL((k_bloom_indices<H, CHUNK>), dim3(grid), dim3(block), 0, L.stream, L.prm, L.blob,
                               L.offsets, L.n, L.indices);
            break;
    }
    return hipGetLastError();
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

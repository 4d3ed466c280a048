// dsy_pipe_kernels.hip -- the responder's line-staged MD5 / SHA-1 hashing as a software pipeline per wave
// (k_pair_pipe), the product path of launch_pair_test_list for prefixes of 1..4 bytes and 2- or 4-byte chunks;
// the reference step it computes is community.py:2555-2567 (not_filter over the claim's rows, bloomfilter.py:185-197).
#include "dsy_kernels.h"

namespace dsy {

// -------------------------------------------------------------------------------------- k_pair_pipe
// The line-staged responder hashing (MD5 / SHA-1, prefixes of 1..4 bytes) as ONE software pipeline per wave over its
// wave-tasks, instead of k_pair_test's task-after-task walk.  In k_pair_test every wave-task started with a chain of
// dependent loads -- the listed slot, its claim, the claim's window size, the pair records, the claim's record --
// each behind its own vmcnt(0), then its first line DMA and another vmcnt(0): ~5-10 us in which the wave issued
// nothing (DSY_PAIR_TRACE: a 4-block wave-task took 5 us per block against 1.8 for a 20-block one; config 5's
// mostly one-stage wave-tasks 8 us per block).  Here, per wave:
//   - the wave-uniform chain (slot -> claim -> window size -> claim record) is read with scalar loads (constant
//     address space: lgkmcnt, not vmcnt, so it never waits for a line DMA in flight);
//   - the NEXT wave-task's pair records are loaded one task ahead, and its first line DMA is issued as soon as the
//     current task's last stage has been copied out of LDS -- it lands while that stage compresses;
//   - a finished task's filter probe is issued just before the next stage wait and tested after it (one wait for
//     the probe words, the next line DMA and the next records together).
// Same answers as k_pair_test (the miss bits of the same window slots); DSY_PAIR_PIPE=0 selects k_pair_test.
// Wave-wide max / min of a lane value, returned wave-uniform (SGPR): DPP within each row of 16 lanes, then the four
// rows' results by readlane.  Needs every lane active.  (The __shfl_xor butterfly costs six ds_bpermute round trips
// and six lane-index registers that the compiler keeps live across the whole walk -- it spilled them.)
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t wave_max_uniform(uint32_t v) {
    v = max(v, dpp_u32<0xB1>(v));   // quad_perm [1, 0, 3, 2]
    v = max(v, dpp_u32<0x4E>(v));   // quad_perm [2, 3, 0, 1]
    v = max(v, dpp_u32<0x141>(v));  // row_half_mirror
    v = max(v, dpp_u32<0x140>(v));  // row_mirror
    const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
    const uint32_t c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
    return max(max(a, b), max(c, d));
}
__device__ __forceinline__ uint32_t wave_min_uniform(uint32_t v) {
    v = min(v, dpp_u32<0xB1>(v));
    v = min(v, dpp_u32<0x4E>(v));
    v = min(v, dpp_u32<0x141>(v));
    v = min(v, dpp_u32<0x140>(v));
    const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
    const uint32_t c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
    return min(min(a, b), min(c, d));
}

// The lane id as an opaque value: every call recomputes it (two VALU), so the compiler does not hoist the lane-derived
// constants of the per-task setup (piece chunk numbers, shuffle addresses) out of the walk and keep -- or spill --
// dozens of them for the whole kernel.
__device__ __forceinline__ uint32_t opaque_lane() {
    uint32_t l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// wave-uniform values made explicit (SGPR): the walk's control flow is then uniform branches, not exec-masked regions
__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t uni(uint64_t x) {
    return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32) | __builtin_amdgcn_readfirstlane((uint32_t)x);
}
__device__ __forceinline__ bool uni(bool b) { return __builtin_amdgcn_readfirstlane((uint32_t)b) != 0; }

template <class T>
__device__ __forceinline__ const __attribute__((address_space(4))) T* cview(const T* p) {
    return (const __attribute__((address_space(4))) T*)(p);
}

// A wave-task as the pipeline walks it (wave-uniform): wave-task v is chunk v / n_list of window slot req_list[v %
// n_list]; its pairs are the window's task records [base, base + n_in)
struct PipeTask {
    uint32_t v, a_slot, r, n_in;
    uint64_t base;
};

// the first non-empty wave-task at or after v along the grid stride (v == total: none)
__device__ __forceinline__ bool pipe_find(const RespondLaunch& L, const uint32_t* req_list, uint32_t n_list,
                                          uint32_t total, uint32_t wstride, uint32_t W, uint32_t v, PipeTask& t) {
    for (v = uni(v); v < total; v += wstride) {
        const uint32_t a = uni(cview(req_list)[v % n_list]);
        const uint32_t r = uni(cview(L.act)[a]);
        const uint64_t n = uni(cview(L.state)[r].n_window);
        const uint64_t i0 = (uint64_t)(v / n_list) * 64;
        if (i0 >= n) continue;  // past this claim's window
        if (n > W) {            // (cannot happen: the fill never places more than W pairs)
            if ((threadIdx.x & 63) == 0) guard_trip(L.h_status, kGuardWindow);
            continue;
        }
        t.v = v;
        t.a_slot = a;
        t.r = r;
        t.n_in = (uint32_t)min<uint64_t>(64, n - i0);
        t.base = (uint64_t)a * W + i0;
        return true;
    }
    t.v = total;
    return false;
}

// The line DMA pieces one lane moves for its wave's 64 packets (DmaLinePieces' layout, dsy_message.h, with an XOR
// swizzle in place of the rotation: piece i is 16-byte chunk c_i of key p_i = 8 i + lane / 8, c_i = (lane % 8) ^
// (p_i / 2 % 8); a key's chunk q then sits at (its row) | 16 (q ^ r), so its reader forms the eight addresses with
// one XOR each and the lanes of every ds_read_b128 group still hit 16 distinct 4-bank groups), kept as what the
// issue needs:
// lc_i = 8 x (key p_i's first line, counted from the line copy's base) + c_i -- the piece of stage s is 16 bytes at
// base + 16 (lc_i + 8 s) -- and the number of stages in which the piece holds packet bytes (two per register).
// The address is formed by one add and one 64-bit shift-add (inline asm, so the compiler neither hoists per-piece
// 64-bit partial sums out of the stage loop -- 16 live VGPRs per task -- nor spills them).  Needs the line copy
// under 64 GiB (lc < 2^32; the host checks it).
struct PipePieces {
    uint32_t lc[8];
    uint32_t ns2[4];
    __device__ __forceinline__ void init(const uint8_t* base, const uint8_t* key, uint32_t len) {
        const uint32_t lane = opaque_lane();
        const uint32_t my_line = (uint32_t)((uint64_t)(key - base) >> 7);
        const uint32_t my_end = len + (uint32_t)kLineBias;  // bytes of the key's lines up to its last packet byte
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int p = 8 * i + (int)(lane / 8);
            const uint32_t c = (lane % 8) ^ (((uint32_t)p >> 1) & 7);
            const uint32_t ln = (uint32_t)__shfl((int)my_line, p, 64);
            const uint32_t end = (uint32_t)__shfl((int)my_end, p, 64);
            lc[i] = (ln << 3) + c;
            const uint32_t ns = end > 16 * c ? (end - 16 * c + 127) >> 7 : 0u;
            if (i & 1) ns2[i / 2] |= ns << 16;
            else ns2[i / 2] = ns;
        }
    }
    template <bool SKIP>
    __device__ __forceinline__ void issue(uint32_t s, const uint8_t* base, uint32_t lds) const {
        if constexpr (SKIP) return;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t ns = (i & 1) ? ns2[i / 2] >> 16 : ns2[i / 2] & 0xffffu;
            if (s < ns) {
                const uint64_t x = lc[i] + (s << 3);
                uint64_t a;
                asm volatile("v_lshl_add_u64 %0, %1, 4, %2" : "=v"(a) : "v"(x), "s"(base));
                __builtin_amdgcn_global_load_lds((const void*)(uintptr_t)a,
                                                 (__attribute__((address_space(3))) void*)(uintptr_t)(lds + i * 1024),
                                                 16, 0, 0);
            }
        }
    }
};

// One lane's part of a wave-task in the pipeline, from its pair record: the packet's length, the slot its miss bit
// goes to, and the hash state.  (The line pieces are kept apart, PipePieces: the next task's replace the current
// task's as soon as its last stage is issued, so only one set is ever live.)
template <class H>
struct PipeLane {
    H st;
    uint32_t len, total, nb, slot, carry;
    bool active;
};
// the wave-uniform part: the claim's prefix handling and filter, and the stage count
struct PipeUni {
    uint32_t nst, tmin, rr, sh, slack, plen, k, recip, a_slot;
    uint64_t m;
    const uint32_t* filt;
};

__device__ __forceinline__ PipeUni uni(const PipeUni& a) {
    PipeUni b;
    b.nst = uni(a.nst); b.tmin = uni(a.tmin); b.rr = uni(a.rr); b.sh = uni(a.sh); b.slack = uni(a.slack);
    b.plen = uni(a.plen); b.k = uni(a.k); b.recip = uni(a.recip); b.a_slot = uni(a.a_slot); b.m = uni(a.m);
    b.filt = (const uint32_t*)(uintptr_t)uni((uint64_t)(uintptr_t)a.filt);
    return b;
}

// The lane's pair of wave-task t from its record: the packet's place in the line copy and length, and its window
// slot -- or an idle lane (an empty key past the guard) when the lane is past the task or the record fails the
// bounds check (reported through the status word, never dereferenced)
__device__ __forceinline__ bool pipe_key(const RespondLaunch& L, const PipeTask& t, const PairTask& tk, uint32_t lane,
                                         const uint8_t*& key, uint32_t& len, uint32_t& slot) {
    key = L.st.lines + DSY_BLOB_GUARD;
    len = 0;
    slot = 0;
    if (lane >= t.n_in) return false;
    if (tk.off < DSY_BLOB_GUARD || tk.off + tk.len + DSY_BLOB_GUARD > L.st.lines_bytes || tk.slot >= L.window) {
        guard_trip(L.h_status, kGuardTask);
        return false;
    }
    key = L.st.lines + tk.off;
    len = tk.len;
    slot = tk.slot;
    return true;
}

// the rest of wave-task t's per-lane and uniform state (its pieces were set up when its first line went out)
template <class H>
__device__ __forceinline__ void pipe_setup(const RespondLaunch& L, const PipeTask& t, const PairTask& tk,
                                           PipeLane<H>& c, PipeUni& u, uint32_t& acc_slots) {
    const uint32_t lane = opaque_lane();
    const auto* q = cview(L.reqs) + uni(t.r);
    const uint32_t plen = uni(q->prefix_len), preword = uni(q->prefix_word);
    u.plen = plen;
    u.k = uni(q->k);
    u.recip = uni(q->m_recip);
    u.m = uni(q->m_bits);
    u.filt = (const uint32_t*)(L.filters + uni(q->filter_offset));
    u.a_slot = uni(t.a_slot);
    const uint8_t* key;
    uint32_t len, slot;
    const bool active = pipe_key(L, t, tk, lane, key, len, slot);
    c.active = active;
    c.len = len;
    c.slot = slot;
    c.total = plen + len;
    c.nb = active ? n_blocks(c.total, 64, H::len_bytes) : 0u;
    // the wave's longest lane (stages) and shortest active message (the partial-block test), wave-uniform
    const uint32_t mx = wave_max_uniform(c.nb), mn = wave_min_uniform(active ? c.total : 0xffffffffu);
    u.nst = uni((mx + 1) / 2);
    u.tmin = uni(mn);
    acc_slots += 64u * mx;
    // prefix handling as hash_key_dma_lines: message byte j is line byte j - rr
    const uint32_t rr = plen - 1;
    u.rr = rr;
    u.sh = (4 - rr) & 3;
    u.slack = (preword >> (8 * rr)) & 0xffu;
    c.carry = rr ? (preword & low_bytes_mask(rr)) << (8 * (4 - rr)) : 0u;
    c.st.init();
}

// the wave's issue priority for a wave-task of `blocks` blocks in its longest lane (k_pair_test's pair_prio rule)
__device__ __forceinline__ void pipe_prio(int mode, uint32_t blocks) {
    const uint32_t b = mode == 2 ? blocks * 16 : mode == 1 ? blocks : 0u;
    if (b >= 256) __builtin_amdgcn_s_setprio(3);
    else if (b >= 64) __builtin_amdgcn_s_setprio(2);
    else if (b >= 32) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}

// LDS per wave: the 8 KiB stage buffer, then the claim's filter (the probe reads it from LDS: lgkmcnt, so it never
// waits for the next task's line DMA already in flight).  4 waves x 9.5 KiB + 96 B per workgroup, 4 workgroups per CU.
static constexpr uint32_t kPipeFilterBytes = 1536;  // filters of up to 12288 bits (MTU filters are ~10 Kbit)
static constexpr uint32_t kPipeWaveBytes = DmaGeometry<2, 1>::kWaveBytes + kPipeFilterBytes;

// the claim's filter words into the wave's LDS filter slot (1 KiB per wave-instruction; up to 15 bytes read past
// the filter, inside the filter blob's 64-byte tail)
template <bool SKIP>
__device__ __forceinline__ void pipe_filter_dma(const uint32_t* filt, uint64_t m, uint32_t lds_filter) {
    if constexpr (SKIP) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nbytes = (uint32_t)((m + 31) / 32) * 4;
    if (nbytes > kPipeFilterBytes) return;  // probed from global memory instead (pipe_probe_word)
#pragma unroll
    for (uint32_t i = 0; i < (kPipeFilterBytes + 1023) / 1024; ++i) {
        const uint32_t o = i * 1024 + 16 * lane;
        if (o < nbytes)
            __builtin_amdgcn_global_load_lds((const void*)((const uint8_t*)filt + o),
                                             (__attribute__((address_space(3))) void*)(uintptr_t)(lds_filter + i * 1024),
                                             16, 0, 0);
    }
}

template <class H, int CHUNK, int MODE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8)))
k_pair_pipe(RespondLaunch L, const uint32_t* __restrict__ req_list, uint32_t n_list, uint32_t fam) {
    static_assert(H::block_bytes == 64, "LDS-DMA staging is for 64-byte blocks");
    extern __shared__ __attribute__((aligned(16))) uint8_t dma_lds[];
    using G = DmaGeometry<2, 1>;
    constexpr int kmax = ChunkLimit<H, CHUNK>::kmax;
    (void)fam;
    const uint32_t W = (uint32_t)L.window;
    const uint32_t total = n_list * min(cview(L.flags)[kFlagChunks], W / 64);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave_in_wg = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t wave0 = blockIdx.x * (blockDim.x >> 6) + wave_in_wg;
    const uint32_t wstride = gridDim.x * (blockDim.x >> 6);
    uint8_t* my_lds = dma_lds + wave_in_wg * kPipeWaveBytes;
    const uint32_t* my_filter = (const uint32_t*)(my_lds + G::kWaveBytes);
    const uint32_t lds = lds_local(my_lds);
    const uint32_t lds_filter = lds + G::kWaveBytes;
    const uint8_t* lines = L.st.lines;
    uint32_t acc_blocks = 0;
    uint64_t acc_bytes = 0;
    uint32_t acc_slots = 0;  // the wave's sum of 64 x its longest lane per wave-task (wave-uniform)

    // one setup site: the walk starts with an empty task (no stages, inactive lanes) whose "last stage" sets up the
    // first real one
    PipeTask nt;
    bool have_n = pipe_find(L, req_list, n_list, total, wstride, W, wave0, nt);
    if (have_n) {
        PipeLane<H> c;
        PipeUni u;
        PipePieces dl;  // the line pieces of the task whose stages are being issued
        c.active = false;
        c.nb = 0;
        u.nst = 0;
        PairTask ntk{};
        if (lane < nt.n_in) ntk = L.task[nt.base + lane];
        uint32_t s = 0;
        for (;;) {
            __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): this stage (and the claim's filter, the next records)
            __builtin_amdgcn_wave_barrier();
            const bool last = uni(s + 1 >= u.nst);  // (an empty task: "last" at once)
            uint32_t d[33];
            const bool staged = uni(u.nst != 0);
            if (staged) {
                d[0] = c.carry;
                {
                    // key k's chunk q: LDS (k / 8) KiB + 128 (k % 8) + 16 (q ^ (k / 2 % 8)) of the wave's buffer
                    const uint32_t k = opaque_lane();
                    const uint32_t row = (k >> 3) * 1024 + 128 * (k & 7) + 16 * ((k >> 1) & 7);
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        const uint4 v = *(const uint4*)(my_lds + (row ^ (16u * q)));
                        d[1 + 4 * q] = v.x; d[2 + 4 * q] = v.y; d[3 + 4 * q] = v.z; d[4 + 4 * q] = v.w;
                    }
                }
                if (s == 0) d[1] = (d[1] & ~0xffu) | u.slack;
                __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the buffer is free again
                __builtin_amdgcn_wave_barrier();
            }
            if (!last) {
                dl.template issue<MODE == 1>(s + 1, lines, lds);
            } else if (have_n) {  // the next task's first line lands while this stage compresses
                const uint8_t* nkey;
                uint32_t nlen, nslot;
                pipe_key(L, nt, ntk, opaque_lane(), nkey, nlen, nslot);
                dl.init(lines, nkey, nlen);
                dl.template issue<MODE == 1>(0, lines, lds);
            }
            if (staged) {
                c.carry = d[32];
#pragma unroll
                for (int bb = 0; bb < 2; ++bb) {
                    const uint32_t b = 2 * s + bb;
                    if (b < c.nb) {
                        uint32_t x[16];
                        if (u.rr == 0) {
#pragma unroll
                            for (int i = 0; i < 16; ++i) x[i] = d[1 + 16 * bb + i];
                        } else {
#pragma unroll
                            for (int i = 0; i < 16; ++i)
                                x[i] = __builtin_amdgcn_alignbyte(d[1 + 16 * bb + i], d[16 * bb + i], u.sh);
                        }
                        const uint32_t o0 = b * 64;
                        finish_block<H>(x, o0, c.total, b + 1 == c.nb, o0 + 64 <= u.tmin);
                        if (MODE != 2) c.st.template compress<true>(x);
                        else c.st.h[0] ^= x[0] ^ x[5] ^ x[10] ^ x[15];
                    }
                    // keep block 1's message words from being formed while block 0 compresses
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            if (!last) {
                ++s;
                continue;
            }
            if (staged) {  // the task is hashed: k probes of the claim's filter in LDS (bloomfilter.py:185-197)
                uint32_t w[kmax], sh[kmax];
#pragma unroll
                for (int j = 0; j < kmax; ++j) {
                    const uint32_t pos =
                        (uint32_t)bit_position<CHUNK>(digest_chunk<H, CHUNK>(c.st, j), u.m, u.recip);
                    // (a filter too large for the LDS slot is probed in global memory: its loads wait for the
                    // next task's line DMA too -- correct, slower; MTU filters never take it)
                    w[j] = u.m <= 8 * kPipeFilterBytes ? my_filter[pos >> 5] : u.filt[pos >> 5];
                    sh[j] = pos & 31u;
                }
                uint32_t ok = 1;
#pragma unroll
                for (int j = 0; j < kmax; ++j) ok &= (w[j] >> sh[j]) | (uint32_t)(j >= (int)u.k);
                if (c.active && !(ok & 1u) && MODE == 0)
                    atomicOr((unsigned long long*)&L.miss_mask[(uint64_t)u.a_slot * (W / 64) + c.slot / 64],
                             1ull << (c.slot % 64));
                if (c.active) {
                    acc_blocks += c.nb;
                    acc_bytes += c.len;
                }
                __builtin_amdgcn_s_waitcnt(0xc07f);  // the probe's LDS reads retired: the filter slot may refill
                __builtin_amdgcn_wave_barrier();
            }
            if (!have_n) break;
            pipe_setup<H>(L, nt, ntk, c, u, acc_slots);  // the next task becomes the current one
            u = uni(u);
            pipe_filter_dma<MODE == 1>(u.filt, u.m, lds_filter);
            s = 0;
            pipe_prio(L.pair_prio, 2 * u.nst);
            have_n = uni(pipe_find(L, req_list, n_list, total, wstride, W, nt.v + wstride, nt));
            if (have_n && lane < nt.n_in) ntk = L.task[nt.base + lane];
        }
        __builtin_amdgcn_s_setprio(0);
    }
    __shared__ unsigned long long red[3][4];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        acc_blocks += (uint32_t)__shfl_xor((int)acc_blocks, d, 64);
        acc_bytes += __shfl_xor(acc_bytes, d, 64);
    }
    if (lane == 0) {
        red[0][wave_in_wg] = acc_blocks;
        red[1][wave_in_wg] = acc_bytes;
        red[2][wave_in_wg] = acc_slots;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long b = 0, y = 0, z = 0;
        for (uint32_t wv = 0; wv < blockDim.x / 64; ++wv) b += red[0][wv], y += red[1][wv], z += red[2][wv];
        if (b) atomicAdd(counter(L.counters, kCntBlocks), b);
        if (y) atomicAdd(counter(L.counters, kCntBytes), y);
        if (z) atomicAdd(counter(L.counters, kCntSlots), z);
    }
}

hipError_t launch_pair_pipe(const RespondLaunch& L, int kind, uint32_t chunk, const uint32_t* list, uint32_t n_list,
                            uint32_t blocks, size_t lds) {
    void (*kern)(RespondLaunch, const uint32_t*, uint32_t, uint32_t) = nullptr;
    const int mode = L.diag == 1 ? 1 : L.diag == 2 ? 2 : 0;
#define DSY_PIPE_PICK(HH, CC)                                                                                  \
    kern = mode == 1 ? k_pair_pipe<HH, CC, 1> : mode == 2 ? k_pair_pipe<HH, CC, 2> : k_pair_pipe<HH, CC, 0>
    if (kind == DSY_MD5 && chunk == 2) DSY_PIPE_PICK(Md5, 2);
    else if (kind == DSY_MD5 && chunk == 4) DSY_PIPE_PICK(Md5, 4);
    else if (kind == DSY_SHA1 && chunk == 2) DSY_PIPE_PICK(Sha1, 2);
    else if (kind == DSY_SHA1 && chunk == 4) DSY_PIPE_PICK(Sha1, 4);
    else return hipErrorInvalidValue;
#undef DSY_PIPE_PICK
    (void)lds;
    launch_timed(kern, dim3(blocks), dim3(256), 4 * kPipeWaveBytes, L.stream, L.ev_start, L.ev_stop, L, list, n_list, (uint32_t)0);
    return hipSuccess;
}

}  // namespace dsy

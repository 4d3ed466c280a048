// dsy_sim_kernels.hip -- the multi-peer epidemic-sync simulator (BASELINE config 3) on gfx950.
//
// Every simulated peer runs the reference protocol once per round:
//   requester: _dispersy_claim_sync_bloom_filter_largest's "fewer than capacity packets" branch
//              (community.py:808-821): an MTU filter over its packets in global-time order, prefix one random
//              byte, range [1, acceptable] (or [1, gt of the capacity-th packet] when over-full)
//   responder: _get_packets_for_bloomfilters + the byte-limited not_filter loop (community.py:2555-2567) over its
//              own packets in global-time order
//   requester: stores what it received (Dispersy._store, dispersy.py:1475-1532)
// Peers are sharded over ranks by contiguous blocks; claims and responses travel between ranks as fixed-size
// records (the host side runs the two all-to-all(v) exchanges over RCCL).  Stores are bitsets over a universe of
// U packets with global_time(i) = i + 1, so "ascending global time" is "ascending bit index".
#include "dsy_kernels.h"

namespace dsy {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

__device__ __forceinline__ uint64_t sim_partner(const dsy_sim_config& c, uint32_t round, uint64_t p) {
    const uint64_t h = splitmix64(c.seed ^ ((uint64_t)round << 40) ^ (p * 0x2545f4914f6cdd1dull));
    return (p + 1 + h % (c.n_peers - 1)) % c.n_peers;
}

__device__ __forceinline__ uint32_t sim_prefix(const dsy_sim_config& c, uint32_t round, uint64_t p) {
    return (uint32_t)(splitmix64(c.seed * 3 + 0x51ed27ull + (uint64_t)round * c.n_peers + p) >> 32) & 0xffu;
}

__device__ __forceinline__ uint32_t sim_owner(const dsy_sim_config& c, uint64_t p) {
    return (uint32_t)(p / c.peers_per_rank);
}

// counts[key] += 1 for every active lane, with one atomic per distinct key in the wave (a million lanes adding to
// the same rank counter one by one serialise on one address); returns the lane's old value + its rank among the
// wave's lanes with the same key, i.e. a unique slot when counts holds running cursors
__device__ __forceinline__ uint32_t wave_count(uint32_t* counts, uint32_t key, bool active) {
    uint64_t pending = __ballot(active);
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
    uint32_t mine = 0;
    while (pending) {
        const int leader = __builtin_ctzll(pending);
        const uint32_t k = __shfl(key, leader, 64);
        const uint64_t same = __ballot(active && key == k) & pending;
        uint32_t base = 0;
        if (lane == (uint32_t)leader) base = atomicAdd(&counts[k], (uint32_t)__popcll(same));
        base = __shfl(base, leader, 64);
        if ((same >> lane) & 1) mine = base + (uint32_t)__popcll(same & below);
        pending &= ~same;
    }
    return mine;
}

// ------------------------------------------------------------------------------------------ seeding
__global__ void k_sim_seed(dsy_sim_config c, uint32_t* __restrict__ bits, uint32_t initial) {
    const uint64_t lp = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lp >= c.peer_end - c.peer_begin) return;
    const uint64_t p = c.peer_begin + lp;
    uint32_t* b = bits + lp * c.words;
    for (uint32_t w = 0; w < c.words; ++w) b[w] = 0;
    uint32_t have = 0;
    for (uint64_t j = 0; have < initial && have < c.universe; ++j) {
        const uint32_t id = (uint32_t)(splitmix64(c.seed * 7 + 0xabcdefull + p * 1000003ull + j) % c.universe);
        const uint32_t m = 1u << (id & 31);
        if (!(b[id >> 5] & m)) {
            b[id >> 5] |= m;
            ++have;
        }
    }
}

// ascending ids of one bitset into an LDS list (whole wave); returns the count
__device__ __forceinline__ uint32_t wave_list_ids(const uint32_t* __restrict__ b, uint32_t words, uint16_t* list,
                                                  uint32_t cap) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t n = 0;
    for (uint32_t w0 = 0; w0 < words; w0 += 64) {
        const uint32_t w = w0 + lane;
        uint32_t word = w < words ? b[w] : 0u;
        const uint32_t pc = __popc(word);
        uint32_t incl = pc;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(incl, d, 64);
            if ((int)lane >= d) incl += o;
        }
        uint32_t pos = n + incl - pc;
        while (word) {
            const uint32_t bit = __builtin_ctz(word);
            word &= word - 1;
            if (pos < cap) list[pos] = (uint16_t)(w * 32 + bit);
            ++pos;
        }
        n += __shfl(incl, 63, 64);
    }
    __builtin_amdgcn_wave_barrier();
    return n;
}

// --------------------------------------------------------------------------------------- claims
__global__ void k_sim_claim_counts(dsy_sim_config c, uint32_t round, uint32_t* __restrict__ counts) {
    const uint64_t lp = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = lp < c.peer_end - c.peer_begin;
    wave_count(counts, active ? sim_owner(c, sim_partner(c, round, c.peer_begin + lp)) : 0u, active);
}

// the round's whole claim traffic: m[r][src][dst] = claims the requesters of rank src send to responders of rank dst,
// for n_rounds rounds from round0 (grid.y = rounds).  Every rank computes the same matrix from the counter RNG, so
// the exchange needs no count all-to-all: a rank's send counts are its row, its receive counts its column.
__global__ void k_sim_claim_matrix(dsy_sim_config c, uint32_t round0, uint32_t n_ranks, uint32_t* __restrict__ m) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t r = blockIdx.y;
    const bool active = p < c.n_peers;
    const uint32_t key = active ? sim_owner(c, p) * n_ranks + sim_owner(c, sim_partner(c, round0 + r, p)) : 0u;
    wave_count(m + (uint64_t)r * n_ranks * n_ranks, key, active);
}

__global__ void k_sim_cursor_init(SimCursorInit ci, uint32_t* __restrict__ cursor) {
    if (threadIdx.x < ci.n) cursor[threadIdx.x] = ci.start[threadIdx.x];
}

// slot of every local requester's claim record: cursor[dest] starts at the destination's first record
__global__ void k_sim_claim_slots(dsy_sim_config c, uint32_t round, uint32_t* __restrict__ cursor,
                                  uint32_t* __restrict__ slots) {
    const uint64_t lp = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = lp < c.peer_end - c.peer_begin;
    const uint32_t s = wave_count(cursor, active ? sim_owner(c, sim_partner(c, round, c.peer_begin + lp)) : 0u, active);
    if (active) slots[lp] = s;
}

// slot of every received claim's response record (grouped by the requester's rank)
__global__ void k_sim_resp_slots(dsy_sim_config c, const uint8_t* __restrict__ claims, uint64_t n_claims,
                                 uint32_t* __restrict__ cursor, uint32_t* __restrict__ slots) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = i < n_claims;
    uint32_t owner = 0;
    if (active) owner = sim_owner(c, ((const dsy_sim_claim_header*)(claims + i * c.claim_bytes))->requester);
    const uint32_t s = wave_count(cursor, owner, active);
    if (active) slots[i] = s;
}

static constexpr uint32_t kSimListCap = 2048;

// per-wave work counters (compression blocks hashed; 64 x the longest lane's blocks = lane-block slots), spread
// over kSimTestedSlots copies; one atomic pair per wave at its end
__device__ __forceinline__ void wave_work(uint32_t lane_blocks, uint64_t& blocks, uint64_t& slots) {
    uint32_t sum = lane_blocks, mx = lane_blocks;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        sum += __shfl_xor(sum, d, 64);
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, d, 64));
    }
    blocks += sum;
    slots += 64ull * mx;
}
__device__ __forceinline__ void work_flush(unsigned long long* work, int which, uint64_t blocks, uint64_t slots) {
    if (work && (threadIdx.x & 63) == 0) {
        unsigned long long* w = work + ((blockIdx.x * 4 + (threadIdx.x >> 6)) & (kSimTestedSlots - 1)) * 4 + which;
        atomicAdd(w, (unsigned long long)blocks);
        atomicAdd(w + 1, (unsigned long long)slots);
    }
}

// LDS of one requester wave in k_sim_build_claims: its id list (4 KiB, reused as the LDS-DMA stage once the ids are
// pooled), the prefix byte and the filter (sized by m at launch)
__host__ __device__ constexpr uint32_t sim_build_wave_lds(uint32_t nwords) {
    return (2 * kSimListCap + 16 + nwords * 4 + 15) / 16 * 16;
}
// shared by the workgroup's four requesters: their claimed ids pooled in block-count order (id | owner << 16, at most
// 4 x capacity), a 64-bin histogram and the per-wave counts
__host__ __device__ constexpr uint32_t sim_build_lds(uint32_t nwords, uint32_t capacity) {
    return 4 * sim_build_wave_lds(nwords) + 4 * 4 * capacity + 64 * 4 + 16;
}

// One workgroup per four local requesters, each the reference's claim: _dispersy_claim_sync_bloom_filter_largest's
// "fewer than capacity packets" branch (community.py:808-821) over its packets in global-time order.  Every wave
// lists its requester's packets; the workgroup pools the four claims' keys (the filter is an OR, so the hashing
// order is free), sorts them by compression-block count, and the waves hash the pool in chunks of 64 near-equal
// lanes, round-robin, each key into its owner's LDS filter (filter_set_all, OR_MODE as there; a lane's filter is a
// word offset from one LDS base).  Sorting ~4 x 150 keys instead of each requester's ~150 keeps a chunk's lanes
// within a few blocks of each other.  Then every wave writes its claim record.
template <class H, int CHUNK, int OR_MODE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(H::kind == DSY_SHA256 ? 3 : 4, 8)))
k_sim_build_claims(dsy_sim_config c, uint32_t round, const uint8_t* __restrict__ ublob, const uint64_t* __restrict__ uoff,
                   const uint32_t* __restrict__ bits, uint8_t* __restrict__ out, const uint32_t* __restrict__ slots,
                   unsigned long long* __restrict__ work) {
    extern __shared__ __attribute__((aligned(16))) uint8_t sim_lds[];
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;  // (uniform: SALU)
    const uint64_t lp = (uint64_t)blockIdx.x * 4 + wv;
    const bool live = lp < c.peer_end - c.peer_begin;  // wave-uniform; idle waves still meet the barriers
    const uint32_t nwords = (uint32_t)((c.m_bits + 31) / 32);
    const uint32_t wave_b = sim_build_wave_lds(nwords);
    uint8_t* mine = sim_lds + wv * wave_b;
    uint16_t* list = (uint16_t*)mine;  // later: this wave's LDS-DMA stage (4 KiB)
    uint8_t* pre = mine + 2 * kSimListCap;
    uint32_t* filt = (uint32_t*)(pre + 16);
    uint32_t* pool = (uint32_t*)(sim_lds + 4 * wave_b);  // [4 * capacity]
    uint32_t* phist = pool + 4 * c.capacity;            // [64]
    uint32_t* pcnt = phist + 64;                        // [4]
    const uint64_t p = c.peer_begin + lp;
    const uint32_t blk = H::block_bytes, lenb = H::len_bytes;
    auto bin_of = [&](uint32_t id) { return 63u - min(n_blocks(1 + (uint32_t)(uoff[id + 1] - uoff[id]), blk, lenb), 63u); };
    for (uint32_t i = lane; i < nwords; i += 64) filt[i] = 0;
    if (threadIdx.x < 64) phist[threadIdx.x] = 0;
    uint32_t n = live ? wave_list_ids(bits + lp * c.words, c.words, list, kSimListCap) : 0u;
    // _select_and_fix(..., 0, capacity, True): the first capacity packets; over-full drops the (capacity+1)-th
    // global time (global times are distinct here) and the range ends at the last kept one
    uint64_t time_high = 0x7fffffffffffffffull;
    if (n > c.capacity) {
        n = c.capacity;
        time_high = (uint64_t)list[n - 1] + 1;
    }
    const uint32_t prefix = live ? sim_prefix(c, round, p) : 0u;
    if (lane == 0) {
        pre[0] = (uint8_t)prefix;
        pcnt[wv] = n;
    }
    __syncthreads();
    const uint32_t c0 = pcnt[0], c1 = pcnt[1], c2 = pcnt[2];
    const uint32_t pn = c0 + c1 + c2 + pcnt[3];
    for (uint32_t i = lane; i < n; i += 64) atomicAdd(&phist[bin_of(list[i])], 1u);
    __syncthreads();
    if (threadIdx.x < 64) {  // exclusive scan of the bins (longest first)
        const uint32_t hv = phist[threadIdx.x];
        uint32_t incl = hv;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(incl, d, 64);
            if ((int)lane >= d) incl += o;
        }
        phist[threadIdx.x] = incl - hv;
    }
    __syncthreads();
    for (uint32_t i = lane; i < n; i += 64) {
        const uint32_t id = list[i];
        pool[atomicAdd(&phist[bin_of(id)], 1u)] = id | (wv << 16);
    }
    __syncthreads();  // every list has been read: the waves' LDS-DMA stages may overwrite them
    // MD5 / SHA-1 stage the packets through LDS with DMA (hash_key_dma_reg, one 64-byte block per key per stage):
    // 8 keys x 64 contiguous bytes per wave instruction instead of 64 scattered 16-byte loads.  The universe blob keeps
    // DSY_BLOB_GUARD readable bytes on both sides (sim.py); idle lanes hash an empty key at its start.
    constexpr bool kDma = H::kind == DSY_MD5 || H::kind == DSY_SHA1;
    static_assert(DmaGeometry<1, 1>::kWaveBytes == 2 * kSimListCap, "the DMA stage reuses the id list");
    uint8_t* dma_buf = (uint8_t*)list;
    uint64_t wblocks = 0, wslots = 0;
    for (uint32_t j = wv; 64 * j < pn; j += 4) {
        const uint32_t i = 64 * j + lane;
        const bool act = i < pn;
        const uint32_t e = act ? pool[i] : 0u;
        const uint32_t id = e & 0xffffu, own = e >> 16;
        const uint32_t len = act ? (uint32_t)(uoff[id + 1] - uoff[id]) : 0u;
        wave_work(act ? n_blocks(1 + len, blk, lenb) : 0u, wblocks, wslots);
        uint8_t* own_lds = sim_lds + own * wave_b;
        KeyView kv{ublob + uoff[id], len, own_lds + 2 * kSimListCap, 1};
        H st;
        if constexpr (kDma) hash_key_dma_reg<H, 1>(kv, st, dma_buf);
        else if (act) hash_key<H>(kv, st);
        filter_set_all<H, CHUNK, OR_MODE>((uint32_t*)sim_lds, st, c.k, c.m_bits, act,
                                          (own * wave_b + 2 * kSimListCap + 16) / 4);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __syncthreads();
    work_flush(work, 0, wblocks, wslots);
    if (!live) return;
    const uint64_t q = sim_partner(c, round, p);
    uint8_t* rec = out + (uint64_t)slots[lp] * c.claim_bytes;
    if (lane == 0) {
        dsy_sim_claim_header h;
        h.requester = p;
        h.responder = q;
        h.time_high = time_high;
        h.prefix = prefix;
        h.n_sent = n;
        *(dsy_sim_claim_header*)rec = h;
    }
    uint32_t* fw = (uint32_t*)(rec + sizeof(dsy_sim_claim_header));
    for (uint32_t i = lane; i < nwords; i += 64) fw[i] = filt[i];
}

// -------------------------------------------------------------------------------------- responses
__global__ void k_sim_resp_counts(dsy_sim_config c, const uint8_t* __restrict__ claims, uint64_t n_claims,
                                  uint32_t* __restrict__ counts) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = i < n_claims;
    uint32_t owner = 0;
    if (active) owner = sim_owner(c, ((const dsy_sim_claim_header*)(claims + i * c.claim_bytes))->requester);
    wave_count(counts, owner, active);
}

// one wave per incoming claim: the responder's packets in global-time order, 64 at a time; hash + probe; send the
// missing ones until the byte budget is spent (the crossing packet is sent), then stop -- lazily, as the
// reference's generator chain does
// LDS of one responder wave in k_sim_respond: the responder's id list, the claim's filter (sized by m at launch), the
// prefix byte, the response ids and (MD5 / SHA-1) a 4 KiB LDS-DMA stage
__host__ __device__ constexpr uint32_t sim_respond_wave_lds(uint32_t nwords, bool dma) {
    return (2 * kSimListCap + nwords * 4 + 16 + 2 * kSimRespMax + 15) / 16 * 16 + (dma ? 4096u : 0u);
}
// shared by the workgroup's NW claims: one round's pooled candidates (id, owner, position) in block-count order,
// their miss flags per owner, a 64-bin histogram, per-wave counts and the active flags
__host__ __device__ constexpr uint32_t sim_resp_pool_lds(uint32_t nw) {
    return (64 * nw * 2 + 64 * nw + 64 * nw + nw * 64 + 64 * 4 + nw * 4 + 16 + 15) / 16 * 16;
}
__host__ __device__ constexpr uint32_t sim_respond_lds(uint32_t nwords, bool dma, uint32_t nw = 4) {
    return nw * sim_respond_wave_lds(nwords, dma) + sim_resp_pool_lds(nw);
}
// claims (waves) per k_sim_respond workgroup.  DSY_SIM_WAVES=8 pools twice the candidates per round at the same 16
// waves per CU (two 8-wave workgroups): lane utilisation 0.84 -> 0.91 but the launch 13.2 -> 14.2 ms (a round waits
// for the slowest of eight claims at its barriers), so four stay the default
static constexpr uint32_t kSimRespWaves = 8;

// One wave per incoming claim answers it: the responder's packets in global-time order, 64 candidates per round,
// hash + probe, then the missing ones are sent until the byte budget is spent (the crossing packet is sent) and the
// claim stops -- lazily, as the reference's generator chain does.  The workgroup's four claims hash together: each
// round pools every active claim's next <= 64 candidates (<= 256), sorts them by block count, and the four waves hash
// the pool in chunks of 64 equal-length lanes (the filter and prefix of each lane's own claim); then each claim's
// wave applies the budget rule to its candidates in order.  Without the pool a chunk runs as long as its longest
// random-length packet (lane utilisation 0.56).
template <class H, int CHUNK, int NW>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(H::kind == DSY_SHA256 ? 3 : 4, 8)))
k_sim_respond(dsy_sim_config c, const uint8_t* __restrict__ ublob, const uint64_t* __restrict__ uoff,
              const uint32_t* __restrict__ bits, const uint8_t* __restrict__ claims, uint64_t n_claims,
              uint8_t* __restrict__ out, const uint32_t* __restrict__ slots, unsigned long long* __restrict__ tested,
              unsigned long long* __restrict__ work) {
    extern __shared__ __attribute__((aligned(16))) uint8_t sim_lds[];
    // MD5 / SHA-1 stage the packets through LDS with DMA (hash_key_dma_reg, one block per stage), as the claim build
    constexpr bool kDma = H::kind == DSY_MD5 || H::kind == DSY_SHA1;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;  // (uniform: SALU)
    const uint64_t ci = (uint64_t)blockIdx.x * NW + wv;
    const bool live = ci < n_claims;  // wave-uniform; idle waves still meet the barriers
    const uint32_t nwords = (uint32_t)((c.m_bits + 31) / 32);
    const uint32_t wave_b = sim_respond_wave_lds(nwords, kDma);
    auto list_of = [&](uint32_t w) { return (uint16_t*)(sim_lds + w * wave_b + (kDma ? 4096 : 0)); };
    auto filt_of = [&](uint32_t w) { return (uint32_t*)(list_of(w) + kSimListCap); };
    uint8_t* dma_buf = sim_lds + wv * wave_b;  // 4 KiB, first (16-byte aligned)
    uint16_t* list = list_of(wv);
    uint32_t* filt = filt_of(wv);
    uint8_t* pre = (uint8_t*)(filt + nwords);
    uint16_t* outl = (uint16_t*)(pre + 16);
    uint8_t* pool = sim_lds + NW * wave_b;
    uint16_t* pool_id = (uint16_t*)pool;                 // [64 NW]
    uint8_t* pool_own = pool + 128 * NW;                 // [64 NW] owner wave
    uint8_t* pool_pos = pool + 192 * NW;                 // [64 NW] position in the owner's chunk
    uint8_t* flags = pool + 256 * NW;                    // [NW][64] miss flags of the round
    uint32_t* phist = (uint32_t*)(pool + 320 * NW);      // [64]
    uint32_t* pcnt = phist + 64;                         // [NW] candidates per wave this round
    dsy_sim_claim_header h{};
    uint32_t n_sel = 0;
    if (live) {
        const uint8_t* rec = claims + ci * c.claim_bytes;
        h = *(const dsy_sim_claim_header*)rec;
        const uint32_t* fw = (const uint32_t*)(rec + sizeof(dsy_sim_claim_header));
        for (uint32_t i = lane; i < nwords; i += 64) filt[i] = fw[i];
        if (lane == 0) pre[0] = (uint8_t)h.prefix;
        const uint32_t n = min(wave_list_ids(bits + (h.responder - c.peer_begin) * c.words, c.words, list, kSimListCap),
                               kSimListCap);
        // range [1, time_high]: global_time = id + 1, ids ascending, so the candidates are a prefix of the list
        for (uint32_t i0 = 0; i0 < n; i0 += 64)
            n_sel += (uint32_t)__popcll(__ballot(i0 + lane < n && (uint64_t)list[i0 + lane] + 1 <= h.time_high));
    }
    uint32_t sent = 0;
    int64_t spent = 0;
    uint32_t ntested = 0;
    bool done = !live;
    uint64_t wblocks = 0, wslots = 0;
    const uint32_t blk = H::block_bytes, lenb = H::len_bytes;
    auto bin_of = [&](uint32_t id) { return 63u - min(n_blocks(1 + (uint32_t)(uoff[id + 1] - uoff[id]), blk, lenb), 63u); };
    for (uint32_t k = 0;; ++k) {
        const uint32_t base = 64 * k;
        const uint32_t cnt = (!done && base < n_sel) ? min(64u, n_sel - base) : 0u;
        if (lane == 0) pcnt[wv] = cnt;
        if (threadIdx.x < 64) phist[threadIdx.x] = 0;
        __syncthreads();
        uint32_t pn = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) pn += pcnt[w];
        if (!pn) break;  // workgroup-uniform
        // pool this wave's candidates, then rank them by block count over the workgroup
        uint32_t my_id = 0, my_bin = 0;
        if (lane < cnt) {
            my_id = list[base + lane];
            my_bin = bin_of(my_id);
            atomicAdd(&phist[my_bin], 1u);
        }
        __syncthreads();
        if (threadIdx.x < 64) {
            const uint32_t hv = phist[threadIdx.x];
            uint32_t incl = hv;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_up(incl, d, 64);
                if ((int)lane >= d) incl += o;
            }
            phist[threadIdx.x] = incl - hv;
        }
        __syncthreads();
        if (lane < cnt) {
            const uint32_t slot = atomicAdd(&phist[my_bin], 1u);
            pool_id[slot] = (uint16_t)my_id;
            pool_own[slot] = (uint8_t)wv;
            pool_pos[slot] = (uint8_t)lane;
        }
        __syncthreads();
        if (wv * 64 < pn) {  // wave wv hashes pooled chunk wv (workgroup-uniform per wave)
            const uint32_t i = wv * 64 + lane;
            const bool act = i < pn;
            const uint32_t id = act ? pool_id[i] : 0u;
            const uint32_t own = act ? pool_own[i] : 0u;
            const uint32_t len = act ? (uint32_t)(uoff[id + 1] - uoff[id]) : 0u;
            wave_work(act ? n_blocks(1 + len, blk, lenb) : 0u, wblocks, wslots);
            const uint32_t* own_filt = filt_of(own);
            KeyView kv{ublob + uoff[id], len, (const uint8_t*)(own_filt + nwords), 1};
            H st;
            if constexpr (kDma) hash_key_dma_reg<H, 1>(kv, st, dma_buf);
            else if (act) hash_key<H>(kv, st);
            if (act) flags[own * 64 + pool_pos[i]] = (uint8_t)!filter_has_all<H, CHUNK>(own_filt, st, c.k, c.m_bits);
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __syncthreads();
        if (cnt) {  // this claim's budget rule over its candidates, in order
            const uint32_t id = lane < cnt ? list[base + lane] : 0u;
            const bool miss = lane < cnt && flags[wv * 64 + lane];
            const int64_t len = miss ? (int64_t)(uoff[id + 1] - uoff[id]) : 0;
            ntested += cnt;
            int64_t incl = len;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int64_t o = __shfl_up(incl, d, 64);
                if ((int)lane >= d) incl += o;
            }
            const uint64_t mmask = __ballot(miss);
            const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
            const uint32_t rank = __popcll(mmask & lt);
            const bool inc = miss && ((sent + rank == 0) || (spent + incl - len < c.byte_limit));
            const uint64_t imask = __ballot(inc);
            const uint32_t nin = __popcll(imask);
            if (inc && sent + rank < kSimRespMax) outl[sent + rank] = (uint16_t)id;
            if (nin) spent += __shfl(incl, 63 - __builtin_clzll(imask), 64);
            sent += nin;
            if (sent > 0 && spent >= c.byte_limit) done = true;
        }
        __syncthreads();  // the pool and the flags are rewritten next round
    }
    work_flush(work, 2, wblocks, wslots);
    if (!live) return;
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    uint8_t* o = out + (uint64_t)slots[ci] * c.resp_bytes;
    dsy_sim_resp_header* oh = (dsy_sim_resp_header*)o;
    const uint32_t cnt = min(sent, (uint32_t)kSimRespMax);
    if (lane == 0) {
        oh->requester = h.requester;
        oh->count = cnt;
        oh->overflow = sent > kSimRespMax;
        atomicAdd(&tested[blockIdx.x & (kSimTestedSlots - 1)], (unsigned long long)ntested);  // spread
    }
    uint16_t* ids = (uint16_t*)(o + sizeof(dsy_sim_resp_header));
    if (lane < cnt) ids[lane] = outl[lane];
}

// ------------------------------------------------------------------------------------------- merge
__global__ void k_sim_merge(dsy_sim_config c, uint32_t* __restrict__ bits, const uint8_t* __restrict__ resps,
                            uint64_t n_resps, uint32_t* __restrict__ overflow) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_resps) return;
    const uint8_t* r = resps + i * c.resp_bytes;
    const dsy_sim_resp_header h = *(const dsy_sim_resp_header*)r;
    if (h.overflow) atomicOr(overflow, 1u);
    uint32_t* b = bits + (h.requester - c.peer_begin) * c.words;
    const uint16_t* ids = (const uint16_t*)(r + sizeof(dsy_sim_resp_header));
    for (uint32_t j = 0; j < h.count; ++j) b[ids[j] >> 5] |= 1u << (ids[j] & 31);  // one response per requester
}

// per-rank digest of the stores: number of packets held and an order-independent checksum
__global__ void k_sim_stats(dsy_sim_config c, const uint32_t* __restrict__ bits, unsigned long long* __restrict__ out) {
    const uint64_t lp = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lp >= c.peer_end - c.peer_begin) return;
    const uint32_t* b = bits + lp * c.words;
    unsigned long long held = 0, h = 0;
    for (uint32_t w = 0; w < c.words; ++w) {
        held += __popc(b[w]);
        h ^= splitmix64(((c.peer_begin + lp) << 20) ^ ((uint64_t)w << 32) ^ b[w]);
    }
    atomicAdd(&out[0], held);
    atomicXor(&out[1], h);
}

// ---------------------------------------------------------------------------------------- launchers
template <class H, int CHUNK>
static hipError_t sim_family(int op, const SimLaunch& L) {
    const uint64_t local = L.cfg.peer_end - L.cfg.peer_begin;
    if (op == 0) {
        if (!local) return hipSuccess;
        const size_t lds = sim_build_lds((uint32_t)((L.cfg.m_bits + 31) / 32), L.cfg.capacity);
        auto kern = L.or_mode == 0 ? k_sim_build_claims<H, CHUNK, 0>
                                   : L.or_mode == 2 ? k_sim_build_claims<H, CHUNK, 2> : k_sim_build_claims<H, CHUNK, 1>;
        hipLaunchKernelGGL(kern, dim3((uint32_t)((local + 3) / 4)), dim3(256), lds, L.stream, L.cfg, L.round, L.ublob,
                           L.uoff, L.bits, L.out, L.slots, L.work);
    } else {
        if (!L.n_in) return hipSuccess;
        constexpr bool dma = H::kind == DSY_MD5 || H::kind == DSY_SHA1;
        static const uint32_t nw = getenv("DSY_SIM_WAVES") && atoi(getenv("DSY_SIM_WAVES")) == 8 ? kSimRespWaves : 4;
        const uint32_t nwords = (uint32_t)((L.cfg.m_bits + 31) / 32);
        if (nw == 4)
            hipLaunchKernelGGL((k_sim_respond<H, CHUNK, 4>), dim3((uint32_t)((L.n_in + 3) / 4)), dim3(256),
                               sim_respond_lds(nwords, dma, 4), L.stream, L.cfg, L.ublob, L.uoff, L.bits, L.in, L.n_in,
                               L.out, L.slots, L.tested, L.work);
        else
            hipLaunchKernelGGL((k_sim_respond<H, CHUNK, kSimRespWaves>), dim3((uint32_t)((L.n_in + kSimRespWaves - 1) / kSimRespWaves)),
                               dim3(64 * kSimRespWaves), sim_respond_lds(nwords, dma, kSimRespWaves), L.stream, L.cfg,
                               L.ublob, L.uoff, L.bits, L.in, L.n_in, L.out, L.slots, L.tested, L.work);
    }
    return hipGetLastError();
}

hipError_t launch_sim(int op, const SimLaunch& L) {
    const dsy_sim_config& c = L.cfg;
    const uint64_t local = c.peer_end - c.peer_begin;
    switch (op) {
        case kSimSeed:
            if (local) hipLaunchKernelGGL(k_sim_seed, dim3((uint32_t)((local + 255) / 256)), dim3(256), 0, L.stream, c, L.bits, L.initial);
            return hipGetLastError();
        case kSimClaimCounts:
            if (local) hipLaunchKernelGGL(k_sim_claim_counts, dim3((uint32_t)((local + 255) / 256)), dim3(256), 0, L.stream, c, L.round, L.counts);
            return hipGetLastError();
        case kSimClaimSlots:
            if (local) hipLaunchKernelGGL(k_sim_claim_slots, dim3((uint32_t)((local + 255) / 256)), dim3(256), 0, L.stream, c, L.round, L.cursor, L.slots);
            return hipGetLastError();
        case kSimRespSlots:
            if (L.n_in) hipLaunchKernelGGL(k_sim_resp_slots, dim3((uint32_t)((L.n_in + 255) / 256)), dim3(256), 0, L.stream, c, L.in, L.n_in, L.cursor, L.slots);
            return hipGetLastError();
        case kSimRespCounts:
            if (L.n_in) hipLaunchKernelGGL(k_sim_resp_counts, dim3((uint32_t)((L.n_in + 255) / 256)), dim3(256), 0, L.stream, c, L.in, L.n_in, L.counts);
            return hipGetLastError();
        case kSimMerge:
            if (L.n_in) hipLaunchKernelGGL(k_sim_merge, dim3((uint32_t)((L.n_in + 255) / 256)), dim3(256), 0, L.stream, c, L.bits, L.in, L.n_in, L.counts);
            return hipGetLastError();
        case kSimClaimMatrix:
            if (c.n_peers && L.n_rounds)
                hipLaunchKernelGGL(k_sim_claim_matrix, dim3((uint32_t)((c.n_peers + 255) / 256), L.n_rounds), dim3(256), 0,
                                   L.stream, c, L.round, L.n_ranks, L.counts);
            return hipGetLastError();
        case kSimCursorInit:
            hipLaunchKernelGGL(k_sim_cursor_init, dim3(1), dim3(kSimMaxRanks), 0, L.stream, L.cursor_init, L.cursor);
            return hipGetLastError();
        case kSimStats:
            if (local) hipLaunchKernelGGL(k_sim_stats, dim3((uint32_t)((local + 255) / 256)), dim3(256), 0, L.stream, c, L.bits, L.stats);
            return hipGetLastError();
        case kSimBuild:
        case kSimRespond: {
            const int o = op == kSimBuild ? 0 : 1;
            switch (c.hash_kind) {
                case DSY_MD5: return c.chunk_bytes == 2 ? sim_family<Md5, 2>(o, L) : sim_family<Md5, 4>(o, L);
                case DSY_SHA1: return c.chunk_bytes == 2 ? sim_family<Sha1, 2>(o, L) : sim_family<Sha1, 4>(o, L);
                default: return c.chunk_bytes == 2 ? sim_family<Sha256, 2>(o, L) : sim_family<Sha256, 4>(o, L);
            }
        }
    }
    return hipErrorInvalidValue;
}

}  // namespace dsy

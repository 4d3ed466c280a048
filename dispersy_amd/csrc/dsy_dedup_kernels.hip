// Duplicate check of received sync packets as a GPU hash join:
// `_is_duplicate_sync_message` (dispersy.py:831-918) looks every received message up by
// `SELECT packet, undone FROM sync WHERE community = ? AND member = ? AND global_time = ?` and compares packets.
// Here the store carries an open-addressing table over (member, global_time) -> row, and one wave per received
// message probes 64 slots per step (ballot of matches and empty slots) and compares the two packets 64 bytes per
// step (ballot of the first differing byte):
//   k_dup_insert   one lane per row: claim the first free slot from the key's hash (keys are unique: the table
//                  mirrors UNIQUE(community, member, global_time), dispersydatabase.py:53-64)
//   k_dup_rehash   growth: every occupied slot of the old table into the new one (tombstones dropped)
//   k_dup_erase    DELETE: the deleted rows' slots become tombstones
//   k_dup_check    verdict per message (DSY_DUP_*), with the stored row
//   k_rec_scatter  dsy_store_replace: point rows at their replacement packets in the line copy
#include "dsy_kernels.h"

namespace dsy {

static constexpr uint64_t kDupEmpty = ~0ull;

__device__ __forceinline__ uint64_t dup_hash(uint64_t member, uint64_t gt) {
    uint64_t x = member * 0x9e3779b97f4a7c15ull ^ (gt + 0x632be59bd9b4e019ull);
    x ^= x >> 31; x *= 0xbf58476d1ce4e5b9ull; x ^= x >> 29; x *= 0x94d049bb133111ebull; x ^= x >> 32;
    return x;
}

// (tombstoned slots are never reused: a rehash on growth drops them)
__device__ __forceinline__ void dup_put(DupSlot* __restrict__ tab, uint64_t mask, uint64_t member, uint64_t gt,
                                        uint64_t row) {
    uint64_t h = dup_hash(member, gt) & mask;
    for (;;) {
        if (atomicCAS((unsigned long long*)&tab[h].row, (unsigned long long)kDupEmpty, (unsigned long long)row) ==
            (unsigned long long)kDupEmpty) {
            tab[h].member = member;
            tab[h].gt = gt;
            return;
        }
        h = (h + 1) & mask;
    }
}

__global__ void __launch_bounds__(256) k_dup_insert(const uint64_t* __restrict__ member, const uint64_t* __restrict__ gt,
                                                    uint64_t first_row, uint64_t n, DupSlot* __restrict__ tab,
                                                    uint64_t mask, DupKey* __restrict__ keys) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t m = member[i], g = gt[i];
    keys[first_row + i] = DupKey{m, g};
    dup_put(tab, mask, m, g, first_row + i);
}

// DELETE FROM sync (GlobalTimePruning, sequence-number conflicts, LastSync history): the deleted rows' slots become
// tombstones, so a later (member, global_time) lookup no longer finds them (dispersy.py:868 sees no row after the
// DELETE).  One lane per deleted row walks its key's probe chain to the slot holding that row.
__global__ void __launch_bounds__(256) k_dup_erase(const uint64_t* __restrict__ rows, const uint64_t* __restrict__ live_row,
                                                   uint64_t a, uint64_t k, const DupKey* __restrict__ keys,
                                                   DupSlot* __restrict__ tab, uint64_t mask) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= k) return;
    const uint64_t row = rows ? rows[i] : (live_row ? live_row[a + i] : a + i);
    const DupKey key = keys[row];
    uint64_t h = dup_hash(key.member, key.gt) & mask;
    for (uint64_t step = 0; step <= mask; ++step) {
        const uint64_t r = tab[h].row;
        if (r == kDupEmpty) return;  // not in the table (deleted before)
        if (r == row) {
            tab[h].row = kDupTomb;
            return;
        }
        h = (h + 1) & mask;
    }
}

__global__ void __launch_bounds__(256) k_dup_rehash(const DupSlot* __restrict__ old, uint64_t old_cap,
                                                    DupSlot* __restrict__ tab, uint64_t mask) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < old_cap && old[i].row != kDupEmpty && old[i].row != kDupTomb)
        dup_put(tab, mask, old[i].member, old[i].gt, old[i].row);
}

// One wave per received message.
__global__ void __launch_bounds__(256) k_dup_check(const DupSlot* __restrict__ tab, uint64_t mask,
                                                   const uint8_t* __restrict__ lines, const RowRec* __restrict__ rec,
                                                   const uint64_t* __restrict__ member, const uint64_t* __restrict__ gt,
                                                   const uint8_t* __restrict__ blob, const uint64_t* __restrict__ offsets,
                                                   const uint32_t* __restrict__ sig_len, uint64_t m,
                                                   uint8_t* __restrict__ verdict, uint64_t* __restrict__ out_row) {
    const uint64_t j = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    if (j >= m) return;  // wave-uniform
    const uint64_t mj = member[j], gj = gt[j];
    // probe 64 consecutive slots per step: the key is present iff a match comes before the first empty slot
    uint64_t row = kDupEmpty;
    const uint64_t h0 = dup_hash(mj, gj);
    for (uint64_t base = 0; base <= mask; base += 64) {
        const DupSlot sl = tab[(h0 + base + lane) & mask];
        const bool empty = sl.row == kDupEmpty;
        const uint64_t hit = __ballot(!empty && sl.row != kDupTomb && sl.member == mj && sl.gt == gj);
        const uint64_t gap = __ballot(empty);
        if (hit && (!gap || __ffsll((unsigned long long)hit) < __ffsll((unsigned long long)gap))) {
            row = __shfl(sl.row, __ffsll((unsigned long long)hit) - 1, 64);
            break;
        }
        if (gap) break;
    }
    if (row == kDupEmpty) {
        if (lane == 0) {
            verdict[j] = DSY_DUP_NEW;
            out_row[j] = kDupEmpty;
        }
        return;
    }
    const RowRec rr = rec[row];
    const uint8_t* have = lines + rr.off;
    const uint8_t* mine = blob + offsets[j];
    const uint64_t lh = rr.len, ln = offsets[j + 1] - offsets[j], mn = lh < ln ? lh : ln;
    // first differing byte (mn when none)
    uint64_t fd = mn;
    for (uint64_t p0 = 0; p0 < mn; p0 += 64) {
        const uint64_t p = p0 + lane;
        const uint64_t d = __ballot(p < mn && have[p] != mine[p]);
        if (d) {
            fd = p0 + __ffsll((unsigned long long)d) - 1;
            break;
        }
    }
    if (lane == 0) {
        uint8_t v;
        if (fd == mn && lh == ln) {
            v = DSY_DUP_EXACT;  // binary duplicate (dispersy.py:872)
        } else {
            // have_packet[:signature_length] == message.packet[:signature_length]   (dispersy.py:893)
            const uint64_t sl = sig_len[j];
            const uint64_t ah = lh < sl ? lh : sl, an = ln < sl ? ln : sl;
            if (ah == an && fd >= ah) {
                // have_packet < message.packet: bytewise, a proper prefix is smaller   (dispersy.py:901)
                const bool less = fd < mn ? have[fd] < mine[fd] : lh < ln;
                v = less ? DSY_DUP_REPLACE : DSY_DUP_KEEP;
            } else {
                v = DSY_DUP_TRIPLET;  // same (community, member, global_time), different message (dispersy.py:910)
            }
        }
        verdict[j] = v;
        out_row[j] = row;
    }
}

__global__ void __launch_bounds__(256) k_rec_scatter(RowRec* __restrict__ rec, const uint64_t* __restrict__ rows,
                                                     const RowRec* __restrict__ src, uint64_t k) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < k) rec[rows[i]] = src[i];
}

static uint32_t grid_of(uint64_t lanes) { return (uint32_t)((lanes + 255) / 256); }

hipError_t launch_dup_insert(const uint64_t* member, const uint64_t* gt, uint64_t first_row, uint64_t n, DupSlot* tab,
                             uint64_t mask, DupKey* keys, hipStream_t stream) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_dup_insert, dim3(grid_of(n)), dim3(256), 0, stream, member, gt, first_row, n, tab, mask, keys);
    return hipGetLastError();
}

hipError_t launch_dup_erase(const uint64_t* rows, const uint64_t* live_row, uint64_t a, uint64_t k, const DupKey* keys,
                            DupSlot* tab, uint64_t mask, hipStream_t stream) {
    if (!k) return hipSuccess;
    hipLaunchKernelGGL(k_dup_erase, dim3(grid_of(k)), dim3(256), 0, stream, rows, live_row, a, k, keys, tab, mask);
    return hipGetLastError();
}

hipError_t launch_dup_rehash(const DupSlot* old, uint64_t old_cap, DupSlot* tab, uint64_t mask, hipStream_t stream) {
    if (!old_cap) return hipSuccess;
    hipLaunchKernelGGL(k_dup_rehash, dim3(grid_of(old_cap)), dim3(256), 0, stream, old, old_cap, tab, mask);
    return hipGetLastError();
}

hipError_t launch_dup_check(const DupSlot* tab, uint64_t mask, const uint8_t* lines, const RowRec* rec,
                            const uint64_t* member, const uint64_t* gt, const uint8_t* blob, const uint64_t* offsets,
                            const uint32_t* sig_len, uint64_t m, uint8_t* verdict, uint64_t* out_row,
                            hipStream_t stream) {
    if (!m) return hipSuccess;
    hipLaunchKernelGGL(k_dup_check, dim3(grid_of(m * 64)), dim3(256), 0, stream, tab, mask, lines, rec, member, gt,
                       blob, offsets, sig_len, m, verdict, out_row);
    return hipGetLastError();
}

hipError_t launch_rec_scatter(RowRec* rec, const uint64_t* rows, const RowRec* src, uint64_t k, hipStream_t stream) {
    if (!k) return hipSuccess;
    hipLaunchKernelGGL(k_rec_scatter, dim3(grid_of(k)), dim3(256), 0, stream, rec, rows, src, k);
    return hipGetLastError();
}

}  // namespace dsy

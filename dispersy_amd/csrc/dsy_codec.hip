// dsy_codec.hip -- the introduction-request sync block on the wire (conversion.py:712-730 encode, :732-799 decode),
// batched on the host side of the C-ABI: a receive batch of claims is decoded straight into dsy_request records and
// 4-byte-aligned filter words that dsy_sync_respond consumes, with the reference's validation (its DropPacket
// reasons become per-item status codes).  Layout (struct '>QQHHBH', conversion.py:193): time_low u64, time_high
// u64, modulo u16, offset u16, functions u8, size u16 (bits), then the 1-byte prefix, then size/8 filter bytes that
// run to the end of the payload.  No device work: this is byte parsing at PCIe ingress.
#include <hip/hip_runtime.h>

#include <cstring>

#include "dsy_kernels.h"

namespace {

uint64_t be64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
    return v;
}
uint32_t be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
void put_be64(uint8_t* p, uint64_t v) {
    for (int i = 7; i >= 0; --i, v >>= 8) p[i] = (uint8_t)v;
}
void put_be16(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}

// bloomfilter.py:134-156 -- 0 when (m, k) needs more than 512 digest bits (the constructor asserts)
int family_of(uint64_t m, uint32_t k, int32_t* kind, uint32_t* chunk) {
    const uint32_t c = m >= (1ull << 31) ? 8 : (m >= (1ull << 15) ? 4 : 2);
    const uint64_t bits = (uint64_t)c * k * 8;
    if (bits > 512) return 0;
    *kind = bits > 384 ? DSY_SHA512 : bits > 256 ? DSY_SHA384 : bits > 160 ? DSY_SHA256 : bits > 128 ? DSY_SHA1 : DSY_MD5;
    *chunk = c;
    return 1;
}

constexpr uint64_t kMaxGt = 0x7fffffffffffffffull;

}  // namespace

extern "C" {

int dsy_sync_decode(const uint8_t* blob, const uint64_t* offsets, uint32_t n, uint64_t responder_global_time,
                    dsy_request* out_reqs, uint8_t* out_filters, uint64_t filters_cap, uint64_t* out_filters_len,
                    int32_t* out_status) {
    if ((n && (!blob || !offsets || !out_reqs || !out_status)) || !out_filters_len) return DSY_EINVAL;
    uint64_t at = 0;
    for (uint32_t i = 0; i < n; ++i) {
        dsy_request& q = out_reqs[i];
        std::memset(&q, 0, sizeof q);
        const uint8_t* d = blob + offsets[i];
        const uint64_t len = offsets[i + 1] - offsets[i];
        int32_t st = DSY_DROP_OK;
        // conversion.py:763-789, in the reference's order
        if (len < DSY_SYNC_HEADER) {
            st = DSY_DROP_SIZE;
        } else {
            const uint64_t time_low = be64(d), time_high = be64(d + 8);
            const uint32_t modulo = be16(d + 16), off = be16(d + 18), functions = d[20], size = be16(d + 21);
            const uint8_t prefix = d[23];
            const uint64_t length = (size + 7) / 8;
            int32_t kind = 0;
            uint32_t chunk = 0;
            if (!(time_low > 0)) st = DSY_DROP_TIME_LOW;
            else if (!(time_high == 0 || time_low <= time_high)) st = DSY_DROP_TIME_HIGH;
            else if (!(0 < modulo)) st = DSY_DROP_MODULO;
            else if (!(off < modulo)) st = DSY_DROP_OFFSET;
            else if (!(0 < functions)) st = DSY_DROP_FUNCTIONS;
            else if (!(0 < size)) st = DSY_DROP_SIZE_VALUE;
            else if (size % 8) st = DSY_DROP_SIZE_MULT8;
            else if (length != len - DSY_SYNC_HEADER) st = DSY_DROP_LENGTH;
            // BloomFilter(bytes, functions, prefix) (:791) asserts 0 < k <= m and a <= 512-bit digest
            // (bloomfilter.py:129, :144): an AssertionError, not a DropPacket, and nothing on the decode path catches it
            else if (functions > size || !family_of(size, functions, &kind, &chunk)) st = DSY_DECODE_ASSERT;
            if (st == DSY_DROP_OK) {
                const uint64_t words = (size + 31) / 32;
                if (at + words * 4 > filters_cap) {
                    *out_filters_len = at + words * 4;  // what the batch would need so far
                    return DSY_ECAPACITY;
                }
                std::memcpy(out_filters + at, d + DSY_SYNC_HEADER, length);
                std::memset(out_filters + at + length, 0, words * 4 - length);
                q.time_low = time_low;
                q.time_high = time_high;
                if (responder_global_time) {  // community.py:2545-2553
                    if (!q.time_high) q.time_high = responder_global_time;
                    if (q.time_low > kMaxGt) q.time_low = kMaxGt;
                    if (q.time_high > kMaxGt) q.time_high = kMaxGt;
                }
                q.modulo = modulo;
                q.offset = off;
                q.filter_offset = at;
                q.m_bits = size;
                q.k = functions;
                q.hash_kind = kind;
                q.chunk_bytes = chunk;
                q.prefix_len = 1;
                q.prefix[0] = prefix;
                at += words * 4;
            }
        }
        out_status[i] = st;
    }
    *out_filters_len = at;
    return DSY_OK;
}

int dsy_sync_encode(const dsy_request* reqs, uint32_t n, const uint8_t* filters, uint8_t* out, uint64_t out_cap,
                    uint64_t* out_offsets) {
    if ((n && (!reqs || !filters || !out)) || !out_offsets) return DSY_EINVAL;
    uint64_t at = 0;
    out_offsets[0] = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const dsy_request& q = reqs[i];
        // conversion.py:723-726 asserts and the '>QQHHBH' field widths (struct.error in the reference); like the
        // reference, the encoder does not check what only the decoder validates (time_low > 0, offset < modulo, ...)
        if (q.m_bits == 0 || q.m_bits % 8 || q.m_bits > 0xffff || q.k == 0 || q.k > 255 || q.prefix_len != 1 ||
            q.modulo > 0xffff || q.offset > 0xffff)
            return DSY_EINVAL;
        const uint64_t length = q.m_bits / 8, need = DSY_SYNC_HEADER + length;
        if (at + need > out_cap) {
            out_offsets[n] = at + need;
            return DSY_ECAPACITY;
        }
        uint8_t* d = out + at;
        put_be64(d, q.time_low);
        put_be64(d + 8, q.time_high);
        put_be16(d + 16, q.modulo);
        put_be16(d + 18, q.offset);
        d[20] = (uint8_t)q.k;
        put_be16(d + 21, (uint32_t)q.m_bits);
        d[23] = q.prefix[0];
        std::memcpy(d + DSY_SYNC_HEADER, filters + q.filter_offset, length);
        at += need;
        out_offsets[i + 1] = at;
    }
    return DSY_OK;
}

}  // extern "C"

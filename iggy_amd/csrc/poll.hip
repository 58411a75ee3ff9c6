// poll.hip — poll-side decode (core/common/src/types/message/polled_messages.rs:95-150,
// core/binary_protocol/src/responses/messages/poll_messages.rs:132-165): after a
// record's frames are walked on the device, expand each frame into a resolved
// message descriptor (absolute offset / timestamps, zero-copy payload ranges).
#include "codec_common.hpp"

namespace iggy {

__global__ __launch_bounds__(256) void k_poll_fill(const uint8_t *buf, uint64_t rec_off,
                                                   const uint64_t *pos, uint64_t nf,
                                                   iggy_polled_message *out) {
    const uint8_t *rec = buf + rec_off;
    const uint64_t base_offset = ld64_any(rec + 8);
    const uint64_t base_ts = ld64_any(rec + 16);
    const uint64_t origin = ld64_any(rec + 24);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nf;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t p = pos[i];
        const uint8_t *f = rec + kHdr + p;
        iggy_polled_message m;
        m.checksum = ld64_any(f);
        m.id_lo = ld64_any(f + 8);
        m.id_hi = ld64_any(f + 16);
        m.offset = base_offset + ld32_any(f + 24);           // wrapping, as in release Rust
        m.timestamp = base_ts;                               // flat per batch
        m.origin_timestamp = origin + ld32_any(f + 28);
        m.user_headers_length = ld32_any(f + 32);
        m.payload_length = ld32_any(f + 36);
        m.payload_pos = rec_off + kHdr + p + kFrameHdr;
        m.user_headers_pos = m.payload_pos + m.payload_length;
        m._pad = 0;
        out[i] = m;
    }
}

// Context-creation probe: does global_load_lds_dwordx4 deliver the 16 bytes of
// an unaligned source address? (gfx950 supports unaligned global loads; the
// uniform decode kernel stages frames at arbitrary offsets only if this holds.)
__global__ void k_probe_glds_unaligned(const uint8_t *src, uint32_t *ok) {
    extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
    const int lane = threadIdx.x & 63;
    const uint32_t offs[4] = {1, 3, 8, 13};
#pragma unroll
    for (int k = 0; k < 4; ++k) glds16(src + offs[k] + 16 * lane, 1024u * k);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    bool good = true;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint4 a = *(const uint4 *)(sm + 1024 * k + 16 * lane);
        const uint4 b = ld128_any(src + offs[k] + 16 * lane);
        good &= a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w;
    }
    const uint64_t bad = __ballot(!good);
    if (lane == 0) *ok = bad ? 2u : 1u;
}

}  // namespace iggy

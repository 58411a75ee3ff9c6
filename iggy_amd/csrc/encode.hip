// encode.hip — SendMessagesEncoder::encode, batch section
// (core/binary_protocol/src/requests/messages/send_messages.rs:89-181) and its
// server twin SendMessagesOwned::from_messages
// (core/server_common/src/send_messages.rs:104-168), on struct-of-arrays input.
//
//  k_enc_prep   : per 2048-message tile: local exclusive prefix of payload and
//                 user-header lengths, tile sums, tile minimum origin timestamp.
//  k_enc_scan   : one WG: tile offsets (the wavefront prefix scan that places
//                 variable-size frames), batch minimum origin timestamp, length.
//  k_enc_frames : one wave per frame, frames in any order:
//                 writes the 48-B header + payload + user headers with coalesced
//                 16-B stores (unaligned: gfx950 unaligned-buffer-access) and
//                 hashes the same bytes in registers (wave-cooperative XXH3:
//                 lane l owns stripe words 2l, 2l+1 of each 1 KiB block), then
//                 backpatches the frame checksum (send_messages.rs:162-163).
//  then k_bsum_blocks / k_bsum_chain (batch_checksum.hip) over the frame
//  checksums and k_enc_finish (header, error precedence).
#include "codec_common.hpp"

namespace iggy {

constexpr uint32_t kEncTile = 2048;

struct EncScratch {
    uint64_t *pl_local;   // [n] exclusive prefix of payload lengths inside the tile
    uint64_t *uh_local;   // [n]
    uint64_t *tile_pl;    // [ntiles] tile sums -> tile offsets after the scan
    uint64_t *tile_uh;    // [ntiles]
    uint64_t *tile_min;   // [ntiles] minimum origin timestamp
    uint64_t *cs;         // [n] frame checksums
    uint64_t *misc;       // [8]: 0 min origin, 1 blob bytes, 2 ts-error (~index, max), 3 n
    iggy_batch_header *hdr;  // header being built
};

__global__ __launch_bounds__(256) void k_enc_prep(iggy_raw_messages m, EncScratch es) {
    __shared__ uint64_t s_pl[256], s_uh[256], s_min[256];
    const uint64_t n = m.count;
    const uint64_t t = blockIdx.x;
    const uint64_t base = t * kEncTile;
    const uint32_t tid = threadIdx.x;
    // 8 consecutive messages per thread
    uint64_t pl[8], uh[8], mn = ~0ull;
    uint64_t spl = 0, suh = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint64_t i = base + tid * 8 + k;
        pl[k] = (i < n) ? m.payload_lengths[i] : 0;
        uh[k] = (i < n && m.user_headers_lengths) ? m.user_headers_lengths[i] : 0;
        if (i < n) mn = min(mn, m.origin_timestamps[i]);
        spl += pl[k];
        suh += uh[k];
    }
    s_pl[tid] = spl;
    s_uh[tid] = suh;
    s_min[tid] = mn;
    __syncthreads();
    // exclusive scan of the 256 thread sums (Hillis-Steele in LDS)
    for (uint32_t d = 1; d < 256; d <<= 1) {
        const uint64_t a = tid >= d ? s_pl[tid - d] : 0;
        const uint64_t b = tid >= d ? s_uh[tid - d] : 0;
        const uint64_t c = tid >= d ? s_min[tid - d] : ~0ull;
        __syncthreads();
        s_pl[tid] += a;
        s_uh[tid] += b;
        s_min[tid] = min(s_min[tid], c);
        __syncthreads();
    }
    uint64_t opl = s_pl[tid] - spl, ouh = s_uh[tid] - suh;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint64_t i = base + tid * 8 + k;
        if (i < n) {
            es.pl_local[i] = opl;
            es.uh_local[i] = ouh;
        }
        opl += pl[k];
        ouh += uh[k];
    }
    if (tid == 255) {
        es.tile_pl[t] = s_pl[255];
        es.tile_uh[t] = s_uh[255];
        es.tile_min[t] = s_min[255];
    }
}

__global__ __launch_bounds__(256) void k_enc_scan(uint64_t ntiles, uint64_t n, uint64_t partition_id,
                                                  EncScratch es) {
    __shared__ uint64_t s_pl[256], s_uh[256], s_min[256];
    __shared__ uint64_t carry_pl, carry_uh, carry_min;
    const uint32_t tid = threadIdx.x;
    if (tid == 0) { carry_pl = 0; carry_uh = 0; carry_min = ~0ull; }
    __syncthreads();
    for (uint64_t t0 = 0; t0 < ntiles; t0 += 256) {
        const uint64_t t = t0 + tid;
        const uint64_t vpl = t < ntiles ? es.tile_pl[t] : 0;
        const uint64_t vuh = t < ntiles ? es.tile_uh[t] : 0;
        const uint64_t vmn = t < ntiles ? es.tile_min[t] : ~0ull;
        s_pl[tid] = vpl; s_uh[tid] = vuh; s_min[tid] = vmn;
        __syncthreads();
        for (uint32_t d = 1; d < 256; d <<= 1) {
            const uint64_t a = tid >= d ? s_pl[tid - d] : 0;
            const uint64_t b = tid >= d ? s_uh[tid - d] : 0;
            __syncthreads();
            s_pl[tid] += a;
            s_uh[tid] += b;
            __syncthreads();
        }
        if (t < ntiles) {
            es.tile_pl[t] = carry_pl + s_pl[tid] - vpl;
            es.tile_uh[t] = carry_uh + s_uh[tid] - vuh;
        }
        // min reduction
        for (uint32_t d = 128; d > 0; d >>= 1) {
            if (tid < d) s_min[tid] = min(s_min[tid], s_min[tid + d]);
            __syncthreads();
        }
        if (tid == 0) {
            carry_pl += s_pl[255];
            carry_uh += s_uh[255];
            carry_min = min(carry_min, s_min[0]);
        }
        __syncthreads();
    }
    if (tid == 0) {
        const uint64_t origin = (n == 0) ? 0 : carry_min;
        es.misc[0] = origin;
        es.misc[1] = 48 * n + carry_pl + carry_uh;
        es.misc[2] = 0;
        es.misc[3] = n;
        iggy_batch_header h{};
        h.partition_id = partition_id;
        h.base_offset = 0;
        h.base_timestamp = 0;
        h.origin_timestamp = origin;
        h.batch_length = 256 + es.misc[1];
        h.batch_checksum = 0;
        h.message_count = (uint32_t)n;
        *es.hdr = h;
    }
}

// bytes [s, s+8) of the hashed stream H(40) || P(pl) || U(uh), zero past the end
struct FrameStream {
    uint64_t h[5];
    const uint8_t *P, *U;
    uint64_t pl, uh, L;
    __device__ __forceinline__ uint8_t byte(uint64_t s) const {
        if (s < 40) return (uint8_t)(h[s >> 3] >> (8 * (s & 7)));
        if (s < 40 + pl) return P[s - 40];
        if (s < L) return U[s - 40 - pl];
        return 0;
    }
    __device__ __forceinline__ uint64_t get8(uint64_t s) const {
        if (s + 8 <= 40 && (s & 7) == 0) return h[s >> 3];
        if (s >= 40 && s + 8 <= 40 + pl) return ld64_any(P + (s - 40));
        if (s >= 40 + pl && s + 8 <= L) return ld64_any(U + (s - 40 - pl));
        uint64_t v = 0;
        for (int k = 7; k >= 0; --k) v = (v << 8) | byte(s + k);
        return v;
    }
};

// short inputs (40..240 B): XXH3 mid-size paths over a FrameStream
__device__ inline uint64_t xxh3_short_stream(const FrameStream &fs) {
    const uint64_t L = fs.L;
    auto mix16 = [&](uint64_t off, uint64_t s0, uint64_t s1) {
        return fold64(fs.get8(off) ^ s0, fs.get8(off + 8) ^ s1);
    };
    if (L <= 128) {
        uint64_t acc = L * P64_1;
        if (L > 32) {
            if (L > 64) {
                if (L > 96) {
                    acc += mix16(48, Secret::w(96), Secret::w(104));
                    acc += mix16(L - 64, Secret::w(112), Secret::w(120));
                }
                acc += mix16(32, Secret::w(64), Secret::w(72));
                acc += mix16(L - 48, Secret::w(80), Secret::w(88));
            }
            acc += mix16(16, Secret::w(32), Secret::w(40));
            acc += mix16(L - 32, Secret::w(48), Secret::w(56));
        }
        acc += mix16(0, Secret::w(0), Secret::w(8));
        acc += mix16(L - 16, Secret::w(16), Secret::w(24));
        return avalanche(acc);
    }
    uint64_t acc = L * P64_1;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += mix16(16 * i, Secret::w(16 * i), Secret::w(16 * i + 8));
    acc = avalanche(acc);
    const uint32_t rounds = (uint32_t)(L / 16);
#pragma unroll
    for (int i = 8; i < 15; ++i)
        if ((uint32_t)i < rounds)
            acc += mix16(16 * i, Secret::w(16 * (i - 8) + 3), Secret::w(16 * (i - 8) + 11));
    acc += mix16(L - 16, Secret::w(119), Secret::w(127));
    return avalanche(acc);
}

__global__ __launch_bounds__(256) void k_enc_frames(iggy_raw_messages m, EncScratch es,
                                                    uint8_t *out) {
    const int lane = threadIdx.x & 63;
    const uint64_t n = m.count;
    const uint64_t origin = es.misc[0];
    const uint64_t wid = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    // lanes with equal (lane & 3) own accumulators j0 = 2(lane&3), j1 = j0 + 1
    const int q = lane & 3, j0 = 2 * q, j1 = j0 + 1;
    const uint64_t sec0 = kSecretW8[(lane >> 2) + j0];
    const uint64_t sec1 = kSecretW8[(lane >> 2) + j1];
    const uint64_t key0 = kSecretW8[16 + j0], key1 = kSecretW8[16 + j1];
    for (uint64_t i = wid; i < n; i += nwaves) {
        const uint64_t t = i / kEncTile;
        const uint64_t po = es.tile_pl[t] + es.pl_local[i];
        const uint64_t uo = es.tile_uh[t] + es.uh_local[i];
        FrameStream fs;
        fs.pl = m.payload_lengths[i];
        fs.uh = m.user_headers_lengths ? m.user_headers_lengths[i] : 0;
        fs.L = 40 + fs.pl + fs.uh;
        fs.P = m.payloads + po;
        fs.U = m.user_headers ? m.user_headers + uo : m.payloads;
        const uint64_t ots = m.origin_timestamps[i];
        const uint64_t delta = ots - origin;
        if (delta > IGGY_MAX_TIMESTAMP_DELTA_MICROS && lane == 0)
            atomicMax((unsigned long long *)&es.misc[2], (unsigned long long)~i);
        fs.h[0] = m.ids[2 * i];
        fs.h[1] = m.ids[2 * i + 1];
        fs.h[2] = (i & 0xFFFFFFFFull) | ((delta & 0xFFFFFFFFull) << 32);
        fs.h[3] = fs.uh | (fs.pl << 32);
        fs.h[4] = 0;
        uint8_t *dst = out + 256 + 48 * i + po + uo;  // frame start
        const uint64_t L = fs.L;
        const bool is_long = L > 240;
        uint64_t nbF = 0, Kreg = 0;
        if (is_long) {
            nbF = (L - 1) / 1024;
            const uint64_t ns = ((L - 1) - 1024 * nbF) / 64;
            Kreg = 8 * (16 * nbF + ns);
        }
        uint64_t a0 = kAccInit[j0], a1 = kAccInit[j1];
        const uint64_t nblk = (L + 1023) / 1024;
        for (uint64_t b = 0; b < nblk; ++b) {
            const uint64_t s0 = 1024 * b + 16 * (uint64_t)lane;
            uint64_t w0 = 0, w1 = 0;
            if (s0 < L) {
                w0 = fs.get8(s0);
                w1 = fs.get8(s0 + 8);
                uint8_t *d = dst + 8 + s0;
                if (s0 + 16 <= L) {
                    st128_any(d, make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1,
                                            (uint32_t)(w1 >> 32)));
                } else {
                    const uint32_t rem = (uint32_t)(L - s0);
                    for (uint32_t k = 0; k < rem; ++k)
                        d[k] = (uint8_t)((k < 8 ? w0 : w1) >> (8 * (k & 7)));
                }
            }
            if (is_long) {
                const uint64_t k0 = s0 >> 3;  // stream word index of w0
                uint64_t A0 = 0, A1 = 0;      // contributions to acc[j0], acc[j1]
                if (k0 < Kreg) { A0 += mul32x32(w0 ^ sec0); A1 += w0; }
                if (k0 + 1 < Kreg) { A1 += mul32x32(w1 ^ sec1); A0 += w1; }
                A0 += __shfl_xor(A0, 4);  A1 += __shfl_xor(A1, 4);
                A0 += __shfl_xor(A0, 8);  A1 += __shfl_xor(A1, 8);
                A0 += __shfl_xor(A0, 16); A1 += __shfl_xor(A1, 16);
                A0 += __shfl_xor(A0, 32); A1 += __shfl_xor(A1, 32);
                a0 += A0;
                a1 += A1;
                if (b < nbF) {
                    a0 = scramble1(a0, key0);
                    a1 = scramble1(a1, key1);
                }
            }
        }
        uint64_t hsh;
        if (is_long) {
            // last stripe: stream words at L-64+8j, lane j < 8
            const int j = lane & 7;
            const uint64_t v = fs.get8(L - 64 + 8 * j);
            const uint64_t A = mul32x32(v ^ kSecretLast[j]);  // -> acc[j]
            const uint64_t B = v;                              // -> acc[j^1]
            a0 += __shfl(A, j0) + __shfl(B, j1);
            a1 += __shfl(A, j1) + __shfl(B, j0);
            uint64_t acc[8];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                acc[2 * k] = __shfl(a0, k);
                acc[2 * k + 1] = __shfl(a1, k);
            }
            uint64_t r = L * P64_1;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                r += fold64(acc[2 * k] ^ Secret::w(11 + 16 * k), acc[2 * k + 1] ^ Secret::w(19 + 16 * k));
            hsh = avalanche(r);
        } else {
            hsh = (lane == 0) ? xxh3_short_stream(fs) : 0;
        }
        if (lane == 0) {
            st64_any(dst, hsh);
            es.cs[i] = hsh;
        }
    }
}

// error precedence (send_messages.rs:131-174) and the 256-B header
__global__ void k_enc_finish(iggy_raw_messages m, EncScratch es, uint64_t partition_id,
                             const uint64_t *checksum, uint8_t *out, iggy_encode_result *res) {
    const int t = threadIdx.x;
    iggy_batch_header h = *es.hdr;
    h.batch_checksum = *checksum;
    const uint64_t ts_enc = es.misc[2];
    uint32_t kind = IGGY_OK;
    uint64_t a = 0, b = 0;
    if (ts_enc) {
        kind = IGGY_ERR_INVALID_TIMESTAMP_DELTA;
        a = m.origin_timestamps[~ts_enc] - es.misc[0];
    } else if (partition_id == 0 && h.batch_length > 0xFFFFFFFFull) {
        kind = IGGY_ERR_PAYLOAD_TOO_LARGE;
        a = h.batch_length;
        b = 0xFFFFFFFFull;
    }
    // header bytes: 64 threads x 4 bytes
    {
        const uint32_t off = 4 * t;
        uint32_t w = 0;
        if (off < 48) {
            const uint64_t f[6] = {h.partition_id, h.base_offset, h.base_timestamp,
                                   h.origin_timestamp, h.batch_length, h.batch_checksum};
            const uint64_t v = f[off / 8];
            w = (off & 4) ? (uint32_t)(v >> 32) : (uint32_t)v;
        } else if (off == 48) {
            w = h.message_count;
        }
        *(u32_ua *)(out + off) = w;
    }
    if (t == 0) {
        res->header = h;
        res->error.kind = kind;
        res->error.reason = 0;
        res->error.a = a;
        res->error.b = b;
        res->error.c = 0;
        res->batch_length = h.batch_length;
    }
}

}  // namespace iggy

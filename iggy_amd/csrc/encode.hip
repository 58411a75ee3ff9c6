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
//  k_enc_lanes  : batches without user headers: 8 lanes per frame, one 1 KiB
//                 block of the hashed stream per step, stores and hashing fused.
//  k_enc_recs + k_enc_ring : the same for segmented (>= 2^18-message) batches with
//                 the payload reads through LDS rings (per-frame records ahead).
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
    uint64_t *misc;       // [8]: 0 min origin, 1 blob bytes, 2 ts-error (~index, max), 3 n, 4 payload bytes,
                          //      5 batch does not fit the output capacity (nothing is written)
    iggy_batch_header *hdr;  // header being built
    uint32_t dbg;         // ablation bits (diagnostic build only; kDiagMask folds them out)
};

// the scan's result: origin, blob bytes, capacity verdict and the header being built
__device__ inline void enc_scan_result(EncScratch es, uint64_t n, uint64_t partition_id, uint64_t cap,
                                       uint64_t tot_pl, uint64_t tot_uh, uint64_t mn) {
    const uint64_t origin = (n == 0) ? 0 : mn;
    es.misc[0] = origin;
    es.misc[1] = 48 * n + tot_pl + tot_uh;
    es.misc[2] = 0;
    es.misc[3] = n;
    es.misc[4] = tot_pl;  // total payload bytes (bounds the lane-group kernel's loads)
    es.misc[5] = 256 + es.misc[1] > cap ? 1 : 0;
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

// single: the batch is one tile (n <= kEncTile), and this launch also does
// k_enc_scan's work (one launch less for small batches)
__global__ __launch_bounds__(256) void k_enc_prep(iggy_raw_messages m, EncScratch es, uint64_t partition_id,
                                                  uint64_t cap, uint32_t single) {
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
        if (single) {  // the tile's offsets are 0; the totals are the scan's
            es.tile_pl[t] = 0;
            es.tile_uh[t] = 0;
            es.tile_min[t] = s_min[255];
            enc_scan_result(es, n, partition_id, cap, s_pl[255], s_uh[255], s_min[255]);
        } else {
            es.tile_pl[t] = s_pl[255];
            es.tile_uh[t] = s_uh[255];
            es.tile_min[t] = s_min[255];
        }
    }
}

__global__ __launch_bounds__(256) void k_enc_scan(uint64_t ntiles, uint64_t n, uint64_t partition_id,
                                                  uint64_t cap, EncScratch es) {
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
    if (tid == 0) enc_scan_result(es, n, partition_id, cap, carry_pl, carry_uh, carry_min);
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

// one wave per frame, frames wid, wid + nwaves, ... (any layout, user headers included)
__device__ inline void enc_frames_body(const iggy_raw_messages &m, EncScratch es, uint8_t *out, uint64_t wid,
                                       uint64_t nwaves) {
    const int lane = threadIdx.x & 63;
    const uint64_t n = m.count;
    const uint64_t origin = es.misc[0];
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
__global__ __launch_bounds__(256) void k_enc_frames(iggy_raw_messages m, EncScratch es,
                                                    uint8_t *out, uint32_t fallback_only) {
    // fallback_only: the lane-group kernel ran unless the payload area is < 16 B
    if (es.misc[5] || (fallback_only && es.misc[4] >= 16)) return;
    enc_frames_body(m, es, out, ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6,
                    ((uint64_t)gridDim.x * blockDim.x) >> 6);
}

// ---------------------------------------------------------------------------
// k_enc_lanes: the frames step for batches without user headers (every SDK
// producer batch without headers; C3), in the decode's lane-group shape.
// Lane group fg (8 lanes) of wave vw encodes frames i = 8 vw + fg + j * 8 nvw at
// its own pace, one 1024-B block of the hashed stream H(40) || P(pl) per wave
// step, the next block (or the next frame's first block) already loading. Lane
// l = (m, par) carries stream pieces 1024b + 128q + 16(m + 4 par), q = 0..7: it
// loads them once (16 B from the payload), stores them to the frame and
// accumulates them into XXH3 accumulators 2m, 2m+1 for stripe parity par (the
// pair is folded before each scramble). Pieces below stream byte 40 are the
// synthesised header (ids, offset/timestamp deltas, lengths, reserved). The
// payload of frame i is followed by frame i+1's in the SoA buffer, so a piece
// that runs past its payload reads (and discards) the next one's bytes; only
// the buffer's last 15 bytes need a clamped, realigned load.
struct EFrame {
    // i >= count: none. The payload offset is kept as its two loaded halves and added
    // where it is used (the next step): adding them here made the compiler wait for
    // every outstanding load and store (vmcnt(0)) at each frame switch
    uint64_t i, tp, lp, pl;
    __device__ __forceinline__ uint64_t po() const { return tp + lp; }
};
__device__ __forceinline__ EFrame eframe(const iggy_raw_messages &m, const EncScratch &es, uint64_t i,
                                         uint64_t n) {
    EFrame f;
    f.i = i < n ? i : ~0ull;  // past this launch's range: none
    const uint64_t k = i < n ? i : 0;
    f.tp = es.tile_pl[k / kEncTile];
    f.lp = es.pl_local[k];
    f.pl = m.payload_lengths[k];
    return f;
}
// 128-bit little-endian value (lo, hi) moved down by d bytes (0 <= d < 16)
__device__ __forceinline__ void shr_bytes(uint64_t &lo, uint64_t &hi, uint32_t d) {
    const uint32_t n = 8 * d;
    if (n == 0) return;
    if (n < 64) {
        lo = (lo >> n) | (hi << (64 - n));
        hi >>= n;
    } else {
        lo = hi >> (n - 64);
        hi = 0;
    }
}
struct EStep {
    uint4 v[8];    // raw 16-B payload loads of the 8 pieces
    uint4 last;    // last-stripe piece (long frames, first step only)
    uint64_t id0, id1, ots;  // header inputs (first step only)
    bool clamped;  // the pieces took the clamped form (some lane near the payload area's end)
    uint64_t ntp, nlp, npl;  // the record of the frame that becomes `nxt` at the next switch
};
// the loads of frame f's block b (fixed count: unneeded ones read the buffer start)
__device__ __forceinline__ void eissue(const iggy_raw_messages &m, const EncScratch &es, const EFrame &f,
                                       uint32_t b, uint32_t poff, uint32_t mm, uint64_t ptot, uint64_t nrec,
                                       EStep &st) {
    const bool live = f.i < m.count;
    const uint64_t L = 40 + f.pl;
    const uint8_t *P = m.payloads;
    const uint64_t blk = (uint64_t)(b << 10);  // b < 2^22 (frames < 4 GiB): 32-bit shift
    // Common form: every piece of the block lies inside the payload area (the block
    // ends >= 16 B before it), so the 8 loads are one base + constant offsets, with
    // no per-piece select. Pieces past the frame read the next message's payload,
    // which the neighbouring lane group of the same wave reads at the same time.
    const bool near_lane = live ? f.po() + blk + 984 > ptot : ptot < 1024;
    st.clamped = __ballot(near_lane) != 0;
    if (!st.clamped) {
        const uint8_t *base = live ? P + f.po() + blk + poff - 40 : P;
        // piece 0 of block 0: the header pieces (poff 0, 16: value unused) and the
        // reserved | payload[0..8) piece (poff 32) read from the payload start
        const uint8_t *a0 = live ? ((b == 0 && poff <= 32) ? P + f.po() : base) : P;
        st.v[0] = ld128_any(a0);
        const uint64_t rem = live && L > blk + poff ? L - blk - poff : 0;  // stream bytes from piece 0 on
#pragma unroll
        for (int q = 1; q < 8; ++q) st.v[q] = ld128_any(rem > 128 * q ? base + 128 * q : P);
    } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint64_t sp = blk + 128 * q + poff;  // stream position of the piece
            // payload index of the piece's first byte (the s == 32 piece starts 8 B early)
            const uint64_t px = f.po() + (sp >= 40 ? sp - 40 : 0);
            const bool need = live && sp + 16 > 32 && sp < L;
            const uint64_t a = (px + 16 <= ptot) ? px : ptot - 16;  // clamp: realigned at use
            st.v[q] = ld128_any(P + (need ? a : 0));
        }
    }
    const bool lng = live && L > 240 && b == 0;
    st.last = ld128_any(P + (lng ? f.po() + (L - 64 + 16 * mm) - 40 : 0));
    const uint64_t i = live && b == 0 ? f.i : 0;
    st.id0 = m.ids[2 * i];
    st.id1 = m.ids[2 * i + 1];
    st.ots = m.origin_timestamps[i];
    const uint64_t k = nrec < m.count ? nrec : 0;
    st.ntp = es.tile_pl[k / kEncTile];
    st.nlp = es.pl_local[k];
    st.npl = m.payload_lengths[k];
}

__device__ inline void enc_short_frame(const iggy_raw_messages &m, EncScratch es, uint8_t *out, uint64_t origin,
                                       uint64_t i);
// own_tail (unsegmented launches of small batches): this launch also runs the < 16-B
// payload-area fallback and hashes the frames of <= 240 B (a slice per wave after its
// loop) -- two launches fewer than k_enc_frames + k_enc_short
// (a template parameter: the segmented launches keep the code without the tail)
template <bool OWN_TAIL>
__global__ __launch_bounds__(256, 2) void k_enc_lanes(iggy_raw_messages m, EncScratch es, uint8_t *out,
                                                       uint64_t f_lo, uint64_t f_hi) {
    const uint64_t ptot = es.misc[4];
    if (ptot < 16 || es.misc[5]) {  // tiny payload area: the fallback (k_enc_frames' body) encodes it
        if (OWN_TAIL && !es.misc[5])
            enc_frames_body(m, es, out, ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6,
                            ((uint64_t)gridDim.x * blockDim.x) >> 6);
        return;
    }
    const uint64_t n = f_hi < m.count ? f_hi : m.count;  // this launch: frames [f_lo, f_hi)
    const uint64_t origin = es.misc[0];
    const int lane = threadIdx.x & 63;
    const uint32_t l = lane & 7, mm = l >> 1, par = l & 1, fg = (uint32_t)lane >> 3;
    const uint32_t poff = 16 * (mm + 4 * par);
    const uint32_t vw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nvw = (gridDim.x * blockDim.x) >> 6;
    // stripe secrets live in LDS (one ds_read_b128 per piece) to keep the two
    // in-flight load sets and the accumulators in registers
    __shared__ uint64_t s_sec[24];
    if (threadIdx.x < 24) s_sec[threadIdx.x] = kSecretW8[threadIdx.x];
    __syncthreads();
    const uint64_t key0 = kSecretW8[16 + 2 * mm], key1 = kSecretW8[17 + 2 * mm];
    const uint64_t init0 = par ? 0 : kAccInit[2 * mm], init1 = par ? 0 : kAccInit[2 * mm + 1];
    const uint64_t last0 = kSecretLast[2 * mm], last1 = kSecretLast[2 * mm + 1];
    const uint64_t mrg0 = kSecretMerge[2 * mm], mrg1 = kSecretMerge[2 * mm + 1];
    const uint64_t stride = 8ull * nvw;
    const uint32_t sbase = par + 2 * mm;  // secret word of piece q: sbase + 2q (and + 1)

    EFrame cur = eframe(m, es, f_lo + 8ull * vw + fg, n);
    EFrame nxt = eframe(m, es, cur.i == ~0ull ? ~0ull : cur.i + stride, n);
    // The record of the frame after `nxt` travels with each step's load set (Y.n*),
    // so that a frame switch only moves registers whose loads the step already
    // waited for: a record loaded at the (divergent) switch itself was merged by
    // register moves right after its load, a vmcnt(0) that drained every
    // outstanding load and store of the wave at each frame switch.
    auto rec_after = [&](uint64_t c, bool sw) -> uint64_t {  // frame after nxt once the next step is done
        if (c == ~0ull) return ~0ull;
        const uint64_t r = c + (sw ? 3 : 2) * stride;
        return r < n ? r : ~0ull;
    };
    uint32_t b = 0;
    uint64_t a0 = init0, a1 = init1;
    uint64_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;  // header words of the current frame
    uint4 lastp = make_uint4(0, 0, 0, 0);      // the current frame's last-stripe piece
    // process the step whose loads are in X, issue the next step's into Y
    auto step = [&](EStep &X, EStep &Y) {
        if (cur.i >= n) return;
        const uint64_t L = 40 + cur.pl;
        const bool lng = L > 240;
        const uint64_t nbF = lng ? (L - 1) / 1024 : 0;
        const uint64_t ns = lng ? ((L - 1) - 1024 * nbF) / 64 : 0;
        const uint32_t nblk = (uint32_t)((L + 1023) / 1024);
        const bool fin = b + 1 == nblk;
        eissue(m, es, fin ? nxt : cur, fin ? 0u : b + 1, poff, mm, ptot, rec_after(cur.i, fin), Y);
        if (b == 0) {
            const uint64_t delta = X.ots - origin;
            if (delta > IGGY_MAX_TIMESTAMP_DELTA_MICROS && l == 0)
                atomicMax((unsigned long long *)&es.misc[2], (unsigned long long)~cur.i);
            h0 = X.id0;
            h1 = X.id1;
            h2 = (cur.i & 0xFFFFFFFFull) | ((delta & 0xFFFFFFFFull) << 32);
            h3 = cur.pl << 32;  // user_headers_len 0 | payload_len
            lastp = X.last;
        }
        uint8_t *F = out + 256 + 48 * cur.i + cur.po();  // frame start
        uint64_t p0[4] = {0, 0, 0, 0}, p1[4] = {0, 0, 0, 0};
        uint64_t tw0 = 0, tw1 = 0, tsp = ~0ull;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint64_t sp = (uint64_t)((b << 10) + 128 * q + poff);
            uint64_t w0 = (uint64_t)X.v[q].x | ((uint64_t)X.v[q].y << 32);
            uint64_t w1 = (uint64_t)X.v[q].z | ((uint64_t)X.v[q].w << 32);
            if (X.clamped) {  // a load clamped to the payload area's last 16 B: realign it
                const uint64_t px = cur.po() + (sp >= 40 ? sp - 40 : 0);
                if (px + 16 > ptot) shr_bytes(w0, w1, (uint32_t)(px + 16 - ptot));
            }
            if (sp < 40) {
                if (sp == 0) { w0 = h0; w1 = h1; }
                else if (sp == 16) { w0 = h2; w1 = h3; }
                else { w1 = w0; w0 = 0; }  // reserved | payload[0..8)
            }
            if (kDiagMask && (es.dbg & 0x30000)) {  // ablations: aligned destination / no stores
                if (!(es.dbg & 0x20000) && sp + 16 <= L)
                    *(uint4 *)(((uintptr_t)(F + 8) & ~(uintptr_t)15) + sp) =
                        make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32));
            } else if (sp + 16 <= L) {
                st128_any(F + 8 + sp, make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32)));
            } else if (sp < L) {  // the frame's partial last piece (at most one per lane)
                tw0 = w0; tw1 = w1; tsp = sp;
            }
            if (lng && !(kDiagMask && (es.dbg & 0x40000))) {  // (ablation: no hashing)
                const uint64_t sa = s_sec[sbase + 2 * q], sb = s_sec[sbase + 2 * q + 1];
                if (b < nbF) {
                    p0[q & 3] += mul32x32(w0 ^ sa) + w1;
                    p1[q & 3] += mul32x32(w1 ^ sb) + w0;
                } else if (2 * q + par < ns) {
                    a0 += mul32x32(w0 ^ sa) + w1;
                    a1 += mul32x32(w1 ^ sb) + w0;
                }
            }
        }
        if (tsp != ~0ull) {  // 1..15 bytes: at most one 8-, 4-, 2- and 1-byte store each
            uint8_t *d = F + 8 + tsp;
            const uint32_t rem = (uint32_t)(L - tsp);
            if (rem & 8) {
                st64_any(d, tw0);
                d += 8;
                tw0 = tw1;
            }
            if (rem & 4) {
                *(u32_ua *)d = (uint32_t)tw0;
                d += 4;
                tw0 >>= 32;
            }
            if (rem & 2) {
                *(u16_ua *)d = (uint16_t)tw0;
                d += 2;
                tw0 >>= 16;
            }
            if (rem & 1) *d = (uint8_t)tw0;
        }
        uint64_t hsh = 0;
        if (lng) {
            if (b < nbF) {
                a0 += (p0[0] + p0[1]) + (p0[2] + p0[3]);
                a1 += (p1[0] + p1[1]) + (p1[2] + p1[3]);
                a0 += gdpp64<0xB1>(a0);
                a1 += gdpp64<0xB1>(a1);
                a0 = scramble1(a0, key0);
                a1 = scramble1(a1, key1);
                if (par) { a0 = 0; a1 = 0; }
            }
            if (fin) {
                a0 += gdpp64<0xB1>(a0);
                a1 += gdpp64<0xB1>(a1);
                piece(a0, a1, lastp, last0, last1);
                uint64_t t = fold64(a0 ^ mrg0, a1 ^ mrg1);
                t += gdpp64<0x4E>(t);
                t += gswz_xor4(t);
                hsh = avalanche(L * P64_1 + t);
            }
        }
        if (fin) {
            if (l == 0 && lng) {  // frames of <= 240 hashed bytes: k_enc_short
                st64_any(F, hsh);
                es.cs[cur.i] = hsh;
            }
            cur = nxt;
            // X carries the record of the frame after nxt (issued a step ago)
            const uint64_t ni = cur.i == ~0ull || cur.i + stride >= n ? ~0ull : cur.i + stride;
            nxt.i = ni;
            nxt.tp = X.ntp;
            nxt.lp = X.nlp;
            nxt.pl = X.npl;
            b = 0;
            a0 = init0;
            a1 = init1;
        } else {
            ++b;
        }
    };
    // ping-pong over two load sets (no register copy of in-flight loads)
    EStep A, B;
    eissue(m, es, cur, 0, poff, mm, ptot, rec_after(cur.i, false), A);
    while (__ballot(cur.i < n)) {
        step(A, B);
        if (!__ballot(cur.i < n)) break;
        step(B, A);
    }
    if (OWN_TAIL) {  // frames of <= 240 hashed bytes: one lane each, a slice per wave
        const uint64_t C = (n + nvw - 1) / nvw;
        const uint64_t f1 = min((uint64_t)(vw + 1) * C, n);
        for (uint64_t i = (uint64_t)vw * C + lane; i < f1; i += 64) enc_short_frame(m, es, out, origin, i);
    }
}

// ---------------------------------------------------------------- ring encode
// k_enc_ring: the lane-group encode of segmented launches in the decode rings' shape
// (decode_general.hip verify_frames_dma). k_enc_lanes' waves spend half their
// cycles in s_waitcnt: their loads and their frame stores share one vmcnt, and the
// compiler's waits for the next register set also wait for the previous step's
// stores. Here every wave (8 per CU) streams the payload through a 2-slot LDS ring
// with exactly 9 global_load_lds_dwordx4 per step (the block's 16-B-aligned payload
// window, read back at the byte offset), and issues exactly kErStores stores per
// step from inline asm (8 pieces, 4 tail widths, 2 checksum words; a lane with
// nothing to store writes its sink slot), so one constant vmcnt wait covers both.
// Frame records (payload offset, length, timestamp delta, ids: erec, k_enc_recs)
// reach LDS four frames ahead through the ninth instruction, as vrec does.
#ifndef IGGY_ER_SLOTS
#define IGGY_ER_SLOTS 3  // (build knobs for same-box A/B: ring slots, waves per workgroup)
#endif
#ifndef IGGY_ER_WAVES
#define IGGY_ER_WAVES 4
#endif
constexpr uint32_t kErSlots = IGGY_ER_SLOTS;
constexpr uint32_t kErStep = 9 * 1024;
constexpr uint32_t kErMeta = 8 * 9 * 16;     // 8 groups x (8 records + a spare)
constexpr uint32_t kErWave = kErSlots * kErStep + kErMeta;
constexpr uint32_t kErWaves = IGGY_ER_WAVES;
constexpr uint32_t kErThreads = 64 * kErWaves;
constexpr uint32_t kErLds = kErWaves * kErWave;
#ifndef IGGY_ER_NT
#define IGGY_ER_NT 0
#endif
#ifndef IGGY_ER_NOSTORE
#define IGGY_ER_NOSTORE 0  // (timing-only build knob, wrong output: mode 2 without the frame byte stores)
#endif
#ifndef IGGY_ER_TSTORE
#define IGGY_ER_TSTORE 0  // (timing-only build knob, wrong output: transposed 1-KiB store runs)
#endif
#ifndef IGGY_ER_A128
#define IGGY_ER_A128 0  // (timing-only build knob, wrong output: piece stores to 128-B-aligned runs)
#endif
#ifndef IGGY_ER_MODE
#define IGGY_ER_MODE 2  // (build knob: 0 every store from asm with sinks; 1 the 8 piece stores only;
                        //  2 no unconditional store -- the ring wait then counts loads only;
                        //  3 every store from asm, lanes without bytes masked off, one lane
                        //    writing its sink only when no lane of the wave has bytes)
#endif
constexpr uint32_t kErStores = (IGGY_ER_MODE == 0 || IGGY_ER_MODE == 3) ? 14 : IGGY_ER_MODE == 1 ? 8 : 0;  // stores per step, at least
constexpr uint64_t kErSinkBytes = 256 << 10; // 256 wave slots x 64 lanes x 16 B
static_assert(kErLds <= 160 * 1024, "LDS budget");
static_assert(9 * (kErSlots - 1) + kErStores * kErSlots <= 63, "the ring wait fits vmcnt");
static_assert(IGGY_ER_MODE >= 0 && IGGY_ER_MODE <= 3, "store mode");
// a frame's record is copied into the ring when its group's frame four ahead starts;
// the issue side runs kErSlots steps ahead of that copy, so at most 4 slots (a 5-slot
// build read a stale record and faulted)
static_assert(kErSlots <= 4, "ring deeper than the record lookahead");

typedef uint32_t er_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void er_st16(void *p, uint64_t w0, uint64_t w1) {
    const er_v4u v = {(uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32)};
    asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void er_st8(void *p, uint64_t v) {
    asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void er_st4(void *p, uint32_t v) {
    asm volatile("global_store_dword %0, %1, off" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void er_st2(void *p, uint32_t v) {
    asm volatile("global_store_short %0, %1, off" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void er_st1(void *p, uint32_t v) {
    asm volatile("global_store_byte %0, %1, off" ::"v"(p), "v"(v) : "memory");
}
// (mode 3) exactly one store instruction per call and wave: the lanes with bytes store
// them; when no lane has any, lane 0 alone writes its sink slot (so the instruction
// still issues and counts once in vmcnt)
__device__ __forceinline__ bool er_act(bool has) {
    return has || (__ballot(has) == 0 && (threadIdx.x & 63) == 0);
}

// erec[2 i] = {po lo, po hi, payload length, timestamp delta}, erec[2 i + 1] = the ids;
// erec[2 n], [2 n + 1] = zero (no frame). Also the timestamp-delta check of every frame.
__global__ __launch_bounds__(256) void k_enc_recs(iggy_raw_messages m, EncScratch es, uint4 *erec) {
    const uint64_t n = m.count;
    const uint64_t origin = es.misc[0];
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        if (i == n) {
            erec[2 * n] = make_uint4(0, 0, 0, 0);
            erec[2 * n + 1] = make_uint4(0, 0, 0, 0);
            continue;
        }
        const uint64_t po = es.tile_pl[i / kEncTile] + es.pl_local[i];
        const uint32_t pl = m.payload_lengths[i];
        const uint64_t delta = m.origin_timestamps[i] - origin;
        if (delta > IGGY_MAX_TIMESTAMP_DELTA_MICROS)
            atomicMax((unsigned long long *)&es.misc[2], (unsigned long long)~i);
        const uint64_t id0 = m.ids[2 * i], id1 = m.ids[2 * i + 1];
        erec[2 * i] = make_uint4((uint32_t)po, (uint32_t)(po >> 32), pl, (uint32_t)delta);
        erec[2 * i + 1] = make_uint4((uint32_t)id0, (uint32_t)(id0 >> 32), (uint32_t)id1, (uint32_t)(id1 >> 32));
    }
}

// ---- writer waves (SPLIT form): the hasher waves above store no payload bytes.
// A SPLIT workgroup has kErWaves writer waves beside its kErWaves hashers; writer
// wave kErWaves + w reads hasher w's landed LDS slots back and stores the frames'
// payload bytes, so the hashers' constant-vmcnt ring waits cover their loads (and two
// small stores per frame) only. Hand-off in lockstep: every wave of the workgroup
// runs the same number of steps K (the workgroup's longest hasher sequence) and
// meets the others at one workgroup barrier per step. Step k: a hasher waits for its
// step-k loads, reads the slot, writes the step's descriptors (per frame group: the
// destination of stream byte 0, hashed length, block, window misalignment), reaches
// barrier k, then refills the slot of step k - 1 with step k + S - 1 and hashes step
// k; a writer reaches barrier k, reads slot k and its descriptors, then stores, and
// its reads have returned before it reaches barrier k + 1. Nobody spins: the first
// form of this split (LDS flags, the hasher polling the writer's progress) saw the
// writer's global stores stall for as long as the hasher polled and resume the
// moment it stopped, at the 4-s bug guard; a second form (writer waves copying the
// payloads from the input on their own) was exact but took 2.51-2.71 ms against
// 1.36 ms. This lockstep form is exact and never stalls, but same box: 1.60 ms against
// 1.36 (1.02 ms with the writers storing nothing), so the host builds without it
// (IGGY_ENC_SPLIT 0, codec_api.hip).
// With payloads and output 16-B congruent (P - out = 0 mod 16: 48-B frame headers keep
// every payload at the same offset mod 16 from its source; the host launches the SPLIT
// form only then), each window chunk is one aligned 16-B store, except the chunks that
// straddle the payload's ends (aligned 8/4/2/1-B pieces). The frame header (40 B) and
// the checksum word are the hasher's.
constexpr uint32_t kEsSlots = 4;  // 3 steps in flight while one is hashed
constexpr uint32_t kEsDesc = kEsSlots * 128;  // [slot][group] {dst lo, dst hi, L, block | r << 16 | valid << 24}
constexpr uint32_t kEsWave = kEsSlots * kErStep + kErMeta + kEsDesc;
constexpr uint32_t kEsLds = kErWaves * kEsWave + 16;  // + the hashers' step counts
static_assert(kEsLds <= 160 * 1024 || kErWaves != 4, "LDS budget (split ring; only built with 4 hashers)");
static_assert(kEsSlots <= 4, "the issue side runs kEsSlots - 1 steps ahead of the record copy (<= 4)");

typedef __attribute__((address_space(1))) uint8_t g_u8;
typedef __attribute__((address_space(1))) uint16_t g_u16;
typedef __attribute__((address_space(1))) uint32_t g_u32;
typedef __attribute__((address_space(1))) uint64_t g_u64;
typedef unsigned int es_u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) es_u32x4 g_u128;

// bytes [x0, x1) of the 16-B value v to the 16-B-aligned address d: aligned 8/4/2/1-B pieces
__device__ inline void es_store_range(g_u8 *d, es_u32x4 v, uint32_t x0, uint32_t x1) {
    while (x0 < x1) {
        const uint32_t dw = x0 >> 2;
        const uint32_t w = dw == 0 ? v.x : dw == 1 ? v.y : dw == 2 ? v.z : v.w;
        if ((x0 & 7) == 0 && x0 + 8 <= x1) {
            const uint32_t w2 = dw == 0 ? v.y : v.w;
            *(g_u64 *)(d + x0) = (uint64_t)w | ((uint64_t)w2 << 32);
            x0 += 8;
        } else if ((x0 & 3) == 0 && x0 + 4 <= x1) {
            *(g_u32 *)(d + x0) = w;
            x0 += 4;
        } else if ((x0 & 1) == 0 && x0 + 2 <= x1) {
            *(g_u16 *)(d + x0) = (uint16_t)(w >> (8 * (x0 & 3)));
            x0 += 2;
        } else {
            d[x0] = (uint8_t)(w >> (8 * (x0 & 3)));
            x0 += 1;
        }
    }
}

// the workgroup barrier without a memory fence (__syncthreads would drain every
// wave's vmcnt: the hashers' loads in flight and the writers' stores)
__device__ __forceinline__ void es_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// writer wave of the hasher whose LDS region is `region`: K lockstep steps
__device__ __forceinline__ void enc_ring_writer(const uint8_t *smem, uint32_t region, int lane, uint32_t K) {
    const uint32_t l = lane & 7, fg = (uint32_t)lane >> 3;
    for (uint32_t k = 0; k < K; ++k) {
        es_barrier();  // step k's slot and descriptors are in
        const uint32_t slot = region + (k % kEsSlots) * kErStep;
        const uint4 dsc = *(const uint4 *)(smem + region + kEsSlots * kErStep + kErMeta + 128 * (k % kEsSlots) + 16 * fg);
        es_u32x4 c[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) c[q] = *(const es_u32x4 *)(smem + slot + 1024u * q + 16u * (uint32_t)lane);
        const es_u32x4 c64 = *(const es_u32x4 *)(smem + slot + 8192u + 128u * fg);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read out before barrier k + 1 (the refill)
        if ((dsc.w >> 24) == 0) continue;
        g_u8 *F8 = (g_u8 *)((uint64_t)dsc.x | ((uint64_t)dsc.y << 32));  // destination of stream byte 0
        const int64_t L = dsc.z;
        const int64_t pb = dsc.w & 0xffff;
        const int64_t r = (dsc.w >> 16) & 0xff;
        // window chunk cc covers stream [pb * 1024 + 16 cc - r, + 16): r == 0 -> chunks
        // 0..63, r > 0 -> 1..64 (chunk 0 straddles the block start: the previous block's 64)
#pragma unroll
        for (int q = 0; q < 9; ++q) {
            if (q == 8 && l != 0) break;
            const int64_t cc = q < 8 ? 8 * q + l : 64;
            if (cc == 0 && r != 0) continue;
            if (cc == 64 && r == 0) continue;
            const int64_t sp = pb * 1024 + 16 * cc - r;
            const int64_t a = sp > 40 ? sp : 40, b = sp + 16 < L ? sp + 16 : L;
            if (a >= b) continue;
            const es_u32x4 v = q < 8 ? c[q] : c64;
            g_u8 *d = F8 + sp;
            if (a == sp && b == sp + 16) *(g_u128 *)d = v;
            else es_store_range(d, v, (uint32_t)(a - sp), (uint32_t)(b - sp));
        }
    }
}

template <bool SPLIT>
__global__ __launch_bounds__(SPLIT ? 2 * kErThreads : kErThreads, 1) void k_enc_ring(iggy_raw_messages m, EncScratch es,
                                                                                uint8_t *out, uint64_t f_lo, uint64_t f_hi,
                                                                                const uint4 *erec, uint8_t *sink) {
    constexpr uint32_t S = SPLIT ? kEsSlots : kErSlots;   // ring slots per hasher wave
    constexpr uint32_t WAVE = SPLIT ? kEsWave : kErWave;   // LDS per hasher wave
    constexpr uint32_t AHEAD = SPLIT ? S - 1 : S;           // steps issued ahead of the processed one
    const uint64_t ptot = es.misc[4];
    if (ptot < 16 || es.misc[5]) return;  // tiny payload area (k_enc_frames) or over capacity
    const uint64_t N = m.count;           // erec[2 N]: the "no frame" record
    const uint64_t n = f_hi < N ? f_hi : N;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    typedef __attribute__((address_space(3))) uint8_t lds_u8;
    const uint32_t lbase = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_u8 *)smem);
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t *s_steps = (uint32_t *)(smem + kErWaves * kEsWave);  // (SPLIT) each hasher wave's step count
    if (SPLIT && wave >= kErWaves) {  // the writer of hasher wave - kErWaves
        es_barrier();                 // the step counts are in
        const uint32_t K = max(max(s_steps[0], s_steps[1]), max(s_steps[2], s_steps[3]));
        enc_ring_writer(smem, (wave - kErWaves) * WAVE, lane, K);
        return;
    }
    const uint32_t l = lane & 7, m8 = l >> 1, par = l & 1, fg = (uint32_t)lane >> 3;
    const uint32_t poff = 16 * (m8 + 4 * par);
    const uint64_t vw = (uint64_t)blockIdx.x * kErWaves + wave, nvw = (uint64_t)gridDim.x * kErWaves;
    const uint64_t stride = 8 * nvw;
    const uint32_t region = __builtin_amdgcn_readfirstlane(wave * WAVE);
    const uint8_t *P = m.payloads;
    const uint8_t *dummy = P;  // (ptot >= 16)
    uint8_t *my_sink = sink + ((vw & 255) << 10) + 16 * lane;
    uint64_t s0[8], s1[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        s0[q] = kSecretW8[2 * q + par + 2 * m8];
        s1[q] = kSecretW8[2 * q + par + 2 * m8 + 1];
    }
    const uint64_t key0 = kSecretW8[16 + 2 * m8], key1 = kSecretW8[17 + 2 * m8];
    const uint64_t init0 = par ? 0 : kAccInit[2 * m8], init1 = par ? 0 : kAccInit[2 * m8 + 1];
    const uint64_t last0 = kSecretLast[2 * m8], last1 = kSecretLast[2 * m8 + 1];
    const uint64_t mrg0 = kSecretMerge[2 * m8], mrg1 = kSecretMerge[2 * m8 + 1];
    {  // every constant waited for before the first DMA (see verify_frames_dma)
        uint64_t sk = key0 ^ key1 ^ init0 ^ init1 ^ last0 ^ last1 ^ mrg0 ^ mrg1;
#pragma unroll
        for (int q = 0; q < 8; ++q) sk ^= s0[q] ^ s1[q];
        asm volatile("" : "+v"(sk));
    }
    // the group's frames: ordinal j is frame f_lo + 8 vw + fg + j stride (N: none)
    const uint64_t fbase = f_lo + 8 * vw + fg;
    auto fidx = [&](uint64_t j) -> uint64_t {
        const uint64_t f = fbase + j * stride;
        return f < n ? f : N;
    };
    uint32_t K = 0;  // (SPLIT) the workgroup's lockstep step count
    if (SPLIT) {
        // this wave's steps: per frame group the sum of its frames' blocks, the max over
        // the groups; the workgroup runs the largest of its hashers' counts
        uint32_t st = 0;
        for (uint64_t j = l;; j += 8) {
            const uint64_t f = fidx(j);
            if (!__ballot(f < N)) break;
            if (f < N) st += (uint32_t)((40 + (uint64_t)erec[2 * f].z + 1023) >> 10);
        }
        st += __shfl_xor(st, 1);
        st += __shfl_xor(st, 2);
        st += __shfl_xor(st, 4);
        st = max(st, (uint32_t)__shfl_xor(st, 8));
        st = max(st, (uint32_t)__shfl_xor(st, 16));
        st = max(st, (uint32_t)__shfl_xor(st, 32));
        if (lane == 0) s_steps[wave] = st;
        es_barrier();
        K = max(max(s_steps[0], s_steps[1]), max(s_steps[2], s_steps[3]));
    }
    const uint32_t meta = region + S * kErStep + 144 * fg;  // the group's record ring
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k)
        if (l == k) *(uint4 *)(smem + meta + 16 * k) = erec[2 * fidx(k)];
    // issue cursor: ordinal ij, block ib; per-frame state set at the frame's first block
    uint32_t ij = 0, ib = 0, i_nsteps = 1, i_r = 0;
    uint64_t i_L = 0;
    bool i_valid = false;
    const uint8_t *i_g = dummy, *i_x9 = dummy;
    auto issue = [&](uint32_t slot_off) {
        const uint32_t slot = lbase + slot_off;
        const bool first = ib == 0;
        if (first) {
            const uint4 rec = *(const uint4 *)(smem + meta + 16 * (ij & 7));
            const uint64_t f = fidx(ij);
            i_valid = f < N;
            const uint64_t po = (uint64_t)rec.x | ((uint64_t)rec.y << 32), pl = rec.z;
            i_L = 40 + pl;
            i_nsteps = i_valid ? (uint32_t)((i_L + 1023) >> 10) : 1u;
            const uint8_t *W0 = P + po - 40;  // stream position 0 (the header is not loaded)
            i_r = (uint32_t)((uintptr_t)W0 & 15);
            i_g = W0 - i_r + 16 * l;
            const uint64_t hi0 = i_r + (i_L < 1024 ? i_L : 1024);
            const uint8_t *Ls = P + po + pl - 64;  // the last stripe (pl > 200 when it is hashed)
            const uint32_t rl = (uint32_t)((uintptr_t)Ls & 15);
            const bool lng = i_valid && i_L > 240;
            const uint8_t *c0 = (i_valid && hi0 > 1024) ? i_g + 1024 : dummy;  // (l == 0)
            const uint8_t *cl = (lng && (l < 5 || rl)) ? Ls - rl + 16 * (l - 1) : dummy;
            const uint8_t *c6 = i_valid ? (const uint8_t *)(erec + 2 * f + 1) : dummy;
            const uint8_t *c7 = (const uint8_t *)(erec + 2 * fidx(ij + 4));
            i_x9 = l == 0 ? c0 : l <= 5 ? cl : l == 6 ? c6 : c7;
        }
        const uint8_t *g = i_g + ((uint64_t)ib << 10);
        // window bytes of this block: [lo, hi) (block 0 starts after the 40 header bytes)
        const uint64_t rem = i_L - ((uint64_t)ib << 10);
        const uint32_t hi = i_valid ? i_r + (uint32_t)(rem < 1024 ? rem : 1024) : 0u;
        const uint32_t lo = i_r + (first ? 40u : 0u);
#pragma unroll
        for (uint32_t q = 0; q < 8; ++q) {
            const uint32_t c0 = 128 * q + 16 * l;
            glds16(c0 < hi && c0 + 16 > lo ? g + 128 * q : dummy, slot + 1024u * q);
        }
        glds16(first ? i_x9 : ((l == 0 && hi > 1024) ? g + 1024 : dummy), slot + 8u * 1024u);
        if (++ib == i_nsteps) {
            ib = 0;
            ++ij;
        }
    };
    // processing cursor
    uint32_t pj = 0, pb = 0, p_nsteps = 1, rb = 0, rl = 0, p_delta = 0;
    uint64_t p_f = N, p_L = 0, p_pl = 0, nbF = 0, ns = 0;
    bool p_valid = false, lng = false;
    uint8_t *F = my_sink;
    uint32_t o5[5] = {0, 0, 0, 0, 0};
    uint64_t a0 = init0, a1 = init1, id0 = 0, id1 = 0;
    uint4 lastp = make_uint4(0, 0, 0, 0);
    for (uint32_t k = 0; k < AHEAD; ++k) issue(region + k * kErStep);
    uint32_t k = 0;
    for (; !SPLIT || k < K; ++k) {
        if (pb == 0) {
            const uint4 rec = *(const uint4 *)(smem + meta + 16 * (pj & 7));
            p_f = fidx(pj);
            p_valid = p_f < N;
            const uint64_t po = (uint64_t)rec.x | ((uint64_t)rec.y << 32);
            p_pl = rec.z;
            p_delta = rec.w;
            p_L = 40 + p_pl;
            p_nsteps = p_valid ? (uint32_t)((p_L + 1023) >> 10) : 1u;
            lng = p_valid && p_L > 240;
            nbF = (p_L - 1) >> 10;
            ns = ((p_L - 1) & 1023) >> 6;
            const uint32_t r = (uint32_t)((uintptr_t)(P + po - 40) & 15);
            rb = r & 3;
            const uint32_t e = (64 * par + 16 * m8 + r) >> 2;
#pragma unroll
            for (uint32_t j = 0; j < 5; ++j) o5[j] = 1024u * ((e + j) >> 5) + 4u * ((e + j) & 31);
            rl = (uint32_t)((uintptr_t)(P + po + p_pl - 64) & 15);
            F = p_valid ? out + 256 + 48 * p_f + po : my_sink;
            a0 = init0;
            a1 = init1;
        }
        if (!SPLIT && !__ballot(p_valid)) break;
        // step k landed. Issued after its loads: the stores of the kErSlots steps
        // before it and the loads of the later steps -- except in the first kErSlots
        // iterations, which wait for everything.
        if (k < AHEAD) wait_vm_const<0>();
        else if (SPLIT) wait_vm_const<9 * (S - 2)>();
        else wait_vm_const<9 * (kErSlots - 1) + kErStores * kErSlots>();
        if (SPLIT && l == 0) {  // the step's descriptors for the writer (read after barrier k)
            const uint64_t d8 = (uint64_t)(uintptr_t)(F + 8);
            const uint32_t r = (uint32_t)((uintptr_t)(P + (F - out - 256 - 48 * p_f) - 40) & 15);
            *(uint4 *)(smem + region + S * kErStep + kErMeta + 128 * (k % S) + 16 * fg) =
                make_uint4((uint32_t)d8, (uint32_t)(d8 >> 32), (uint32_t)p_L, pb | (r << 16) | ((p_valid ? 1u : 0u) << 24));
        }
        const uint32_t slot = region + (k % S) * kErStep;
        const uint8_t *row = smem + slot + 128 * fg;
        uint4 pc[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            uint32_t d[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) d[j] = *(const uint32_t *)(row + 1024 * q + o5[j]);
            pc[q] = vd_align(d, rb);
        }
        const bool first = pb == 0;
        {  // first block: last-stripe piece, ids, and the record four frames ahead
            uint32_t d[5];
            const uint8_t *ls = row + 8192 + 16 + ((rl + 16 * m8) & ~3u);
#pragma unroll
            for (int j = 0; j < 5; ++j) d[j] = *(const uint32_t *)(ls + 4 * j);
            const uint4 lp = vd_align(d, rl & 3);
            const uint4 ids = *(const uint4 *)(row + 8192 + 96);
            const uint4 rec = *(const uint4 *)(row + 8192 + 112);
            if (l == 7) *(uint4 *)(smem + meta + 16 * (first ? (pj + 4) & 7 : 8u)) = rec;
            lastp.x = first ? lp.x : lastp.x;
            lastp.y = first ? lp.y : lastp.y;
            lastp.z = first ? lp.z : lastp.z;
            lastp.w = first ? lp.w : lastp.w;
            id0 = first ? ((uint64_t)ids.x | ((uint64_t)ids.y << 32)) : id0;
            id1 = first ? ((uint64_t)ids.z | ((uint64_t)ids.w << 32)) : id1;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot read out before it is refilled
        if (SPLIT) {
            es_barrier();  // barrier k: the writer reads slot k; slot k - 1 is free
            issue(region + ((k + S - 1) % S) * kErStep);
        } else {
            issue(slot);
        }
        // the block's pieces: header words substituted, stored, hashed
        const bool full = lng && pb < nbF;
        uint64_t q0[4] = {0, 0, 0, 0}, q1[4] = {0, 0, 0, 0};
        uint64_t tw = 0, tsp = ~0ull;  // the lane's partial last piece (1..15 bytes), if any
        uint64_t tw1 = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint64_t sp = ((uint64_t)pb << 10) + 128 * q + poff;
            uint64_t w0 = (uint64_t)pc[q].x | ((uint64_t)pc[q].y << 32);
            uint64_t w1 = (uint64_t)pc[q].z | ((uint64_t)pc[q].w << 32);
            if (q == 0) {  // stream bytes 0..47 of block 0: the header words
                const bool h = pb == 0;
                const uint64_t hw2 = (p_f & 0xFFFFFFFFull) | ((uint64_t)p_delta << 32), hw3 = p_pl << 32;
                const uint64_t n0 = poff == 0 ? id0 : poff == 16 ? hw2 : 0;
                const uint64_t n1 = poff == 0 ? id1 : poff == 16 ? hw3 : w1;
                w0 = (h && poff <= 32) ? n0 : w0;
                w1 = (h && poff <= 32) ? n1 : w1;
            }
            const bool whole = p_valid && sp + 16 <= p_L;
            if (SPLIT) {
                // (the writer wave stores the payload; the header words are stored below)
            } else if (IGGY_ER_MODE == 3) {
                if (er_act(whole)) er_st16(whole ? (void *)(F + 8 + sp) : (void *)my_sink, w0, w1);
            } else if (IGGY_ER_MODE < 2) {
                er_st16(whole ? (void *)(F + 8 + sp) : (void *)my_sink, w0, w1);
            } else if (IGGY_ER_TSTORE) {
                // (timing only, wrong output: the store pattern of a transposed writer --
                // instruction q writes 1 KiB of group q's frame block, 16-B aligned,
                // every lane one chunk -- with this lane's own piece as the data)
                const uint32_t flo = __builtin_amdgcn_readlane((uint32_t)(uintptr_t)F, 8 * q);
                const uint32_t fhi = __builtin_amdgcn_readlane((uint32_t)((uintptr_t)F >> 32), 8 * q);
                const uint32_t pbq = __builtin_amdgcn_readlane(pb, 8 * q);
                const uint32_t lq = __builtin_amdgcn_readlane((uint32_t)p_L, 8 * q);
                const uint32_t vq = __builtin_amdgcn_readlane(p_valid ? 1u : 0u, 8 * q);
                uint8_t *Fq = (uint8_t *)((((uint64_t)fhi << 32) | flo) & ~(uint64_t)15);
                const uint64_t spt = ((uint64_t)pbq << 10) + 16 * (uint32_t)lane;
                if (vq && spt + 16 <= lq)
                    st128_any(Fq + spt, make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32)));
            } else if (IGGY_ER_A128) {  // (timing only, wrong output: each group's run 128-B aligned)
                if (whole) {
                    uint8_t *Fa = (uint8_t *)((uintptr_t)(F + 8) & ~(uintptr_t)127);
                    st128_any(Fa + sp, make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32)));
                }
            } else if (whole && !IGGY_ER_NOSTORE) {
#if IGGY_ER_NT  // (build knob for a same-box A/B: non-temporal piece stores)
                const er_v4u v = {(uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32)};
                asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(F + 8 + sp), "v"(v) : "memory");
#else
                st128_any(F + 8 + sp, make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32)));
#endif
            }
            const bool part = p_valid && sp < p_L && sp + 16 > p_L;
            tsp = part ? sp : tsp;
            tw = part ? w0 : tw;
            tw1 = part ? w1 : tw1;
            const uint64_t use = 0ull - (uint64_t)(full || (lng && pb == nbF && (uint64_t)(2 * q + par) < ns));
            q0[q & 3] += (mul32x32(w0 ^ s0[q]) + w1) & use;
            q1[q & 3] += (mul32x32(w1 ^ s1[q]) + w0) & use;
        }
        if (SPLIT) {
            // the frame header at its first block: lanes 0-4 of the group store its five
            // words (ids, index | timestamp delta, lengths, reserved) at F + 8
            if (pb == 0 && p_valid && l < 5) {
                const uint64_t hw = l == 0 ? id0 : l == 1 ? id1
                                  : l == 2 ? ((p_f & 0xFFFFFFFFull) | ((uint64_t)p_delta << 32))
                                  : l == 3 ? (p_pl << 32) : 0ull;
                st64_any(F + 8 + 8 * l, hw);
            }
        } else if (IGGY_ER_MODE == 3) {  // the partial piece: 8-, 4-, 2-, 1-byte stores, masked
            const bool has = tsp != ~0ull;
            const uint32_t remb = has ? (uint32_t)(p_L - tsp) : 0u;
            uint8_t *d = F + 8 + (has ? tsp : 0);
            uint64_t v = tw;
            if (er_act(remb & 8)) er_st8((remb & 8) ? (void *)d : (void *)my_sink, v);
            d += (remb & 8);
            v = (remb & 8) ? tw1 : v;
            if (er_act(remb & 4)) er_st4((remb & 4) ? (void *)d : (void *)my_sink, (uint32_t)v);
            d += (remb & 4);
            v = (remb & 4) ? (v >> 32) : v;
            if (er_act(remb & 2)) er_st2((remb & 2) ? (void *)d : (void *)my_sink, (uint32_t)v);
            d += (remb & 2);
            v = (remb & 2) ? (v >> 16) : v;
            if (er_act(remb & 1)) er_st1((remb & 1) ? (void *)d : (void *)my_sink, (uint32_t)v);
        } else if (IGGY_ER_MODE > 0) {  // the partial piece and the checksum words: plain stores
            if (!IGGY_ER_NOSTORE && tsp != ~0ull) {
                uint8_t *d = F + 8 + tsp;
                const uint32_t remb = (uint32_t)(p_L - tsp);
                uint64_t v = tw;
                if (remb & 8) { st64_any(d, v); d += 8; v = tw1; }
                if (remb & 4) { *(u32_ua *)d = (uint32_t)v; d += 4; v >>= 32; }
                if (remb & 2) { *(u16_ua *)d = (uint16_t)v; d += 2; v >>= 16; }
                if (remb & 1) *d = (uint8_t)v;
            }
        } else {  // the partial piece: 8-, 4-, 2-, 1-byte stores (a sink write for each width not used)
            const bool has = tsp != ~0ull;
            const uint32_t remb = has ? (uint32_t)(p_L - tsp) : 0u;
            uint8_t *d = F + 8 + (has ? tsp : 0);
            uint64_t v = tw;
            er_st8((remb & 8) ? (void *)d : (void *)my_sink, v);
            d += (remb & 8);
            v = (remb & 8) ? tw1 : v;
            er_st4((remb & 4) ? (void *)d : (void *)my_sink, (uint32_t)v);
            d += (remb & 4);
            v = (remb & 4) ? (v >> 32) : v;
            er_st2((remb & 2) ? (void *)d : (void *)my_sink, (uint32_t)v);
            d += (remb & 2);
            v = (remb & 2) ? (v >> 16) : v;
            er_st1((remb & 1) ? (void *)d : (void *)my_sink, (uint32_t)v);
        }
        a0 += (q0[0] + q0[1]) + (q0[2] + q0[3]);
        a1 += (q1[0] + q1[1]) + (q1[2] + q1[3]);
        {
            const uint64_t f0 = a0 + gdpp64<0xB1>(a0), f1 = a1 + gdpp64<0xB1>(a1);
            a0 = full ? (par ? 0 : scramble1(f0, key0)) : a0;
            a1 = full ? (par ? 0 : scramble1(f1, key1)) : a1;
        }
        const bool fin = pb + 1 == p_nsteps;
        uint64_t hsh = 0;
        if (__ballot(fin && lng)) {
            uint64_t b0 = a0 + gdpp64<0xB1>(a0), b1 = a1 + gdpp64<0xB1>(a1);
            piece(b0, b1, lastp, last0, last1);
            uint64_t t = fold64(b0 ^ mrg0, b1 ^ mrg1);
            t += gdpp64<0x4E>(t);
            t += gswz_xor4(t);
            hsh = avalanche(p_L * P64_1 + t);
        }
        {  // the frame's checksum word and its batch-checksum input (long frames; short
           // ones are k_enc_short's)
            const bool st = fin && lng && l == 0;
            if (SPLIT) {  // lane 0 the frame's checksum word, lane 2 (the same hash) its copy
                if (fin && lng && l == 0) st64_any(F, hsh);
                if (fin && lng && l == 2) es.cs[p_f] = hsh;
            } else if (IGGY_ER_MODE == 3) {
                if (er_act(st)) er_st8(st ? (void *)F : (void *)my_sink, hsh);
                if (er_act(st)) er_st8(st ? (void *)(es.cs + p_f) : (void *)(my_sink + 8), hsh);
            } else if (IGGY_ER_MODE > 0) {
                if (st) {
                    st64_any(F, hsh);
                    es.cs[p_f] = hsh;
                }
            } else {
                er_st8(st ? (void *)F : (void *)my_sink, hsh);
                er_st8(st ? (void *)(es.cs + p_f) : (void *)(my_sink + 8), hsh);
            }
        }
        if (++pb == p_nsteps) {
            pb = 0;
            ++pj;
        }
    }
    wait_vm_const<0>();
}

// Frames of <= 240 hashed bytes of a lane-group encode: one lane each hashes the
// stream (XXH3 17-128 / 129-240 paths) from the SoA input and backpatches.
__device__ inline void enc_short_frame(const iggy_raw_messages &m, EncScratch es, uint8_t *out, uint64_t origin,
                                       uint64_t i) {
    const uint64_t pl = m.payload_lengths[i];
    if (40 + pl > 240) return;
    const uint64_t po = es.tile_pl[i / kEncTile] + es.pl_local[i];
    FrameStream fs;
    fs.pl = pl;
    fs.uh = 0;
    fs.L = 40 + pl;
    fs.P = m.payloads + po;
    fs.U = m.payloads;
    const uint64_t delta = m.origin_timestamps[i] - origin;
    fs.h[0] = m.ids[2 * i];
    fs.h[1] = m.ids[2 * i + 1];
    fs.h[2] = (i & 0xFFFFFFFFull) | ((delta & 0xFFFFFFFFull) << 32);
    fs.h[3] = pl << 32;
    fs.h[4] = 0;
    const uint64_t hsh = xxh3_short_stream(fs);
    st64_any(out + 256 + 48 * i + po, hsh);
    es.cs[i] = hsh;
}
__global__ __launch_bounds__(256) void k_enc_short(iggy_raw_messages m, EncScratch es, uint8_t *out) {
    if (es.misc[4] < 16 || es.misc[5]) return;  // the fallback kernel encoded everything
    const uint64_t n = m.count;
    const uint64_t origin = es.misc[0];
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        enc_short_frame(m, es, out, origin, i);
}

// error precedence (send_messages.rs:131-174) and the 256-B header (64 threads)
__device__ inline void enc_finish(const iggy_raw_messages &m, EncScratch es, uint64_t partition_id, uint64_t cap,
                                  uint64_t checksum, uint8_t *out, iggy_encode_result *res, int t) {
    iggy_batch_header h = *es.hdr;
    h.batch_checksum = checksum;
    const uint64_t ts_enc = es.misc[2];
    const bool over = es.misc[5] != 0;
    uint32_t kind = IGGY_OK;
    uint64_t a = 0, b = 0;
    if (over) {  // the caller's buffer cannot hold the batch: nothing was written
        kind = IGGY_ERR_CAPACITY;
        a = h.batch_length;
        b = cap;
    } else if (ts_enc) {
        kind = IGGY_ERR_INVALID_TIMESTAMP_DELTA;
        a = m.origin_timestamps[~ts_enc] - es.misc[0];
    } else if (partition_id == 0 && h.batch_length > 0xFFFFFFFFull) {
        kind = IGGY_ERR_PAYLOAD_TOO_LARGE;
        a = h.batch_length;
        b = 0xFFFFFFFFull;
    }
    // header bytes: 64 threads x 4 bytes
    if (!over) {
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
__global__ void k_enc_finish(iggy_raw_messages m, EncScratch es, uint64_t partition_id, uint64_t cap,
                             const uint64_t *checksum, uint8_t *out, iggy_encode_result *res) {
    enc_finish(m, es, partition_id, cap, *checksum, out, res, threadIdx.x);
}

// Small unsegmented batches (at most kEncTailBlocks checksum blocks, ~8 K messages):
// block sums (4 waves, into LDS), the chain and the finish in one launch instead of
// k_bsum_blocks + k_bsum_chain + k_enc_finish.
constexpr uint32_t kEncTailBlocks = 64;
__global__ __launch_bounds__(256) void k_enc_tail_small(iggy_raw_messages m, EncScratch es, uint64_t partition_id,
                                                        uint64_t cap, uint8_t *small, uint8_t *out,
                                                        iggy_encode_result *res) {
    __shared__ uint64_t s_bs[kEncTailBlocks * 8];
    __shared__ uint64_t s_ck;
    const iggy_batch_header h = *es.hdr;
    const uint64_t N = es.misc[3];
    const CsSource src{es.cs, nullptr, nullptr};
    const CsPlan pl = cs_plan(N);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (pl.long_cs) {
        const uint64_t sec[2] = {block_word_secret(0, lane), block_word_secret(1, lane)};
        for (uint64_t b = wave; b <= pl.nb; b += 4) {  // as k_bsum_blocks
            uint64_t x = 0, y = 0;
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                const uint64_t mw = 128 * b + 64 * half + lane;
                if (mw < pl.Mreg) {
                    const uint64_t v = cs_word(mw, h, src);
                    y += v;
                    x += mul32x32(v ^ sec[half]);
                }
            }
            x += __shfl_xor(x, 8); y += __shfl_xor(y, 8);
            x += __shfl_xor(x, 16); y += __shfl_xor(y, 16);
            x += __shfl_xor(x, 32); y += __shfl_xor(y, 32);
            const uint64_t t8 = x + __shfl_xor(y, 1);
            if (lane < 8) s_bs[b * 8 + lane] = t8;
        }
    }
    __syncthreads();
    if (wave != 0) return;
    if (pl.long_cs) {  // as k_bsum_chain, from LDS
        const int j = lane & 7;
        const uint64_t key = kSecretW8[16 + j];
        const uint32_t klo = (uint32_t)key, khi = (uint32_t)(key >> 32);
        uint64_t acc = kAccInit[j];
        for (uint64_t b = 0; b < pl.nb; ++b) acc = scramble_fast(acc + s_bs[8 * b + j], klo, khi);
        acc += s_bs[pl.nb * 8 + j];
        const uint64_t v = src(N - 8 + j);
        acc += __shfl_xor(v, 1);
        acc += mul32x32(v ^ kSecretLast[j]);
        uint64_t a[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = __shfl(acc, i);
        uint64_t r = pl.n * P64_1;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            r += fold64(a[2 * i] ^ Secret::w(11 + 16 * i), a[2 * i + 1] ^ Secret::w(19 + 16 * i));
        if (lane == 0) s_ck = avalanche(r);
    } else if (lane == 0) {
        for (uint64_t mw = 0; mw < 5; ++mw) st64_any(small + 8 * mw, cs_word(mw, h, src));
        *(uint32_t *)(small + 40) = h.message_count;
        for (uint64_t i = 0; i < N; ++i) st64_any(small + 44 + 8 * i, src(i));
        s_ck = xxh3_64_lane(small, pl.n);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    enc_finish(m, es, partition_id, cap, s_ck, out, res, lane);
}

}  // namespace iggy

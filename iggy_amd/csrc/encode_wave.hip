// encode_wave.hip — the frames step of SendMessagesEncoder::encode
// (core/binary_protocol/src/requests/messages/send_messages.rs:131-181) for segmented
// batches without user headers, shaped like a copy kernel (round 6).
//
// k_enc_ring (encode.hip) hashes and stores with four fat waves per CU; its stores
// add to its time instead of hiding under the hashing. A plain copy of
// the same bytes with many light waves takes 0.78-0.82 ms against the ring's 1.36.
// Here ONE wave encodes ONE frame at a time, 16 waves per CU:
//  * instruction i of a frame covers stream block i (stream = H(40) || payload): lane l
//    loads the 16-B ALIGNED source chunk that holds stream bytes 1024 i + 16 l - r ..
//    (r = the frame's stream misalignment), and stores it, aligned, to the frame (the
//    payload and the output are 16-B congruent: P - out = 0 mod 16, checked by the host);
//  * the same chunk, funnel-shifted by r with its right neighbour (DPP wave_shl:1; lane
//    63 loads one more chunk), is stream piece 64 i + l: 16 B at the stripe-word pair
//    (2m, 2m + 1), m = l & 3, of stripe l >> 2 of block i. A lane's XXH3 contribution
//    is additive within a block, so the block's accumulators are the sum over the 16
//    lanes with the same m (DPP row rotations, then two cross-row shuffles), then the
//    scramble. Every lane holds its pair of the running accumulators.
//  * the 40 header bytes are synthesised (ids, index | timestamp delta, lengths,
//    reserved) into pieces 0-2 and stored as five 8-B words; the last stripe, the merge
//    and the avalanche follow XXH3's long form; lane 0 stores the checksum word.
// Frames of <= 240 hashed bytes are copied here and hashed by k_enc_short (XXH3's
// short forms), as with the ring. The batch checksum chain is the segments' (host_encode).
#include "codec_common.hpp"

namespace iggy {

constexpr uint32_t kEwThreads = 1024;  // 16 waves: one workgroup per CU (kEwLds keeps a second off it)
constexpr uint32_t kEwLds = 96 * 1024;  // (unused: it reserves the CU, so the grid leaves one CU to the chain)
#ifndef IGGY_EW_NOSTORE
#define IGGY_EW_NOSTORE 0  // (timing-only build knobs, wrong output: no payload stores / no hashing)
#endif
#ifndef IGGY_EW_NOHASH
#define IGGY_EW_NOHASH 0
#endif
constexpr int kEwGroup = 3;             // stream blocks whose loads are issued together

typedef uint32_t ew_v4u __attribute__((ext_vector_type(4)));

// 16 B at [a, a + 16) of the payload buffer [lo, hi): one load when inside, else the
// bytes that are inside (the buffer's first and last chunks only), zeros elsewhere
__device__ __forceinline__ uint4 ew_chunk(const uint8_t *a, const uint8_t *lo, const uint8_t *hi) {
    if (a >= lo && a + 16 <= hi) return *(const uint4 *)a;
    uint32_t w[4] = {0, 0, 0, 0};
    for (int k = 0; k < 16; ++k)
        if (a + k >= lo && a + k < hi) w[k >> 2] |= (uint32_t)a[k] << (8 * (k & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// bytes [r, r + 16) of (c || n), r in 0..15 (wave-uniform)
__device__ __forceinline__ uint4 ew_funnel(uint4 c, uint4 n, uint32_t r) {
    const uint32_t b = r & 3;
    uint32_t d0, d1, d2, d3, d4;
    switch (r >> 2) {
        case 0: d0 = c.x; d1 = c.y; d2 = c.z; d3 = c.w; d4 = n.x; break;
        case 1: d0 = c.y; d1 = c.z; d2 = c.w; d3 = n.x; d4 = n.y; break;
        case 2: d0 = c.z; d1 = c.w; d2 = n.x; d3 = n.y; d4 = n.z; break;
        default: d0 = c.w; d1 = n.x; d2 = n.y; d3 = n.z; d4 = n.w; break;
    }
    return make_uint4(__builtin_amdgcn_alignbyte(d1, d0, b), __builtin_amdgcn_alignbyte(d2, d1, b),
                      __builtin_amdgcn_alignbyte(d3, d2, b), __builtin_amdgcn_alignbyte(d4, d3, b));
}

// lane l <- lane l + 1 (DPP wave_shl:1); lane 63 keeps `last`
__device__ __forceinline__ uint32_t ew_shl1(uint32_t x, uint32_t last) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)last, (int)x, 0x130, 0xF, 0xF, false);
}

// sum over the 16 lanes with the same lane & 3: row rotations by 4 and 8 inside each
// 16-lane row, then the four rows (xor 16 by swizzle, xor 32 by permute)
__device__ __forceinline__ uint64_t ew_sum16(uint64_t x) {
    x += gdpp64<0x124>(x);  // row_ror:4
    x += gdpp64<0x128>(x);  // row_ror:8
    {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)x, 0x401F);  // xor 16
        const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)(x >> 32), 0x401F);
        x += (uint64_t)lo | ((uint64_t)hi << 32);
    }
    x += (uint64_t)__shfl_xor((unsigned long long)x, 32);
    return x;
}

// bytes [x0, x1) of the 16-B value v to the 16-B-aligned address d
__device__ inline void ew_store_range(uint8_t *d, uint4 v, uint32_t x0, uint32_t x1) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    while (x0 < x1) {
        const uint32_t dw = x0 >> 2;
        if ((x0 & 7) == 0 && x0 + 8 <= x1) {
            *(uint64_t *)(d + x0) = (uint64_t)w[dw] | ((uint64_t)w[dw + 1] << 32);
            x0 += 8;
        } else if ((x0 & 3) == 0 && x0 + 4 <= x1) {
            *(uint32_t *)(d + x0) = w[dw];
            x0 += 4;
        } else if ((x0 & 1) == 0 && x0 + 2 <= x1) {
            *(uint16_t *)(d + x0) = (uint16_t)(w[dw] >> (8 * (x0 & 3)));
            x0 += 2;
        } else {
            d[x0] = (uint8_t)(w[dw] >> (8 * (x0 & 3)));
            x0 += 1;
        }
    }
}

// A frame's geometry for the loop below.
struct EwFrame {
    uint64_t f, po, pl, L;
    uint4 ids;
    uint32_t delta, r;
    const uint8_t *A0;  // aligned source address of the chunk holding stream byte 0
    uint64_t nins;      // instructions (1-KiB stream blocks) covering every stream chunk
};
__device__ __forceinline__ EwFrame ew_frame(const uint4 *erec, uint64_t f, uint64_t n, const uint8_t *P) {
    EwFrame e;
    e.f = f;
    const bool valid = f < n;
    const uint4 rec = valid ? erec[2 * f] : make_uint4(0, 0, 0, 0);
    e.ids = valid ? erec[2 * f + 1] : make_uint4(0, 0, 0, 0);
    e.po = (uint64_t)rec.x | ((uint64_t)rec.y << 32);
    e.pl = rec.z;
    e.delta = rec.w;
    e.L = 40 + e.pl;
    const uint8_t *B0 = P + e.po - 40;
    e.r = (uint32_t)((uintptr_t)B0 & 15);
    e.A0 = B0 - e.r;
    e.nins = valid ? ((e.L - 1 + e.r) >> 10) + 1 : 0;
    return e;
}

// frames [f_lo, f_hi) of a batch without user headers; erec: k_enc_recs' records
// (erec[2 i] = {po lo, po hi, payload length, timestamp delta}, erec[2 i + 1] = ids).
// A wave's frames are f_lo + wave + k nwaves. The first kEwGroup blocks of the NEXT
// frame are loaded before the current frame is hashed and stored, so a wave keeps two
// frames' loads in flight; the blocks past a frame's first kEwGroup load when reached.
// Lane 63's right neighbour is lane 0 of the next block's chunk (a readlane), or, for a
// group's last block, one more chunk loaded by lane 63.
__global__ __launch_bounds__(kEwThreads, 1) void k_enc_wave(iggy_raw_messages m, EncScratch es, uint8_t *out,
                                                           uint64_t f_lo, uint64_t f_hi, const uint4 *erec) {
    const uint64_t ptot = es.misc[4];
    if (ptot < 16 || es.misc[5]) return;  // tiny payload area (k_enc_frames) or over capacity
    const uint64_t n = f_hi < m.count ? f_hi : m.count;
    const int lane = threadIdx.x & 63;
    const uint32_t l = (uint32_t)lane, mm = l & 3;
    const uint64_t wave = (uint64_t)blockIdx.x * (kEwThreads / 64) + (threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * (kEwThreads / 64);
    const uint8_t *P = m.payloads, *Pend = m.payloads + ptot;
    // this lane's secrets: stripe l >> 2 of a block, word pair mm
    const uint64_t s0 = kSecretW8[(l >> 2) + 2 * mm], s1 = kSecretW8[(l >> 2) + 2 * mm + 1];
    const uint64_t key0 = kSecretW8[16 + 2 * mm], key1 = kSecretW8[17 + 2 * mm];
    const uint64_t init0 = kAccInit[2 * mm], init1 = kAccInit[2 * mm + 1];
    const uint64_t last0 = kSecretLast[2 * mm], last1 = kSecretLast[2 * mm + 1];
    const uint64_t mrg0 = kSecretMerge[2 * mm], mrg1 = kSecretMerge[2 * mm + 1];
    // a group of blocks [i0, i0 + kEwGroup) of frame fr: chunks c, lane 63's extra chunk e
    auto load_group = [&](const EwFrame &fr, uint64_t i0, uint4 (&c)[kEwGroup], uint4 &e) {
#pragma unroll
        for (int g = 0; g < kEwGroup; ++g) {
            const bool in = i0 + g < fr.nins;
            c[g] = in ? ew_chunk(fr.A0 + 1024 * (i0 + g) + 16 * l, P, Pend) : make_uint4(0, 0, 0, 0);
        }
        const bool ex = l == 63 && i0 + kEwGroup < fr.nins;
        e = ex ? ew_chunk(fr.A0 + 1024 * (i0 + kEwGroup), P, Pend) : make_uint4(0, 0, 0, 0);
    };
    // one frame: its header words, the copy of every stream chunk, the hash; c / e hold
    // its first kEwGroup blocks' loads (issued earlier)
    auto process = [&](const EwFrame &cur, uint4 (&cc)[kEwGroup], uint4 &ce) {
        const uint64_t f = cur.f, po = cur.po, pl = cur.pl, L = cur.L;
        const uint32_t r = cur.r;
        const uint8_t *A0 = cur.A0;
        uint8_t *F = out + 256 + 48 * f + po;  // the frame
        const int64_t D = (int64_t)((F + 8) - (A0 + r));  // source -> frame offset of every stream byte (= 0 mod 16)
        // the header words: stream bytes 0..39 (ids, index | delta, user-headers length | payload length, reserved)
        const uint64_t hw0 = (uint64_t)cur.ids.x | ((uint64_t)cur.ids.y << 32);
        const uint64_t hw1 = (uint64_t)cur.ids.z | ((uint64_t)cur.ids.w << 32);
        const uint64_t hw2 = (f & 0xFFFFFFFFull) | ((uint64_t)cur.delta << 32), hw3 = pl << 32;
        if (l < 5) st64_any(F + 8 + 8 * l, l == 0 ? hw0 : l == 1 ? hw1 : l == 2 ? hw2 : l == 3 ? hw3 : 0ull);
        const bool lng = L > 240;
        const uint64_t nbF = lng ? (L - 1) >> 10 : 0, ns = lng ? ((L - 1) & 1023) >> 6 : 0;
        uint64_t a0 = init0, a1 = init1;
        for (uint64_t i0 = 0; i0 < cur.nins; i0 += kEwGroup) {
            if (i0) load_group(cur, i0, cc, ce);  // (frames of more than kEwGroup blocks)
#pragma unroll
            for (int g = 0; g < kEwGroup; ++g) {
                const uint64_t i = i0 + g;
                if (i >= cur.nins) break;  // (wave-uniform)
                // the copy: stream bytes [s, s + 16) of this chunk, those in [40, L)
                const int64_t s = (int64_t)(1024 * i + 16 * l) - (int64_t)r;
                const int64_t x0 = s < 40 ? 40 - s : 0, x1 = (int64_t)L - s < 16 ? (int64_t)L - s : 16;
                uint8_t *d = (uint8_t *)(A0 + 1024 * i + 16 * l) + D;
                if (!IGGY_EW_NOSTORE) {
                    if (x0 == 0 && x1 == 16) *(uint4 *)d = cc[g];
                    else if (x0 < x1) ew_store_range(d, cc[g], (uint32_t)x0, (uint32_t)x1);
                }
                if (IGGY_EW_NOHASH || !lng || i > nbF || (i == nbF && ns == 0)) continue;  // nothing hashed in this block
                // stream piece 64 i + l: this chunk and its right neighbour
                uint4 nb4;
                if (g + 1 < kEwGroup) {
                    const uint4 z = cc[g + 1];  // (lane 0 of the next block's chunk, for lane 63)
                    nb4 = make_uint4(ew_shl1(cc[g].x, __builtin_amdgcn_readlane(z.x, 0)),
                                     ew_shl1(cc[g].y, __builtin_amdgcn_readlane(z.y, 0)),
                                     ew_shl1(cc[g].z, __builtin_amdgcn_readlane(z.z, 0)),
                                     ew_shl1(cc[g].w, __builtin_amdgcn_readlane(z.w, 0)));
                } else {
                    nb4 = make_uint4(ew_shl1(cc[g].x, ce.x), ew_shl1(cc[g].y, ce.y), ew_shl1(cc[g].z, ce.z),
                                     ew_shl1(cc[g].w, ce.w));
                }
                const uint4 p = ew_funnel(cc[g], nb4, r);
                uint64_t w0 = (uint64_t)p.x | ((uint64_t)p.y << 32), w1 = (uint64_t)p.z | ((uint64_t)p.w << 32);
                if (i == 0 && l < 3) {  // stream bytes 0..47: the header words (piece 2: reserved | payload 0..7)
                    w0 = l == 0 ? hw0 : l == 1 ? hw2 : 0ull;
                    w1 = l == 0 ? hw1 : l == 1 ? hw3 : w1;
                }
                const bool full = i < nbF;
                const uint64_t use = 0ull - (uint64_t)(full || (uint64_t)(l >> 2) < ns);
                a0 += ew_sum16((mul32x32(w0 ^ s0) + w1) & use);
                a1 += ew_sum16((mul32x32(w1 ^ s1) + w0) & use);
                if (full) {
                    a0 = scramble1(a0, key0);
                    a1 = scramble1(a1, key1);
                }
            }
        }
        if (lng) {
            // the last stripe: stream bytes [L - 64, L), piece q in lane q < 4
            const uint8_t *ls = A0 + r + L - 64;
            const uint32_t rl = (uint32_t)((uintptr_t)ls & 15);
            const uint8_t *la = ls - rl + 16 * l;
            const uint4 lc = l < 4 ? ew_chunk(la, P, Pend) : make_uint4(0, 0, 0, 0);
            const uint4 ln = l < 4 ? ew_chunk(la + 16, P, Pend) : make_uint4(0, 0, 0, 0);
            const uint4 p = ew_funnel(lc, ln, rl);
            const uint64_t w0 = (uint64_t)p.x | ((uint64_t)p.y << 32), w1 = (uint64_t)p.z | ((uint64_t)p.w << 32);
            const uint64_t use = 0ull - (uint64_t)(l < 4);
            a0 += ew_sum16((mul32x32(w0 ^ last0) + w1) & use);
            a1 += ew_sum16((mul32x32(w1 ^ last1) + w0) & use);
            // merge: lanes 0..3 hold pairs m = 0..3
            uint64_t t = fold64(a0 ^ mrg0, a1 ^ mrg1);
            t += gdpp64<0xB1>(t);  // quad_perm [1,0,3,2]
            t += gdpp64<0x4E>(t);  // quad_perm [2,3,0,1]
            const uint64_t h = avalanche(L * P64_1 + t);
            if (l == 0) {
                st64_any(F, h);
                es.cs[f] = h;
            }
        }
    };
    // The next frame's first blocks load while this one is processed, and the frame
    // records (k_enc_recs) load two frames further ahead: a record is a dependent round
    // trip in front of its frame's data loads.
    uint64_t f = f_lo + wave;
    EwFrame fa = ew_frame(erec, f, n, P);
    EwFrame fb = ew_frame(erec, f + nwaves, n, P);
    uint4 ca[kEwGroup], ea;
    load_group(fa, 0, ca, ea);
    while (f < n) {
        const EwFrame fc = ew_frame(erec, f + 2 * nwaves, n, P);  // (records, two frames ahead)
        uint4 cb[kEwGroup], eb;
        load_group(fb, 0, cb, eb);  // (the next frame's data, in flight while this one is processed)
        process(fa, ca, ea);
        f += nwaves;
        fa = fb;
        fb = fc;
#pragma unroll
        for (int g = 0; g < kEwGroup; ++g) ca[g] = cb[g];
        ea = eb;
    }
}

}  // namespace iggy

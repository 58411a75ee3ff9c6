// decode_general.hip — decode_batch_slice_with (core/binary_protocol/src/batch.rs:391-527)
// for records with arbitrary frame sizes: the exact serial walk of
// BatchIteratorWithOffsets (batch.rs:329-355) rebuilt in parallel.
//
// One persistent launch (grid = every co-resident WG, bounded grid barriers)
// that returns immediately unless the uniform-stride kernel left
// result->status == kStatusNeedGeneral. The blob is cut into tiles of
// T = 2^sh bytes, sized from the header's message count to hold ~8 frames
// (4 KiB <= T <= 1 MiB); tiles form groups of 64. Phases:
//   A  locate : one lane per tile finds the first candidate frame start (8 zero
//               reserved bytes at +40 and lengths inside the blob; 256-B vector
//               scan for a zero dword) and walks the candidate chain from it
//               until it leaves the tile: start s_t, exit x_t, count cnt_t.
//   B1 groups : one wave per group: is the group self-consistent when entered at
//               its first start (every later tile entered at its own start, or
//               spanned by one frame when it has none)? -> (S, X, CNT, ok, term).
//   B2 link   : one wave chains groups from offset 0, 64 per ballot step; a
//               group that is not entered at S or is not self-consistent is
//               linked tile by tile (spans skipped, entries re-walked). The
//               result is exactly the reference walk: true frame starts are
//               always candidates and the first non-candidate ends the walk.
//   C  scatter: one lane per accepted tile re-walks from its true entry: frame
//               positions and stored checksums in walk order.
//   E  sums   : XXH3 stripe sums of the batch-checksum input, one wave / block.
//   D + F     : wave 0 of WG 0 runs the serial scramble chain over the block
//               sums while every other wave verifies frames, eight per wave
//               (8 lanes per frame, 16 B per lane per stripe pair); then
//               precedence resolution and the result.
#include "codec_common.hpp"

namespace iggy {

constexpr uint32_t kTileShiftMin = 12, kTileShiftMax = 20;
constexpr uint64_t kTileMin = 1ull << kTileShiftMin;  // host sizing unit
constexpr uint64_t kNoStart = ~0ull;
constexpr uint64_t kStopBit = 1ull << 63;
constexpr uint32_t kGrpWords = 6;  // S, X, CNT, flags | base, mode
constexpr uint64_t kGrpOk = 1, kGrpTerm = 2;

struct GeneralScratch {
    uint64_t *tile_s;    // [ntiles] first candidate start (blob offset) or kNoStart
    uint64_t *tile_x;    // [ntiles] exit position (| kStopBit when the walk stopped inside)
    uint32_t *tile_cnt;  // [ntiles] frames on the candidate chain inside the tile
    uint64_t *tile_e;    // [ntiles] repaired groups: true entry (~0: no frame starts here)
    uint64_t *tile_base; // [ntiles] repaired groups: frames before the tile
    uint64_t *grp;       // [ngroups * kGrpWords]
    uint64_t *fpos;      // [max_frames] frame starts in walk order
    uint64_t *cs;        // [max_frames] stored checksums in walk order
    uint64_t *bsums;     // [max_blocks * 8]
    uint64_t *misc;      // [16]: 0 nwalk, 1 end (with stop bit), 2 first_bad enc
    uint32_t *bar;       // [4]: arrive counter, exit counter
    uint8_t *small;      // >= 512 B
    uint64_t ntiles, max_frames, max_blocks;  // ntiles: capacity in kTileMin tiles
};

// ---------------------------------------------------------------- helpers
__device__ __forceinline__ bool candidate(const uint8_t *blob, uint64_t bl, uint64_t p,
                                          uint64_t *end) {
    if (p >= bl || bl - p < kFrameHdr) return false;
    const uint4 w = ld128_any(blob + p + 32);  // lengths at +32/+36, reserved at +40
    if ((w.z | w.w) != 0) return false;
    const uint64_t e = p + kFrameHdr + (uint64_t)w.x + w.y;
    if (e > bl) return false;
    *end = e;
    return true;
}

// grid barrier: monotonic arrive counter, agent release/acquire, bounded
__device__ bool grid_barrier(uint32_t *bar, uint32_t target, uint64_t t0) {
    __syncthreads();
    bool ok = true;
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(2);
            if (rt_now() - t0 > kSpinLimitTicks) { ok = false; break; }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    return ok;
}

// phase clock (diagnostics): WG 0 stamps the ticks since entry after every
// barrier at small+512 (u64 [1..6]); [8..] are counters of the link phase
__device__ __forceinline__ void gstamp(const GeneralScratch &gs, int idx, uint64_t v) {
    if (blockIdx.x == 0 && threadIdx.x == 0) ((uint64_t *)(gs.small + 512))[idx] = v;
}

// tile size: ~8 frames of the header's average size, a power of two in range
__device__ __forceinline__ uint32_t tile_shift(uint64_t bl, uint32_t message_count) {
    const uint64_t want = 8 * (message_count ? bl / message_count : bl);
    uint32_t sh = kTileShiftMin;
    while (sh < kTileShiftMax && (1ull << sh) < want) ++sh;
    return sh;
}

// walk the candidate chain from p while p < hi (hi <= bl); EMIT writes every
// frame's position (and stored checksum) at index base + k
template <bool EMIT, bool CS>
__device__ inline uint32_t walk(const uint8_t *blob, uint64_t bl, uint64_t p, uint64_t hi,
                                uint64_t *x_out, uint64_t base = 0, uint64_t *fpos = nullptr,
                                uint64_t *cs = nullptr, uint64_t *frame_pos = nullptr,
                                uint64_t cap = 0) {
    uint32_t cnt = 0;
    while (p < hi) {
        uint64_t e;
        if (!candidate(blob, bl, p, &e)) {
            *x_out = p | kStopBit;
            return cnt;
        }
        if (EMIT) {
            const uint64_t i = base + cnt;
            fpos[i] = p;
            if (CS) cs[i] = ld64_any(blob + p);
            if (frame_pos && i < cap) frame_pos[i] = p;
        }
        ++cnt;
        p = e;
    }
    *x_out = p;  // >= hi (== bl: clean end)
    return cnt;
}

// Test the candidate window starts whose 8-byte reserved window [ws, ws+8)
// contains the zero dword at aligned address ad (ws in [ad-3, ad]), increasing.
__device__ __forceinline__ bool dword_candidates(const uint8_t *blob, uint64_t bl, uint64_t lo,
                                                 uint64_t hi, uintptr_t ad, uint64_t *out) {
    const uintptr_t base = (uintptr_t)blob;
    for (int d = 3; d >= 0; --d) {
        const uintptr_t ws = ad - d;  // window start = blob + p + 40
        if (ws < base + lo + 40) continue;
        const uint64_t p = (uint64_t)(ws - base) - 40;
        if (p >= hi) return false;
        uint64_t e;
        if (candidate(blob, bl, p, &e)) {
            *out = p;
            return true;
        }
    }
    return false;
}

// First candidate start in [lo, hi) (hi <= bl). An all-zero reserved window at
// p+40 contains the aligned dword at 4*ceil((p+40)/4), so scanning aligned
// dwords for zeros in increasing order finds every candidate in order. The scan
// reads 256 B per step with 16 independent 16-B loads.
__device__ inline uint64_t first_candidate(const uint8_t *blob, uint64_t bl, uint64_t lo,
                                           uint64_t hi) {
    if (lo >= hi) return kNoStart;
    const uintptr_t base = (uintptr_t)blob;
    const uintptr_t a_end = base + hi + 43;  // dwords holding a window of some p < hi
    const uintptr_t blob_end = base + bl;
    uintptr_t a = (base + lo + 40) & ~(uintptr_t)15;
    uint64_t p;
    while (a < a_end && a + 256 <= blob_end) {
        uint4 v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = *(const uint4 *)(a + 16 * k);
        uint64_t zmask = 0;  // bit 4k+q: dword q of v[k] is zero
#pragma unroll
        for (int k = 0; k < 16; ++k)
            zmask |= (uint64_t)((v[k].x == 0) | ((v[k].y == 0) << 1) | ((v[k].z == 0) << 2) |
                                ((v[k].w == 0) << 3)) << (4 * k);
        while (zmask) {
            const int bit = __builtin_ctzll(zmask);
            zmask &= zmask - 1;
            const uintptr_t ad = a + 4 * bit;
            if (ad >= a_end) return kNoStart;
            if (dword_candidates(blob, bl, lo, hi, ad, &p)) return p;
        }
        a += 256;
    }
    for (; a < a_end && a + 4 <= blob_end; a += 4)
        if (*(const uint32_t *)a == 0 && dword_candidates(blob, bl, lo, hi, a, &p)) return p;
    return kNoStart;
}

// The tile's speculative entry. Frame headers themselves hold zero runs
// (timestamp delta, user-header length, the high bytes of a small offset
// delta) that pass the reserved-bytes test a few bytes BEFORE a true start,
// with random "lengths" that usually still fit the blob. So rather than the
// first candidate, take the first of up to kPickTries candidates whose chain is
// confirmed (its successor starts inside the tile and the chain leaves the tile
// cleanly); failing that, the clean chain with the nearest exit, else the first
// candidate. Only speed depends on this choice: the link phase re-walks any tile
// whose pick disagrees with the true entry.
constexpr int kPickTries = 8;
__device__ inline void pick_start(const uint8_t *blob, uint64_t bl, uint64_t lo, uint64_t hi,
                                  uint64_t *s_out, uint64_t *x_out, uint32_t *cnt_out) {
    uint64_t bs = kNoStart, bx = kNoStart;
    uint32_t bc = 0;
    bool bclean = false;
    uint64_t from = lo;
    for (int k = 0; k < kPickTries; ++k) {
        const uint64_t c = first_candidate(blob, bl, from, hi);
        if (c == kNoStart) break;
        uint64_t x;
        const uint32_t n = walk<false, false>(blob, bl, c, hi, &x);
        const bool clean = !(x & kStopBit);
        if (clean && n >= 2) {
            bs = c; bx = x; bc = n;
            break;
        }
        if (bs == kNoStart || (clean && (!bclean || x < bx))) {
            bs = c; bx = x; bc = n; bclean = clean;
        }
        from = c + 1;
    }
    *s_out = bs;
    *x_out = bx;
    *cnt_out = bc;
}

// XXH3 stripe contribution of checksum-input word m (value v)
__device__ __forceinline__ void word_contrib(uint64_t m, uint64_t v, uint64_t &x, uint64_t &y) {
    // x -> acc[j], y -> acc[j^1]
    const uint32_t j = (uint32_t)(m & 7), sib = (uint32_t)((m >> 3) & 15);
    y = v;
    x = mul32x32(v ^ kSecretW8[sib + j]);
}

template <int CTRL>
__device__ __forceinline__ uint64_t gdpp64(uint64_t x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)x, CTRL, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(x >> 32), CTRL, 0xF, 0xF, false);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
__device__ __forceinline__ uint64_t gswz_xor4(uint64_t x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)x, 0x101F);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)(x >> 32), 0x101F);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
__device__ __forceinline__ void piece(uint64_t &a0, uint64_t &a1, uint4 p, uint64_t s0, uint64_t s1) {
    const uint64_t w0 = (uint64_t)p.x | ((uint64_t)p.y << 32);
    const uint64_t w1 = (uint64_t)p.z | ((uint64_t)p.w << 32);
    a0 += mul32x32(w0 ^ s0) + w1;
    a1 += mul32x32(w1 ^ s1) + w0;
}

// Frame verification, 8 frames per wave step: lane group fg (8 lanes) hashes
// frame 8k+fg of the walk. Lane l = (m, par) owns accumulators 2m, 2m+1 for the
// stripes of parity par: in every 1024-B block it reads the 16 B at
// 128q + 16(m + 4 par), q = 0..7 (stripe 2q+par, words 2m, 2m+1). The pair of
// parity lanes is folded before each scramble; the last stripe and merge follow
// the XXH3 long form (> 240 B). Shorter frames are hashed by one lane.
__device__ inline void verify_frames(const uint8_t *blob, const GeneralScratch &gs, uint64_t nwalk,
                                     uint32_t vw, uint32_t nvw, int lane) {
    const uint32_t l = lane & 7, m = l >> 1, par = l & 1, fg = (uint32_t)lane >> 3;
    const uint32_t poff = 16 * (m + 4 * par);
    uint64_t s0[8], s1[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        s0[q] = kSecretW8[2 * q + par + 2 * m];
        s1[q] = kSecretW8[2 * q + par + 2 * m + 1];
    }
    const uint64_t key0 = kSecretW8[16 + 2 * m], key1 = kSecretW8[17 + 2 * m];
    const uint64_t init0 = par ? 0 : kAccInit[2 * m], init1 = par ? 0 : kAccInit[2 * m + 1];
    const uint64_t last0 = kSecretLast[2 * m], last1 = kSecretLast[2 * m + 1];
    const uint64_t mrg0 = kSecretMerge[2 * m], mrg1 = kSecretMerge[2 * m + 1];
    for (uint64_t k = vw; 8 * k < nwalk; k += nvw) {
        const uint64_t f = 8 * k + fg;
        const bool valid = f < nwalk;
        const uint64_t p = valid ? gs.fpos[f] : 0;
        const uint64_t stored = valid ? gs.cs[f] : 0;
        const uint64_t lens = ld64_any(blob + p + 32);
        const uint64_t L = 40 + (uint64_t)(uint32_t)lens + (lens >> 32);
        const bool lng = valid && L > 240;
        const uint64_t nbF = lng ? (L - 1) / 1024 : 0;
        const uint64_t ns = lng ? ((L - 1) - 1024 * nbF) / 64 : 0;
        const uint32_t nsteps = (uint32_t)(nbF + (ns > 0));
        uint32_t maxs = nsteps;
        maxs = max(maxs, (uint32_t)__shfl_xor((int)maxs, 8));
        maxs = max(maxs, (uint32_t)__shfl_xor((int)maxs, 16));
        maxs = max(maxs, (uint32_t)__shfl_xor((int)maxs, 32));
        const uint8_t *hb = blob + p + 8 + poff;
        uint64_t a0 = init0, a1 = init1;
        uint4 cur[8];
        if (nsteps > 0) {
#pragma unroll
            for (int q = 0; q < 8; ++q)
                cur[q] = (nbF > 0 || 2 * q + par < ns) ? ld128_any(hb + 128 * q) : make_uint4(0, 0, 0, 0);
        }
        for (uint32_t b = 0; b < maxs; ++b) {
            if (b < nsteps) {
                uint4 nxt[8];
                const uint32_t b1 = b + 1;
                if (b1 < nsteps) {
                    const uint8_t *nb = hb + 1024ull * b1;
#pragma unroll
                    for (int q = 0; q < 8; ++q)
                        nxt[q] = (b1 < nbF || 2 * q + par < ns) ? ld128_any(nb + 128 * q) : make_uint4(0, 0, 0, 0);
                }
                if (b < nbF) {
                    uint64_t p0[4] = {0, 0, 0, 0}, p1[4] = {0, 0, 0, 0};
#pragma unroll
                    for (int q = 0; q < 8; ++q) piece(p0[q & 3], p1[q & 3], cur[q], s0[q], s1[q]);
                    a0 += (p0[0] + p0[1]) + (p0[2] + p0[3]);
                    a1 += (p1[0] + p1[1]) + (p1[2] + p1[3]);
                    a0 += gdpp64<0xB1>(a0);
                    a1 += gdpp64<0xB1>(a1);
                    a0 = scramble1(a0, key0);
                    a1 = scramble1(a1, key1);
                    if (par) { a0 = 0; a1 = 0; }
                } else {
#pragma unroll
                    for (int q = 0; q < 8; ++q)
                        if (2 * q + par < ns) piece(a0, a1, cur[q], s0[q], s1[q]);
                }
                if (b1 < nsteps) {
#pragma unroll
                    for (int q = 0; q < 8; ++q) cur[q] = nxt[q];
                }
            }
        }
        uint64_t h = 0;
        if (lng) {
            a0 += gdpp64<0xB1>(a0);
            a1 += gdpp64<0xB1>(a1);
            piece(a0, a1, ld128_any(blob + p + 8 + L - 64 + 16 * m), last0, last1);
            uint64_t t = fold64(a0 ^ mrg0, a1 ^ mrg1);
            t += gdpp64<0x4E>(t);
            t += gswz_xor4(t);
            h = avalanche(L * P64_1 + t);
        } else if (valid && l == 0) {
            h = xxh3_64_lane(blob + p + 8, L);
        }
        if (valid && l == 0 && h != stored)
            atomicMax((unsigned long long *)&gs.misc[2], (unsigned long long)~f);
    }
}

// ------------------------------------------------------------------ kernel
template <bool VERIFY>
__global__ __launch_bounds__(256) void k_decode_general(const uint8_t *__restrict__ body,
                                                        uint64_t len, uint64_t *frame_pos,
                                                        uint64_t cap, iggy_decode_result *result,
                                                        GeneralScratch gs) {
    if (__hip_atomic_load(&result->status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) !=
        kStatusNeedGeneral)
        return;
    const uint64_t t0 = rt_now();
    const iggy_batch_header h = result->header;
    const uint8_t *blob = body + kHdr;
    const uint64_t bl = h.batch_length - kHdr;
    const uint32_t sh = tile_shift(bl, h.message_count);
    const uint64_t T = 1ull << sh;
    const uint64_t ntiles = (bl + T - 1) >> sh;
    const uint64_t ngroups = (ntiles + 63) / 64;
    const uint32_t nwg = gridDim.x;
    const uint64_t gtid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t gthreads = (uint64_t)nwg * blockDim.x;
    const int lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    const uint64_t wid = gtid >> 6, nwaves = gthreads >> 6;
    uint32_t phase = 0;
    bool ok = true;

    // ---------------- A: locate
    for (uint64_t t = gtid; t < ntiles; t += gthreads) {
        const uint64_t lo = t << sh, hi = min(lo + T, bl);
        uint64_t s = kNoStart, x = kNoStart;
        uint32_t cnt = 0;
        if (t == 0) {
            s = 0;
            cnt = walk<false, false>(blob, bl, 0, hi, &x);
        } else {
            pick_start(blob, bl, lo, hi, &s, &x, &cnt);
        }
        gs.tile_s[t] = s;
        gs.tile_cnt[t] = cnt;
        gs.tile_x[t] = x;
    }
    ok &= grid_barrier(gs.bar, nwg * ++phase, t0);
    gstamp(gs, 1, rt_now() - t0);

    // ---------------- B1: group summaries (one wave per 64 tiles)
    for (uint64_t g = wid; g < ngroups; g += nwaves) {
        const uint64_t t = 64 * g + lane;
        const bool in = t < ntiles;
        const uint64_t s = in ? gs.tile_s[t] : kNoStart;
        const uint64_t x = in ? gs.tile_x[t] : 0;
        const uint32_t cnt = in ? gs.tile_cnt[t] : 0;
        const bool has = s != kNoStart;
        const uint64_t termmask = __ballot(has && ((x & kStopBit) || x >= bl));
        const int last = termmask ? __builtin_ctzll(termmask) : 63;
        const uint64_t hasmask = __ballot(has && lane <= last);
        uint64_t S = kNoStart, X = 0, CNT = 0, flags = kGrpOk;
        if (hasmask) {
            const int f0 = __builtin_ctzll(hasmask);
            const int lh = 63 - __builtin_clzll(hasmask);
            // predecessor exit of lane l: max exit over the group's live starts before l
            uint64_t pm = (has && lane <= last) ? x : 0;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint64_t o = __shfl_up(pm, d);
                if (lane >= d) pm = max(pm, o);
            }
            uint64_t pred = __shfl_up(pm, 1);
            const uint64_t hi_t = min((t + 1) << sh, bl);
            const bool okl = !in || lane <= f0 || lane > last || (has ? s == pred : pred >= hi_t);
            if (__ballot(!okl)) flags = 0;
            uint64_t c = (has && lane <= last) ? cnt : 0;
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d);
            S = __shfl(s, f0);
            X = __shfl(x, lh);
            CNT = c;
            if (termmask) flags |= kGrpTerm;
        }
        if (lane == 0) {
            uint64_t *q = gs.grp + kGrpWords * g;
            q[0] = S; q[1] = X; q[2] = CNT; q[3] = flags;
        }
    }
    ok &= grid_barrier(gs.bar, nwg * ++phase, t0);
    gstamp(gs, 2, rt_now() - t0);

    // ---------------- B2: link (one wave)
    if (blockIdx.x == 0 && wave == 0) {
        uint64_t e = 0;      // true entry into the next group
        uint64_t total = 0;  // frames accepted so far
        bool ended = false;  // the walk stopped (stop bit) or reached the blob end
        uint64_t nfast = 0, nsum = 0, nspan = 0, nrep = 0;  // diagnostics
        for (uint64_t G0 = 0; G0 < ngroups; G0 += 64) {
            const uint64_t g = G0 + lane;
            const bool in = g < ngroups;
            uint64_t *q = gs.grp + kGrpWords * g;
            if (ended) {
                if (in) q[5] = 0;
                continue;
            }
            const uint64_t S = in ? q[0] : kNoStart, X = in ? q[1] : 0, CNT = in ? q[2] : 0;
            const uint64_t flags = in ? q[3] : 0;
            const bool has = S != kNoStart;
            const uint64_t termmask = __ballot(in && has && (flags & kGrpTerm));
            const int last = termmask ? __builtin_ctzll(termmask) : 63;
            uint64_t pm = (in && has && lane <= last) ? X : 0;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint64_t o = __shfl_up(pm, d);
                if (lane >= d) pm = max(pm, o);
            }
            uint64_t pred = __shfl_up(pm, 1);
            if (lane == 0) pred = 0;
            pred = max(pred, e);
            const uint64_t ghi = min(min(64 * (g + 1), ntiles) << sh, bl);
            const bool okl = !in || lane > last || ((flags & kGrpOk) && (has ? S == pred : pred >= ghi));
            if (__ballot(!okl) == 0) {
                const uint64_t c = (in && has && lane <= last) ? CNT : 0;
                uint64_t inc = c;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint64_t o = __shfl_up(inc, d);
                    if (lane >= d) inc += o;
                }
                if (in) {
                    q[4] = total + inc - c;
                    q[5] = (has && lane <= last) ? 1 : 0;
                }
                total += __shfl(inc, 63);
                ++nfast;
                if (termmask) {
                    e = __shfl(X, last);
                    ended = true;
                } else {
                    e = max(e, __shfl(pm, 63));
                }
                continue;
            }
            // exact sequential rule, group by group
            for (int l = 0; l < 64; ++l) {
                const uint64_t gg = G0 + l;
                if (gg >= ngroups) break;
                const uint64_t Sl = __shfl(S, l), Xl = __shfl(X, l), Cl = __shfl(CNT, l);
                const uint64_t Fl = __shfl(flags, l);
                const uint64_t ghl = __shfl(ghi, l);
                uint64_t *ql = gs.grp + kGrpWords * gg;
                if (ended) {
                    if (lane == 0) ql[5] = 0;
                    continue;
                }
                if ((Fl & kGrpOk) && Sl != kNoStart && Sl == e) {
                    if (lane == 0) { ql[4] = total; ql[5] = 1; }
                    total += Cl;
                    ++nsum;
                    e = Xl;
                    if (Fl & kGrpTerm) ended = true;
                    continue;
                }
                if ((Fl & kGrpOk) && Sl == kNoStart && e >= ghl) {
                    if (lane == 0) ql[5] = 0;  // one frame spans the whole group
                    ++nspan;
                    continue;
                }
                // tile by tile
                const uint64_t t = 64 * gg + lane;
                const bool tin = t < ntiles;
                const uint64_t ts = tin ? gs.tile_s[t] : kNoStart, tx = tin ? gs.tile_x[t] : 0;
                const uint32_t tc = tin ? gs.tile_cnt[t] : 0;
                for (int u = 0; u < 64; ++u) {
                    const uint64_t tt = 64 * gg + u;
                    if (tt >= ntiles) break;
                    const uint64_t su = __shfl(ts, u), xu = __shfl(tx, u);
                    const uint32_t cu = __shfl(tc, u);
                    if (lane == 0) {
                        const uint64_t hi = min((tt + 1) << sh, bl);
                        uint64_t te = ~0ull;
                        if (!ended && e < hi) {
                            te = e;
                            gs.tile_base[tt] = total;
                            if (e == su) {
                                total += cu;
                                e = xu;
                            } else {
                                uint64_t x2;
                                total += walk<false, false>(blob, bl, e, hi, &x2);
                                e = x2;
                            }
                            if ((e & kStopBit) || e >= bl) ended = true;
                        }
                        gs.tile_e[tt] = te;
                    }
                    e = __shfl(e, 0);
                    total = __shfl(total, 0);
                    ended = __shfl((int)ended, 0) != 0;
                }
                if (lane == 0) ql[5] = 2;
                ++nrep;
            }
        }
        if (lane == 0) {
            uint64_t *st = (uint64_t *)(gs.small + 512);
            st[8] = nfast; st[9] = nsum; st[10] = nspan; st[11] = nrep; st[12] = ntiles; st[13] = sh;
            __hip_atomic_store(&gs.misc[0], total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&gs.misc[1], e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    ok &= grid_barrier(gs.bar, nwg * ++phase, t0);
    gstamp(gs, 3, rt_now() - t0);

    const uint64_t nwalk = __hip_atomic_load(&gs.misc[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // ---------------- C: scatter frame positions (walk order), one wave per group
    for (uint64_t g = wid; g < ngroups; g += nwaves) {
        const uint64_t *q = gs.grp + kGrpWords * g;
        const uint64_t mode = q[5];
        if (mode == 0) continue;
        const uint64_t t = 64 * g + lane;
        const bool in = t < ntiles;
        uint64_t entry = ~0ull, base = 0;
        if (mode == 1) {
            const uint64_t s = in ? gs.tile_s[t] : kNoStart;
            const uint64_t x = in ? gs.tile_x[t] : 0;
            const uint32_t cnt = in ? gs.tile_cnt[t] : 0;
            const bool has = s != kNoStart;
            const uint64_t termmask = __ballot(has && ((x & kStopBit) || x >= bl));
            const int last = termmask ? __builtin_ctzll(termmask) : 63;
            const bool live = has && lane <= last;
            const uint64_t c = live ? cnt : 0;
            uint64_t inc = c;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint64_t o = __shfl_up(inc, d);
                if (lane >= d) inc += o;
            }
            if (live) { entry = s; base = q[4] + inc - c; }
        } else if (in) {
            entry = gs.tile_e[t];
            if (entry != ~0ull) base = gs.tile_base[t];
        }
        if (entry != ~0ull) {
            uint64_t x;
            walk<true, VERIFY>(blob, bl, entry, min((t + 1) << sh, bl), &x, base, gs.fpos, gs.cs,
                               frame_pos, cap);
        }
    }
    ok &= grid_barrier(gs.bar, nwg * ++phase, t0);
    gstamp(gs, 4, rt_now() - t0);

    // ---------------- E: checksum-input block sums (one wave per block)
    const uint64_t n = 44 + 8 * nwalk;
    const bool long_cs = VERIFY && n > 240;
    uint64_t nb = 0, Mreg = 0;
    if (long_cs) {
        nb = (n - 1) / 1024;
        const uint64_t ns = ((n - 1) - 1024 * nb) / 64;
        Mreg = 8 * (16 * nb + ns);
        for (uint64_t b = wid; b <= nb; b += nwaves) {
            uint64_t x = 0, y = 0;
            for (int half = 0; half < 2; ++half) {
                const uint64_t mw = 128 * b + 64 * half + lane;
                if (mw < Mreg) {
                    uint64_t v;
                    if (mw < 5) {
                        v = mw == 0 ? h.partition_id : mw == 1 ? h.base_offset : mw == 2 ? h.base_timestamp
                                                      : mw == 3 ? h.origin_timestamp : h.batch_length;
                    } else if (mw == 5) {
                        v = (uint64_t)h.message_count | (gs.cs[0] << 32);
                    } else {
                        v = (gs.cs[mw - 6] >> 32) | (gs.cs[mw - 5] << 32);
                    }
                    uint64_t xx, yy;
                    word_contrib(mw, v, xx, yy);
                    x += xx;
                    y += yy;
                }
            }
            x += __shfl_xor(x, 8); y += __shfl_xor(y, 8);
            x += __shfl_xor(x, 16); y += __shfl_xor(y, 16);
            x += __shfl_xor(x, 32); y += __shfl_xor(y, 32);
            const uint64_t t8 = x + __shfl_xor(y, 1);
            if (lane < 8) gs.bsums[b * 8 + lane] = t8;
        }
    }
    ok &= grid_barrier(gs.bar, nwg * ++phase, t0);
    gstamp(gs, 5, rt_now() - t0);

    // ---------------- D + F: chain (wave 0 of WG 0) beside frame verification
    uint64_t computed = 0;
    if (blockIdx.x == 0 && wave == 0) {
        if (long_cs) {
            const int j = lane & 7;
            uint64_t acc = kAccInit[j];
            const uint64_t key = kSecretW8[16 + j];
            // block sums arrive 8 blocks per 64-lane load, 64 blocks ahead of the chain
            uint64_t cur[8], nxt[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const uint64_t ix = 64 * r + lane;
                cur[r] = ix < 8 * nb ? gs.bsums[ix] : 0;
            }
            for (uint64_t B0 = 0; B0 < nb; B0 += 64) {
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    const uint64_t ix = 8 * (B0 + 64) + 64 * r + lane;
                    nxt[r] = ix < 8 * nb ? gs.bsums[ix] : 0;
                }
                const uint64_t left = nb - B0;  // scalar: the tail group stops early
#pragma unroll
                for (int r = 0; r < 8; ++r)
#pragma unroll
                    for (int c = 0; c < 8; ++c)
                        if ((uint64_t)(8 * r + c) < left) acc = scramble1(acc + __shfl(cur[r], 8 * c + j), key);
#pragma unroll
                for (int r = 0; r < 8; ++r) cur[r] = nxt[r];
            }
            acc += gs.bsums[nb * 8 + j];
            const uint64_t v = gs.cs[nwalk - 8 + j];
            const uint64_t vx = __shfl_xor(v, 1);
            acc += vx;
            acc += mul32x32(v ^ kSecretLast[j]);
            uint64_t a[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) a[i] = __shfl(acc, i);
            uint64_t r = n * P64_1;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                r += fold64(a[2 * i] ^ Secret::w(11 + 16 * i), a[2 * i + 1] ^ Secret::w(19 + 16 * i));
            computed = avalanche(r);
        } else if (VERIFY && lane == 0) {
            uint8_t *s = gs.small;
            const uint64_t w[5] = {h.partition_id, h.base_offset, h.base_timestamp,
                                   h.origin_timestamp, h.batch_length};
            for (int i = 0; i < 5; ++i)
                for (int k = 0; k < 8; ++k) s[8 * i + k] = (uint8_t)(w[i] >> (8 * k));
            for (int k = 0; k < 4; ++k) s[40 + k] = (uint8_t)(h.message_count >> (8 * k));
            for (uint64_t i = 0; i < nwalk; ++i)
                for (int k = 0; k < 8; ++k) s[44 + 8 * i + k] = (uint8_t)(gs.cs[i] >> (8 * k));
            computed = xxh3_64_lane(s, n);
        }
    } else if (VERIFY) {
        const uint32_t vw = blockIdx.x * (blockDim.x >> 6) + wave - 1;
        const uint32_t nvw = nwg * (blockDim.x >> 6) - 1;
        verify_frames(blob, gs, nwalk, vw, nvw, lane);
    }
    ok &= grid_barrier(gs.bar, nwg * ++phase, t0);
    gstamp(gs, 6, rt_now() - t0);

    // ---------------- resolution (wave 0 of WG 0)
    if (blockIdx.x == 0 && wave == 0 && lane == 0) {
        HeaderInfo hi;
        hi.h = h;
        const uint64_t end = __hip_atomic_load(&gs.misc[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t fb_enc = __hip_atomic_load(&gs.misc[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t kind = IGGY_OK, reason = 0;
        uint64_t a = 0, b = 0, c = 0;
        if (!ok) {
            kind = IGGY_ERR_TIMEOUT;
        } else if (VERIFY && fb_enc != 0) {
            const uint64_t i = ~fb_enc, p = gs.fpos[i];
            const uint64_t L = 40 + (uint64_t)ld32_any(blob + p + 36) + ld32_any(blob + p + 32);
            kind = IGGY_ERR_INVALID_MESSAGE_CHECKSUM;
            a = gs.cs[i];
            b = xxh3_64_lane(blob + p + 8, L);
            c = sat_add(h.base_offset, ld32_any(blob + p + 24));
        } else if (nwalk != (uint64_t)h.message_count || (end & kStopBit) || end != bl) {
            kind = IGGY_ERR_VALIDATION;
            reason = IGGY_V_FRAMES_DO_NOT_TILE;
        } else if (VERIFY && computed != h.batch_checksum) {
            kind = IGGY_ERR_INVALID_BATCH_CHECKSUM;
            a = h.batch_checksum; b = computed; c = h.base_offset;
        }
        write_result(result, hi, kind, reason, a, b, c, nwalk, computed, 2, kStatusDone, end & ~kStopBit);
    }
    // retire: the last WG out re-arms the barrier words and misc for the next call
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t prev = __hip_atomic_fetch_add(&gs.bar[1], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == nwg - 1) {
            __hip_atomic_store(&gs.bar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&gs.bar[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&gs.misc[2], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    (void)len;
}

template __global__ void k_decode_general<true>(const uint8_t *__restrict__, uint64_t, uint64_t *,
                                                uint64_t, iggy_decode_result *, GeneralScratch);
template __global__ void k_decode_general<false>(const uint8_t *__restrict__, uint64_t, uint64_t *,
                                                 uint64_t, iggy_decode_result *, GeneralScratch);

}  // namespace iggy

// decode_general.hip — decode_batch_slice_with (core/binary_protocol/src/batch.rs:391-527)
// for records with arbitrary frame sizes: the exact serial walk of
// BatchIteratorWithOffsets (batch.rs:329-355) rebuilt in parallel.
//
// One persistent launch (grid = CUs, all WGs co-resident, bounded grid
// barriers) that returns immediately unless the uniform-stride kernel left
// result->status == kStatusNeedGeneral. Phases:
//   A  locate  : the blob is cut into 4 KiB tiles; one lane per tile finds the
//                first candidate frame start (8 zero reserved bytes at +40 and
//                lengths inside the blob) and walks the candidate chain until it
//                leaves the tile. Output: start s_t, exit x_t, frame list.
//   B  link    : one wave chains tiles from offset 0: a tile is accepted when
//                its speculative start equals the true entry (64 tiles per step
//                by ballot), otherwise it is re-walked from the true entry.
//                The result is exactly the reference walk (true frame starts are
//                always candidates; the first non-candidate ends the walk).
//   C  scatter : frame positions in walk order (prefix over tiles).
//   D  verify  : one lane per frame: XXH3 of frame[8..end), stored checksum
//                kept for the batch checksum, first mismatch by atomic max.
//   E  sums    : XXH3 stripe sums of the batch-checksum input, one wave / block.
//   F  chain   : serial scramble chain, precedence resolution, result.
#include "codec_common.hpp"

namespace iggy {

constexpr uint64_t kTile = 4096;
constexpr uint32_t kTileCap = kTile / kFrameHdr + 1;  // 86 frame starts per tile max
constexpr uint64_t kNoStart = ~0ull;
constexpr uint64_t kStopBit = 1ull << 63;

struct GeneralScratch {
    uint64_t *tile_s;    // [ntiles] speculative start (blob offset) or kNoStart
    uint64_t *tile_x;    // [ntiles] exit position (| kStopBit when the walk stopped inside)
    uint32_t *tile_cnt;  // [ntiles] frames found
    uint16_t *tile_list; // [ntiles * kTileCap] tile-relative starts
    uint64_t *tile_base; // [ntiles] exclusive prefix of accepted counts (~0 = none)
    uint64_t *fpos;      // [max_frames] frame starts in walk order
    uint64_t *cs;        // [max_frames] stored checksums in walk order
    uint64_t *bsums;     // [max_blocks * 8]
    uint64_t *misc;      // [16]: 0 nwalk, 1 end (with stop bit), 2 first_bad enc, 3 computed
    uint32_t *bar;       // [4]: arrive counter, exit counter
    uint8_t *small;      // >= 512 B
    uint64_t ntiles, max_frames, max_blocks;
};

// ---------------------------------------------------------------- helpers
__device__ __forceinline__ bool candidate(const uint8_t *blob, uint64_t bl, uint64_t p,
                                          uint64_t *end) {
    if (p >= bl || bl - p < kFrameHdr) return false;
    if (ld64_any(blob + p + 40) != 0) return false;
    const uint64_t e = p + kFrameHdr + (uint64_t)ld32_any(blob + p + 36) + ld32_any(blob + p + 32);
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

// walk the candidate chain from p while p lies in [tile_lo, tile_hi)
__device__ inline void walk_tile(const uint8_t *blob, uint64_t bl, uint64_t p, uint64_t tile_lo,
                                 uint64_t tile_hi, uint16_t *list, uint32_t *cnt_out,
                                 uint64_t *exit_out) {
    uint32_t cnt = 0;
    while (p < tile_hi && p < bl) {
        uint64_t e;
        if (!candidate(blob, bl, p, &e)) {
            *cnt_out = cnt;
            *exit_out = p | kStopBit;
            return;
        }
        list[cnt++] = (uint16_t)(p - tile_lo);
        p = e;
    }
    *cnt_out = cnt;
    *exit_out = p;  // >= tile_hi, or == bl (clean end)
}

// first candidate start in [lo, hi): scan aligned dwords for a zero dword A;
// an all-zero 8-byte window at p+40 contains the dword at 4*ceil((p+40)/4).
__device__ inline uint64_t first_candidate(const uint8_t *blob, uint64_t bl, uint64_t lo,
                                           uint64_t hi) {
    if (hi > bl) hi = bl;
    if (lo >= hi) return kNoStart;
    const uintptr_t base = (uintptr_t)blob;
    // absolute aligned dword addresses covering [blob+lo+40, blob+hi-1+40+3]
    uintptr_t a = (base + lo + 40 + 3) & ~(uintptr_t)3;
    const uintptr_t a_end = base + hi + 43;  // windows for p < hi
    const uintptr_t blob_end = base + bl;
    for (; a < a_end && a + 4 <= blob_end; a += 4) {
        if (*(const uint32_t *)a != 0) continue;
        // candidates p with window start in [a-3, a], increasing
        for (int d = 3; d >= 0; --d) {
            const uintptr_t ws = a - d;  // window start = blob + p + 40
            if (ws < base + lo + 40) continue;
            const uint64_t p = (uint64_t)(ws - base) - 40;
            if (p >= hi) break;
            uint64_t e;
            if (candidate(blob, bl, p, &e)) return p;
        }
    }
    return kNoStart;
}

// XXH3 stripe contribution of checksum-input word m (value v) to acc index t
__device__ __forceinline__ void word_contrib(uint64_t m, uint64_t v, uint64_t &x, uint64_t &y) {
    // x -> acc[j], y -> acc[j^1]
    const uint32_t j = (uint32_t)(m & 7), sib = (uint32_t)((m >> 3) & 15);
    y = v;
    x = mul32x32(v ^ kSecretW8[sib + j]);
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
    const uint64_t ntiles = (bl + kTile - 1) / kTile;
    const uint32_t nwg = gridDim.x;
    const uint64_t gtid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t gthreads = (uint64_t)nwg * blockDim.x;
    const int lane = threadIdx.x & 63;
    uint32_t phase = 0;
    bool ok = true;

    // ---------------- A: locate
    for (uint64_t t = gtid; t < ntiles; t += gthreads) {
        const uint64_t lo = t * kTile, hi = lo + kTile;
        const uint64_t s = (t == 0) ? 0 : first_candidate(blob, bl, lo, hi);
        gs.tile_s[t] = s;
        uint32_t cnt = 0;
        uint64_t x = kNoStart;
        if (s != kNoStart) walk_tile(blob, bl, s, lo, hi, gs.tile_list + t * kTileCap, &cnt, &x);
        gs.tile_cnt[t] = cnt;
        gs.tile_x[t] = x;
    }
    ok &= grid_barrier(gs.bar, nwg * ++phase, t0);

    // ---------------- B: link (one wave)
    if (blockIdx.x == 0 && threadIdx.x < 64) {
        uint64_t e = 0;        // true entry into the next tile
        uint64_t total = 0;    // frames accepted so far
        bool ended = false;    // the walk stopped (stop bit) or reached the blob end
        for (uint64_t T0 = 0; T0 < ntiles; T0 += 64) {
            const uint64_t T = T0 + lane;
            const bool in = T < ntiles;
            if (ended) {
                if (in) gs.tile_base[T] = ~0ull;
                continue;
            }
            const uint64_t s = in ? gs.tile_s[T] : kNoStart;
            const uint64_t x = in ? gs.tile_x[T] : kNoStart;
            const uint32_t cnt = in ? gs.tile_cnt[T] : 0;
            // fast form: every in-range tile up to the first terminal one is entered
            // exactly at its speculative start (=> accepted in sequence)
            const uint64_t termmask = __ballot(in && ((x & kStopBit) || x >= bl));
            const uint64_t inmask = __ballot(in);
            const int last = termmask ? __builtin_ctzll(termmask) : 63 - __builtin_clzll(inmask);
            const uint64_t xprev = __shfl_up(x, 1);
            const uint64_t pred = (lane == 0) ? e : xprev;
            const bool chained = !in || lane > last || (s != kNoStart && s == pred);
            if (__ballot(!chained) == 0) {
                const uint64_t c = (in && lane <= last) ? cnt : 0;
                uint64_t inc = c;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint64_t o = __shfl_up(inc, d);
                    if (lane >= d) inc += o;
                }
                if (in) gs.tile_base[T] = (lane <= last) ? total + inc - c : ~0ull;
                total += __shfl(inc, 63);
                e = __shfl(x, last);
                if (termmask) ended = true;
                continue;
            }
            // exact sequential rule, tile by tile (skips, repairs, stops)
            for (int l = 0; l < 64; ++l) {
                const uint64_t TT = T0 + l;
                if (TT >= ntiles) break;
                const uint64_t sl = __shfl(s, l), xl = __shfl(x, l);
                const uint32_t cl = __shfl(cnt, l);
                if (lane == 0) {
                    const uint64_t lo = TT * kTile, hi2 = lo + kTile;
                    if (ended) {
                        gs.tile_base[TT] = ~0ull;
                    } else if (e >= hi2) {
                        gs.tile_base[TT] = ~0ull;  // skipped: one frame spans the tile
                    } else if (e == sl) {
                        gs.tile_base[TT] = total;
                        total += cl;
                        e = xl;
                    } else {
                        uint32_t c2 = 0;
                        uint64_t x2 = 0;
                        walk_tile(blob, bl, e, lo, hi2, gs.tile_list + TT * kTileCap, &c2, &x2);
                        gs.tile_cnt[TT] = c2;
                        gs.tile_base[TT] = total;
                        total += c2;
                        e = x2;
                    }
                    if ((e & kStopBit) || e >= bl) ended = true;
                }
                e = __shfl(e, 0);
                total = __shfl(total, 0);
                ended = __shfl((int)ended, 0) != 0;
            }
        }
        if (lane == 0) {
            __hip_atomic_store(&gs.misc[0], total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&gs.misc[1], e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    ok &= grid_barrier(gs.bar, nwg * ++phase, t0);

    const uint64_t nwalk = __hip_atomic_load(&gs.misc[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // ---------------- C: scatter frame positions (walk order)
    for (uint64_t t = gtid; t < ntiles; t += gthreads) {
        const uint64_t base = gs.tile_base[t];
        if (base == ~0ull) continue;
        const uint32_t cnt = gs.tile_cnt[t];
        const uint16_t *list = gs.tile_list + t * kTileCap;
        for (uint32_t k = 0; k < cnt; ++k) {
            const uint64_t p = t * kTile + list[k];
            if (base + k < gs.max_frames) gs.fpos[base + k] = p;
            if (frame_pos && base + k < cap) frame_pos[base + k] = p;
        }
    }
    ok &= grid_barrier(gs.bar, nwg * ++phase, t0);

    // ---------------- D: verify every walked frame
    if (VERIFY) {
        for (uint64_t i = gtid; i < nwalk; i += gthreads) {
            const uint64_t p = gs.fpos[i];
            const uint64_t L = 40 + (uint64_t)ld32_any(blob + p + 36) + ld32_any(blob + p + 32);
            const uint64_t stored = ld64_any(blob + p);
            gs.cs[i] = stored;
            if (xxh3_64_lane(blob + p + 8, L) != stored)
                atomicMax((unsigned long long *)&gs.misc[2], (unsigned long long)~i);
        }
    }
    ok &= grid_barrier(gs.bar, nwg * ++phase, t0);

    // ---------------- E: checksum-input block sums (one wave per block)
    const uint64_t n = 44 + 8 * nwalk;
    const bool long_cs = VERIFY && n > 240;
    uint64_t nb = 0, Mreg = 0;
    if (long_cs) {
        nb = (n - 1) / 1024;
        const uint64_t ns = ((n - 1) - 1024 * nb) / 64;
        Mreg = 8 * (16 * nb + ns);
        const uint64_t wid = gtid >> 6, nwaves = gthreads >> 6;
        for (uint64_t b = wid; b <= nb; b += nwaves) {
            uint64_t x = 0, y = 0;
            for (int half = 0; half < 2; ++half) {
                const uint64_t m = 128 * b + 64 * half + lane;
                if (m < Mreg) {
                    uint64_t v;
                    if (m < 5) {
                        const uint64_t hw[5] = {h.partition_id, h.base_offset, h.base_timestamp,
                                                h.origin_timestamp, h.batch_length};
                        v = hw[m];
                    } else if (m == 5) {
                        v = (uint64_t)h.message_count | (gs.cs[0] << 32);
                    } else {
                        v = (gs.cs[m - 6] >> 32) | (gs.cs[m - 5] << 32);
                    }
                    uint64_t xx, yy;
                    word_contrib(m, v, xx, yy);
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

    // ---------------- F: chain + resolution (one wave)
    if (blockIdx.x == 0 && threadIdx.x < 64) {
        uint64_t computed = 0;
        if (long_cs) {
            const int j = lane & 7;
            uint64_t acc = kAccInit[j];
            const uint64_t key = kSecretW8[16 + j];
            for (uint64_t b = 0; b < nb; ++b) acc = scramble1(acc + gs.bsums[b * 8 + j], key);
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
        if (lane == 0) {
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

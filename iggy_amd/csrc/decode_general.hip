// decode_general.hip — decode_batch_slice_with (core/binary_protocol/src/batch.rs:391-527)
// for records with arbitrary frame sizes: the exact serial walk of
// BatchIteratorWithOffsets (batch.rs:329-355) rebuilt in parallel.
//
// One persistent launch (bounded grid barriers over the workgroups that joined:
// join_members) that returns immediately unless the uniform-stride kernel left
// result->status == kStatusNeedGeneral. The blob is cut into tiles of
// T bytes, 8-16 average frames (4 KiB <= T <= 1 MiB, tile_bytes); a group is 256
// tiles, 4 per lane of one wave. Phases:
//   A  locate : one lane per tile picks a speculative entry (a confirmed
//               candidate frame start: 8 zero reserved bytes at +40, lengths
//               inside the blob; 256-B vector scan for zero dwords) and walks
//               the candidate chain from it until it leaves the tile, listing
//               the frame offsets: start s_t, exit x_t, count cnt_t, list.
//   B1 groups : one wave per group: is the group self-consistent when entered at
//               its first start (every later tile entered at its own start, or
//               spanned by one frame when it has none)? -> (S, X, CNT, ok, term)
//               and each tile's frame prefix inside the group.
//   B2 link   : one wave chains groups from offset 0, up to 64 per ballot step,
//               advancing to the first group that is not entered at S or not
//               self-consistent; that group is linked tile by tile (spans
//               skipped, entries re-walked and re-listed). The result is exactly
//               the reference walk: true frame starts are always candidates and
//               the first non-candidate ends the walk.
//   C  scatter: sixteen lanes per accepted tile copy its lists to walk order:
//               frame positions and the stored checksums locate read beside them.
//   E  sums   : XXH3 stripe sums of the batch-checksum input, one wave / block.
//   D + F     : wave 0 of WG 0 runs the serial scramble chain over the block
//               sums while every other wave verifies frames (8 lanes per frame,
//               one 1024-B block per step, the next block in flight); then
//               precedence resolution and the result.
#include "codec_common.hpp"

namespace iggy {

constexpr uint32_t kTileShiftMin = 12, kTileShiftMax = 20;
constexpr uint64_t kTileMin = 1ull << kTileShiftMin;  // host sizing unit
constexpr uint64_t kNoStart = ~0ull;
constexpr uint64_t kStopBit = 1ull << 63;
constexpr uint32_t kGrpTiles = 256;  // 4 tiles per lane
constexpr uint32_t kGrpWords = 6;    // S, X, CNT, flags | base, mode
constexpr uint64_t kGrpOk = 1, kGrpTerm = 2;
constexpr uint32_t kNotLive = ~0u;
constexpr uint32_t kGenThreads = 512;  // one WG per CU: half the barrier arrivals of 2 x 256
constexpr uint32_t kBar2Groups = 8, kBar2Words = kBar2Groups + 1;  // grid_barrier2 counters + top

// list entries (u32 offsets from the tile start) per tile of T bytes
__host__ __device__ __forceinline__ uint64_t tile_list_cap(uint64_t T) { return T / 48 + 1; }
// host sizing of the list area for a blob of up to L bytes (any tile size)
__host__ __device__ __forceinline__ uint64_t tile_list_words(uint64_t L) {
    return L / 48 + L / kTileMin + (1ull << kTileShiftMax) / 48 + 64;
}

struct GeneralScratch {
    uint64_t *tile_s;    // [ntiles] speculative entry (blob offset) or kNoStart
    uint64_t *tile_x;    // [ntiles] exit position (| kStopBit when the walk stopped inside)
    uint32_t *tile_cnt;  // [ntiles] frames listed for the tile
    uint32_t *tile_pre;  // [ntiles] frames before the tile inside its group (kNotLive: none)
    uint32_t *tile_list; // [ntiles * tile_list_cap(T)] frame offsets from the tile start
    uint64_t *tile_e;    // [ntiles] repaired groups: true entry (~0: no frame starts here)
    uint64_t *tile_base; // [ntiles] repaired groups: frames before the tile
    uint64_t *grp;       // [ngroups * kGrpWords]
    uint64_t *tile_lcs;  // [ntiles * tile_list_cap(T)] stored checksum of each listed frame
    uint64_t *fpos;      // [max_frames] frame starts in walk order (hashed length of frame f:
                         // fpos[f+1] - fpos[f] - 8, the last frame's from the walk end)
    uint64_t *cs;        // [max_frames] stored checksums in walk order (+16 B: read in aligned pairs)
    uint64_t *vrec;      // [max_frames + 1] x 2: (frame start, hashed length | frame index << 32) in
                         // walk order, then a "none" record (index kVdNone): verify_frames_dma
    uint64_t *bsums;     // [max_blocks * 8]
    uint64_t *misc;      // [16]: 0 nwalk, 1 end (with stop bit), 2 first_bad enc
    uint32_t *bar2;      // [kBar2Words * 32]: two-level barrier counters, 128 B apart (grid_barrier2)
    uint32_t *bar;       // [4]: 2 registration (count | kRegClosed), 3 members
                         // (all re-armed by k_decode_uniform, which always runs first on the stream)
    uint32_t *u_exited;  // the uniform kernel's sync words, re-armed here for the next decode
    uint64_t *u_first_bad, *u_spec_fail;
    uint8_t *small;      // >= 512 B
    uint64_t ntiles, max_frames, max_blocks;  // ntiles: capacity in kTileMin tiles
    uint32_t dbg;        // ablation bits (diagnostic build only; kDiagMask folds them out)
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

// Two-level grid barrier: members arrive on one of kBar2Groups counters (member % 8),
// the last arrival of a counter's phase adds one to the top counter, and everyone
// waits for the top counter. A single counter took all ~256 workgroups' arrivals on
// one address, serialised at the memory side. Monotonic: phase p (1-based) is done
// when the top counter reaches min(nwg, kBar2Groups) * p. Bounded like grid_barrier.
__device__ bool grid_barrier2(uint32_t *bar2, uint32_t member, uint32_t nwg, uint32_t p, uint64_t t0) {
    __syncthreads();
    bool ok = true;
    if (threadIdx.x == 0) {
        const uint32_t g = member % kBar2Groups;
        const uint32_t nsub = (nwg - 1 - g) / kBar2Groups + 1;  // members on counter g (member < nwg)
        const uint32_t ngrp = nwg < kBar2Groups ? nwg : kBar2Groups;
        uint32_t *top = bar2 + 32 * kBar2Groups;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t old = __hip_atomic_fetch_add(bar2 + 32 * g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old + 1 == nsub * p) __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (__hip_atomic_load(top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < ngrp * p) {
            __builtin_amdgcn_s_sleep(1);
            if (rt_now() - t0 > kSpinLimitTicks) { ok = false; break; }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    return ok;
}

// phase clock (diagnostics): member 0 stamps the ticks since entry after every
// barrier at small+512 (u64 [1..6]); [8..] are counters of the link phase
__device__ __forceinline__ void gstamp(const GeneralScratch &gs, uint32_t member, int idx, uint64_t v) {
    if (member == 0 && threadIdx.x == 0) ((uint64_t *)(gs.small + 512))[idx] = v;
}

// Membership: the grid barriers below may only count workgroups that are running.
// Every WG registers with one atomic add; the first to register (member 0) waits a
// bounded time for the rest of the grid, then closes registration with an atomic
// or. WGs that register after the close (still queued behind other work on a
// shared GPU: another context's decode, another process) exit at once, and the
// members split the work. So the barriers never wait for a workgroup that is not
// resident, whatever else holds the chip, and no cooperative launch is needed.
constexpr uint32_t kRegClosed = 1u << 31;
constexpr uint32_t kNotMember = ~0u;
constexpr uint64_t kJoinTicks = 2000;  // 20 us at 100 MHz: the whole grid normally joins in < 2 us
__device__ inline void join_members(const GeneralScratch &gs, uint64_t t0, uint32_t *s_mem) {
    if (threadIdx.x == 0) {
        uint32_t me = kNotMember, nm = 0;
        const uint32_t t = __hip_atomic_fetch_add(&gs.bar[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!(t & kRegClosed)) {
            if (t == 0) {
                while ((__hip_atomic_load(&gs.bar[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ~kRegClosed) <
                           gridDim.x &&
                       rt_now() - t0 < kJoinTicks)
                    __builtin_amdgcn_s_sleep(1);
                const uint32_t old =
                    __hip_atomic_fetch_or(&gs.bar[2], kRegClosed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                nm = old & ~kRegClosed;
                __hip_atomic_store(&gs.bar[3], nm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                while ((nm = __hip_atomic_load(&gs.bar[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0 &&
                       rt_now() - t0 < kSpinLimitTicks)
                    __builtin_amdgcn_s_sleep(1);
            }
            if (nm) me = t;
        }
        s_mem[0] = me;
        s_mem[1] = nm;
    }
    __syncthreads();
}

// Tile size: the smallest power of two holding 8 frames of the header's average
// size; when that holds fewer than 14, 16 frames (a multiple of 64 B) instead;
// always inside [kTileMin, 2^kTileShiftMax]. Same-box phase clocks: C3 (2.1-KB
// frames) 32-KiB tiles (15.4 frames) 0.85-0.88 ms against 0.86-0.90 ms for 31.9-
// and 34.1-KB tiles (15 / 16 frames: locate 10-15 us slower) and 0.886-0.912 ms
// for one 17-KB tile per locate lane; 4 M x U[64, 512] B: 4-KiB tiles (12 frames)
// 1.42-1.47 ms, 5.1-KB (15) 1.38-1.42 ms, 5.4-KB (16) 1.35-1.39 ms.
__device__ __forceinline__ uint64_t tile_bytes(uint64_t bl, uint32_t message_count) {
    const uint64_t avg = message_count ? bl / message_count : bl;
    uint64_t T = kTileMin;
    while (T < (1ull << kTileShiftMax) && T < 8 * avg) T <<= 1;
    if (T < 14 * avg) T = min(max((16 * avg + 63) & ~63ull, kTileMin), 1ull << kTileShiftMax);
    return T;
}

// walk the candidate chain from p while p < hi (hi <= bl); with a list, every
// frame's offset from lo and its stored checksum are recorded (the checksum load
// goes out in the same round as the header test: the scatter phase then copies
// lists instead of re-reading one random header line per frame)
__device__ inline uint32_t walk(const uint8_t *blob, uint64_t bl, uint64_t p, uint64_t hi,
                                uint64_t *x_out, uint32_t *list = nullptr, uint64_t lo = 0,
                                uint64_t *lcs = nullptr) {
    uint32_t cnt = 0;
    while (p < hi) {
        if (p >= bl || bl - p < kFrameHdr) break;
        const uint4 w = ld128_any(blob + p + 32);  // lengths at +32/+36, reserved at +40
        const uint64_t c = lcs ? ld64_any(blob + p) : 0;
        const uint64_t e = p + kFrameHdr + (uint64_t)w.x + w.y;
        if ((w.z | w.w) != 0 || e > bl) break;
        if (list) list[cnt] = (uint32_t)(p - lo);
        if (lcs) lcs[cnt] = c;
        ++cnt;
        p = e;
    }
    *x_out = p < hi ? (p | kStopBit) : p;  // >= hi: left the tile (== bl: clean end)
    return cnt;
}

// Locate's walk: the same chain, with the list entries held in registers and
// stored kLocBuf at a time. The stores share vmcnt with the header loads, so
// walk()'s per-frame stores make every next header load wait for their
// acknowledgement as well. Same box, C3 decode (scripts/gpu_r4j.sh): unbuffered
// 0.6879 ms, 8 entries 0.6734, 16 entries 0.6882.
#ifndef IGGY_LOC_BUF
#define IGGY_LOC_BUF 8
#endif
constexpr int kLocBuf = IGGY_LOC_BUF;
#ifndef IGGY_VREC_U
#define IGGY_VREC_U 8
#endif
constexpr int kVrecU = IGGY_VREC_U;  // phase E's frame records per pass
__device__ inline uint32_t walk_located(const uint8_t *blob, uint64_t bl, uint64_t p, uint64_t hi,
                                        uint64_t *x_out, uint32_t *list, uint64_t lo, uint64_t *lcs) {
    if (kLocBuf <= 1) return walk(blob, bl, p, hi, x_out, list, lo, lcs);
    uint32_t cnt = 0;
    bool go = true;
    while (go) {
        uint32_t bo[kLocBuf > 1 ? kLocBuf : 1];
        uint64_t bc[kLocBuf > 1 ? kLocBuf : 1];
        int n = 0;
#pragma unroll
        for (int k = 0; k < kLocBuf; ++k) {
            bo[k] = 0;
            bc[k] = 0;
            if (go) {
                if (p >= hi || p >= bl || bl - p < kFrameHdr) {
                    go = false;
                } else {
                    const uint4 w = ld128_any(blob + p + 32);
                    const uint64_t c = lcs ? ld64_any(blob + p) : 0;
                    const uint64_t e = p + kFrameHdr + (uint64_t)w.x + w.y;
                    if ((w.z | w.w) != 0 || e > bl) {
                        go = false;
                    } else {
                        bo[k] = (uint32_t)(p - lo);
                        bc[k] = c;
                        n = k + 1;
                        p = e;
                    }
                }
            }
        }
#pragma unroll
        for (int k = 0; k < kLocBuf; ++k)
            if (k < n) {
                list[cnt + k] = bo[k];
                if (lcs) lcs[cnt + k] = bc[k];
            }
        cnt += n;
    }
    *x_out = p < hi ? (p | kStopBit) : p;
    return cnt;
}

// Candidate starts (ascending, at most kPickBatch, all >= from and < hi) from the
// zero dwords of the first 256-B window at or after `from` that has any;
// *next = where the search goes on.
constexpr int kPickBatch = 8;
__device__ inline int window_candidates(const uint8_t *blob, uint64_t bl, uint64_t from, uint64_t hi,
                                        uint64_t (&cp)[kPickBatch], uint64_t *next) {
    if (from >= hi) return 0;
    const uintptr_t base = (uintptr_t)blob;
    const uintptr_t a_end = base + hi + 43;  // dwords holding a window of some p < hi
    const uintptr_t blob_end = base + bl;
    const uintptr_t wlo = base + from + 40;
    uintptr_t a = wlo & ~(uintptr_t)15;
    int nc = 0;
    auto take = [&](uintptr_t ad) {  // the windows [ad-3, ad] of one zero dword, ascending
        for (int d = 3; d >= 0 && nc < kPickBatch; --d) {
            const uintptr_t ws = ad - d;
            if (ws < wlo) continue;
            const uint64_t p = (uint64_t)(ws - base) - 40;
            if (p >= hi) return;
            cp[nc++] = p;
        }
    };
    // 512 B per round (two 256-B windows loaded together): the scan from a tile's
    // start to the first frame header is the long pole of locate, and the wave
    // waits for its slowest lane
    while (a < a_end && a + 512 <= blob_end) {
        uint4 v[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) v[k] = *(const uint4 *)(a + 16 * k);
        uint64_t zm[2] = {0, 0};  // bit 4k+q of zm[h]: dword q of v[16h+k] is zero
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const uint4 w = v[16 * h + k];
                zm[h] |= (uint64_t)((w.x == 0) | ((w.y == 0) << 1) | ((w.z == 0) << 2) |
                                    ((w.w == 0) << 3)) << (4 * k);
            }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint64_t zmask = zm[h];
            while (zmask && nc < kPickBatch) {
                const int bit = __builtin_ctzll(zmask);
                zmask &= zmask - 1;
                const uintptr_t ad = a + 256 * h + 4 * bit;
                if (ad >= a_end) break;
                take(ad);
            }
            if (nc) {
                *next = cp[nc - 1] + 1;
                return nc;
            }
        }
        a += 512;
    }
    for (; a < a_end && a + 4 <= blob_end && nc < kPickBatch; a += 4)
        if (*(const uint32_t *)a == 0) take(a);
    if (nc) *next = cp[nc - 1] + 1;
    return nc;
}

// The tile's speculative entry. Frame headers themselves hold zero runs
// (timestamp delta, user-header length, the high bytes of a small offset
// delta) that pass the reserved-bytes test a few bytes BEFORE a true start,
// with random "lengths" that usually still fit the blob. So the pick is the
// first candidate whose chain is confirmed (its successor starts inside the
// tile); failing that, the candidate whose single frame leaves the tile at the
// nearest exit, else the first valid candidate. Candidates come a window at a
// time and are tested together: their headers in one round of loads, their
// successors in a second. Only speed depends on the pick: the link phase
// re-walks any tile whose pick disagrees with the true entry.
constexpr int kPickWindows = 4;
__device__ inline void pick_start(const uint8_t *blob, uint64_t bl, uint64_t lo, uint64_t hi,
                                  uint32_t *list, uint64_t *lcs, uint64_t *s_out, uint64_t *x_out,
                                  uint32_t *cnt_out) {
    uint64_t pick = kNoStart, clean_p = kNoStart, clean_x = kNoStart, first_valid = kNoStart;
    uint64_t from = lo;
    for (int w = 0; w < kPickWindows && pick == kNoStart; ++w) {
        uint64_t cp[kPickBatch], next = hi;
        const int nc = window_candidates(blob, bl, from, hi, cp, &next);
        if (!nc) break;
        uint4 hv[kPickBatch], sv[kPickBatch];
        uint64_t e[kPickBatch];
        bool val[kPickBatch];
#pragma unroll
        for (int k = 0; k < kPickBatch; ++k)
            hv[k] = ld128_any(blob + ((k < nc && cp[k] + kFrameHdr <= bl) ? cp[k] + 32 : 0));
#pragma unroll
        for (int k = 0; k < kPickBatch; ++k) {
            e[k] = k < nc ? cp[k] + kFrameHdr + (uint64_t)hv[k].x + hv[k].y : 0;
            val[k] = k < nc && cp[k] + kFrameHdr <= bl && (hv[k].z | hv[k].w) == 0 && e[k] <= bl;
            sv[k] = ld128_any(blob + ((val[k] && e[k] < hi && e[k] + kFrameHdr <= bl) ? e[k] + 32 : 0));
        }
        // Zero runs of a true header make false candidates 1-2 B BEFORE its start, whose
        // "payload length" is the true one shifted left a byte; for small payloads that
        // lands inside the tile and, now and then, on another header's zero run, so the
        // false chain is confirmed too (C3: ~2 tiles per decode, each a serial re-walk
        // in the link phase). So a confirmed pick moves to a later confirmed candidate
        // of the same cluster (each within 16 B of the one before).
        bool done = false;
        uint64_t last_c = 0;
#pragma unroll
        for (int k = 0; k < kPickBatch; ++k) {
            if (!val[k] || done) continue;
            if (pick != kNoStart && cp[k] > last_c + 16) {
                done = true;
                continue;
            }
            last_c = cp[k];
            if (first_valid == kNoStart) first_valid = cp[k];
            if (e[k] < hi) {
                const bool conf = e[k] + kFrameHdr <= bl && (sv[k].z | sv[k].w) == 0 &&
                                  e[k] + kFrameHdr + (uint64_t)sv[k].x + sv[k].y <= bl;
                if (conf) pick = cp[k];
            } else if (pick == kNoStart && e[k] < clean_x) {
                clean_p = cp[k];
                clean_x = e[k];
            }
        }
        from = next;
    }
    if (pick == kNoStart) pick = clean_p != kNoStart ? clean_p : first_valid;
    uint64_t x = kNoStart;
    uint32_t cnt = 0;
#ifndef IGGY_DIAG_LOCATE_PICK_ONLY
    if (pick != kNoStart) cnt = walk_located(blob, bl, pick, hi, &x, list, lo, lcs);
#endif
    *s_out = pick;
    *x_out = x;
    *cnt_out = cnt;
}

// XXH3 stripe contribution of checksum-input word m (value v)
__device__ __forceinline__ void word_contrib(uint64_t m, uint64_t v, uint64_t &x, uint64_t &y) {
    // x -> acc[j], y -> acc[j^1]
    const uint32_t j = (uint32_t)(m & 7), sib = (uint32_t)((m >> 3) & 15);
    y = v;
    x = mul32x32(v ^ kSecretW8[sib + j]);
}

// Frame verification. (C3 experiments, scripts/diag_general.py: byte-balanced
// contiguous ranges per group, or a wave's groups claiming its frames as they
// finish, cut the slowest group's 17 % lead over the mean but made the mean 12-16 %
// slower -- the chip-wide front of consecutive frames is worth more; hashing the
// <= 240 B frames inside the loop pushed the kernel past 256 VGPRs and spilled;
// the last 25 % of the frames claimed one per group from a counter took the loop
// from 0.53 to 1.57 ms: 16 K groups' claims on one address serialise in L2.)
// Lane group fg (8 lanes) of verify wave vw hashes frames
// f = 8 vw + fg + j * 8 nvw, j = 0, 1, ... at its own pace: every wave step
// each group hashes one 1024-B block of its current frame while the next block
// (or the next frame's first block and last stripe) is loading into the other
// of two register sets (ping-pong: in-flight loads are never copied, which
// would make the wave wait for them). Positions and stored checksums come from
// the scatter phase's arrays, one frame ahead (a length is the distance to the
// next frame's start). Lane l = (m, par) owns
// accumulators 2m, 2m+1 for the stripes of parity par: in every block it reads
// the 16 B at 128q + 16(m + 4 par), q = 0..7 (stripe 2q+par, words 2m, 2m+1);
// the pair of parity lanes is folded before each scramble; the last stripe and
// merge follow the XXH3 long form (> 240 B). Frames of <= 240 hashed bytes are
// checked before the loop, one lane each.
struct VFrame {
    uint64_t f, p, stored, L;
};
__device__ __forceinline__ VFrame vframe(const GeneralScratch &gs, uint64_t f, uint64_t nwalk, uint64_t wend) {
    VFrame v;
    v.f = f;
    if (f < nwalk) {
        v.p = gs.fpos[f];
        v.stored = gs.cs[f];
        v.L = (f + 1 < nwalk ? gs.fpos[f + 1] : wend) - v.p - 8;  // frames tile the walk
    } else {
        v.p = 0; v.stored = 0; v.L = 0;
    }
    return v;
}
struct VStep {
    uint4 v[8];       // the 8 chunks of one block, loaded from 4-B-aligned addresses
    uint32_t nx[8];   // the dword after each chunk (the bytes the alignment shifted out)
    uint4 last;       // the frame's last-stripe chunk (first block only), aligned the same way
    uint32_t lnx;     // the dword after it
    uint32_t nx7;     // (diagnostic neighbour form) the dword after the block, for lane k = 7
    uint32_t clampm;  // (idem) bit q: chunk q was loaded 12 B early (a neighbour-only chunk at the blob end)
};
// Diagnostic form (dbg bit 0x100000, next-round candidate): the dword after each chunk
// is the first dword of the chunk the next lane of the group loaded (poff order
// k = m + 4 par: lanes l = 0..5 take lane l + 2, lane 6 lane 1, lane 7 lane 0 of the
// next row), moved with DPP instead of loaded: 10 loads per step instead of 18.
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x, int ctrl) {
    switch (ctrl) {
        case 0: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x102, 0xF, 0xF, false);  // row_shl:2
        case 1: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x115, 0xF, 0xF, false);  // row_shr:5
        default: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x117, 0xF, 0xF, false); // row_shr:7
    }
}
// 16 bytes starting r bytes into (w.x, w.y, w.z, w.w, nb)
__device__ __forceinline__ uint4 realign(uint4 w, uint32_t nb, uint32_t r) {
    return make_uint4(__builtin_amdgcn_alignbyte(w.y, w.x, r), __builtin_amdgcn_alignbyte(w.z, w.y, r),
                      __builtin_amdgcn_alignbyte(w.w, w.z, r), __builtin_amdgcn_alignbyte(nb, w.w, r));
}
// the loads of frame v's block b: always 18. Frames start at any byte offset and
// byte-misaligned 16-B loads stream ~25 % slower (profiles/r01_bw_misalign.txt),
// so each chunk is loaded from its 4-B-aligned address plus the dword after it
// (only when the frame is misaligned; that dword holds a byte the hash needs, so
// it never reaches past the 4-B word of a frame byte) and realigned in registers.
__device__ __forceinline__ void vissue(const uint8_t *blob, const VFrame &v, uint64_t nwalk, uint32_t b,
                                       uint32_t par, uint32_t poff, uint32_t m, VStep &st, uint32_t dbg = 0,
                                       const uint8_t *blob_end = nullptr) {
    const bool lng = v.f < nwalk && v.L > 240;
    const uint64_t nbF = lng ? (v.L - 1) / 1024 : 0, ns = lng ? ((v.L - 1) - 1024 * nbF) / 64 : 0;
    const uint8_t *H = blob + v.p + 8;
    const uint32_t r = (uint32_t)((uintptr_t)H & 3);
    const uint8_t *hb = H - r + 1024ull * b + poff;
    if (kDiagMask && (dbg & 0x100000)) {
        // a chunk is loaded when its own piece is hashed, or (misaligned frames) when the
        // piece before it in stream order is: its first dword completes that piece
        const uint32_t k = m + 4 * par;
        st.clampm = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const bool full = b < nbF;
            const bool use = lng && (full || 2 * q + par < ns);
            const uint64_t sprev = k == 0 ? (uint64_t)(2 * q) - 1 : 2 * q + (k - 1 >= 4 ? 1 : 0);
            const bool prev_use = lng && (k != 0 || q != 0) && (full || sprev < ns);
            const bool need = use || (r && prev_use);
            const uint8_t *a = hb + 128 * q;
            // a neighbour-only chunk of the record's last frame may run past the blob
            // end: load the 16 B that end with its first dword instead
            const bool clamp = need && !use && a + 16 > blob_end;
            if (clamp) st.clampm |= 1u << q;
            st.v[q] = ld128_any(need ? (clamp ? a - 12 : a) : blob);
            st.nx[q] = 0;
        }
        const bool use77 = lng && (b < nbF || 15 < ns);  // piece (7, k = 7): stripe 15
        st.nx7 = *(const uint32_t *)((k == 7 && use77 && r) ? hb + 128 * 7 + 16 : blob);
    } else
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const bool use = lng && (b < nbF || 2 * q + par < ns);
        st.v[q] = ld128_any(use ? hb + 128 * q : blob);
        if (kDiagMask && (dbg & 0x80000)) st.nx[q] = 0;  // ablation: no realignment loads (hash wrong)
        else st.nx[q] = *(const uint32_t *)((use && r) ? hb + 128 * q + 16 : blob);
    }
    const uint8_t *E = H + v.L;
    const uint32_t rl = (uint32_t)((uintptr_t)E & 3);
    const uint8_t *lc = E - rl - 64 + 16 * m;
    const bool lp = lng && b == 0;
    st.last = ld128_any(lp ? lc : blob);
    st.lnx = *(const uint32_t *)((lp && rl) ? lc + 16 : blob);
}

// Frames of <= 240 hashed bytes (XXH3's short forms): one lane each, slice sw of nsw.
__device__ inline void verify_short(const uint8_t *blob, const GeneralScratch &gs, uint64_t nwalk, uint64_t wend,
                                    uint32_t sw, uint32_t nsw, int lane) {
    const uint64_t C = (nwalk + nsw - 1) / nsw;
    const uint64_t f1 = min((uint64_t)(sw + 1) * C, nwalk);
    for (uint64_t f = (uint64_t)sw * C + lane; f < f1; f += 64) {
        const uint64_t p = gs.fpos[f];
        const uint64_t L = (f + 1 < nwalk ? gs.fpos[f + 1] : wend) - p - 8;
        if (L <= 240 && xxh3_64_lane(blob + p + 8, L) != gs.cs[f])
            atomicMax((unsigned long long *)&gs.misc[2], (unsigned long long)~f);
    }
}

__device__ inline void verify_frames(const uint8_t *blob, const GeneralScratch &gs, uint64_t nwalk,
                                     uint64_t wend, uint32_t vw, uint32_t nvw, uint32_t member, uint32_t nwg,
                                     uint32_t *s_claim, int lane, uint64_t t0, const uint8_t *blob_end) {
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
    const uint64_t stride = 8ull * nvw;
    // Frames below fdyn follow the static stride (the chip-wide front). The last
    // eighth is split over the workgroups (member m: fdyn + m + k * nwg) and claimed
    // frame by frame from an LDS counter, so lane groups that drew light frames take
    // more and the loop ends near the workgroup's mean group load, not its heaviest
    // wave's (C3: loop end mean ~465 us vs max ~550 us with the stride alone). An
    // LDS claim waits on lgkmcnt, never on the in-flight frame loads (vmcnt).
    // (same-box A/B on C3, loop end mean / max: static only 734-760 / 802-830 us,
    // last quarter claimed 766-771 / 804-818, last eighth 755-761 / 804-807)
    const uint64_t fdyn = nwalk - nwalk / 8;
    auto next_f = [&](uint64_t f) -> uint64_t {  // f: the static successor
        if (f < fdyn) return f;
        uint32_t k = 0;
        if (l == 0) k = atomicAdd(s_claim, 1u);
        k = (uint32_t)__shfl((int)k, lane & ~7);
        return fdyn + member + (uint64_t)nwg * k;  // >= nwalk: none left
    };
    VFrame cur = vframe(gs, next_f(8ull * vw + fg), nwalk, wend);
    VFrame nxt = vframe(gs, cur.f < nwalk ? next_f(cur.f < fdyn ? cur.f + stride : fdyn) : nwalk, nwalk, wend);
    uint32_t b = 0;
    uint64_t a0 = init0, a1 = init1;
    uint4 lastp = make_uint4(0, 0, 0, 0);
    uint64_t bad = ~0ull;  // first mismatching frame of this group
    // hash the step whose loads are in X, issue the next step's into Y
    auto step = [&](VStep &X, VStep &Y) {
        if (cur.f >= nwalk) return;
        const uint64_t L = cur.L;
        const bool lng = L > 240;
        const uint64_t nbF = lng ? (L - 1) / 1024 : 0;
        const uint64_t ns = lng ? ((L - 1) - 1024 * nbF) / 64 : 0;
        const uint32_t nsteps = lng ? (uint32_t)(nbF + (ns > 0)) : 1u;
        const bool fin = b + 1 == nsteps;
        if (!fin) vissue(blob, cur, nwalk, b + 1, par, poff, m, Y, gs.dbg, blob_end);
        else vissue(blob, nxt, nwalk, 0, par, poff, m, Y, gs.dbg, blob_end);
        const uint32_t r = (uint32_t)((uintptr_t)(blob + cur.p + 8) & 3);
        if (b == 0) lastp = realign(X.last, X.lnx, (uint32_t)((uintptr_t)(blob + cur.p + 8 + L) & 3));
        uint4 pc[8];
        if (kDiagMask && (gs.dbg & 0x100000)) {
            uint32_t ex[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) ex[q] = ((X.clampm >> q) & 1) ? X.v[q].w : X.v[q].x;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint32_t a = dpp_u32(ex[q], 0), bb = dpp_u32(ex[q], 1);
                const uint32_t c = q < 7 ? dpp_u32(ex[q < 7 ? q + 1 : q], 2) : X.nx7;
                const uint32_t nx = l <= 5 ? a : (l == 6 ? bb : c);
                pc[q] = realign(X.v[q], nx, r);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 8; ++q) pc[q] = realign(X.v[q], X.nx[q], r);
        }
        if (lng) {
            if (b < nbF) {
                uint64_t p0[4] = {0, 0, 0, 0}, p1[4] = {0, 0, 0, 0};
#pragma unroll
                for (int q = 0; q < 8; ++q) piece(p0[q & 3], p1[q & 3], pc[q], s0[q], s1[q]);
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
                    if (2 * q + par < ns) piece(a0, a1, pc[q], s0[q], s1[q]);
            }
            if (fin) {
                a0 += gdpp64<0xB1>(a0);
                a1 += gdpp64<0xB1>(a1);
                piece(a0, a1, lastp, last0, last1);
                uint64_t t = fold64(a0 ^ mrg0, a1 ^ mrg1);
                t += gdpp64<0x4E>(t);
                t += gswz_xor4(t);
                const uint64_t h = avalanche(L * P64_1 + t);
                if (h != cur.stored && bad == ~0ull) bad = cur.f;
            }
        }
        if (fin) {
            cur = nxt;
            nxt = vframe(gs, cur.f < nwalk ? next_f(cur.f < fdyn ? cur.f + stride : fdyn) : nwalk, nwalk, wend);
            b = 0;
            a0 = init0;
            a1 = init1;
        } else {
            ++b;
        }
    };
    // frames of <= 240 hashed bytes: one lane each, a contiguous slice per wave, before
    // the streaming loop (chunks claimed from one counter after the loop serialised
    // ~4 K claims once the balanced tail made every wave finish together: +40 us on C3)
    verify_short(blob, gs, nwalk, wend, vw, nvw, lane);
    VStep A, B;
    vissue(blob, cur, nwalk, 0, par, poff, m, A, gs.dbg, blob_end);
    while (__ballot(cur.f < nwalk)) {
        step(A, B);
        if (!__ballot(cur.f < nwalk)) break;
        step(B, A);
    }
    if (l == 0 && bad != ~0ull) atomicMax((unsigned long long *)&gs.misc[2], (unsigned long long)~bad);
    uint64_t *vstat = (uint64_t *)(gs.small + 512) + 14;  // phase clock: [14] last / [15] sum of loop ends
    if (lane == 0) {
        const uint64_t d = rt_now() - t0;
        atomicMax((unsigned long long *)&vstat[0], (unsigned long long)d);
        atomicAdd((unsigned long long *)&vstat[1], (unsigned long long)d);
    }
    if (lane == 0) atomicMax((unsigned long long *)&vstat[2], (unsigned long long)(rt_now() - t0));  // [16]
}

// Frame verification through LDS rings (records under 4 GiB: the product form).
// The register loop above keeps one step in flight per wave and loads every chunk
// from its 4-B-aligned address plus the dword after it (18 loads per step). Here
// each verify wave streams like the uniform kernel's lane-group producers
// (decode_uniform.hip): exactly 9 global_load_lds_dwordx4 per step into a
// kVdSlots-slot ring, an explicit constant vmcnt wait, kVdSlots - 1 steps in flight
// (the loop is instruction-bound: six ring waves with two slots each measured
// faster than four with four, in the same LDS). A frame starts at
// any byte, so a lane group loads its block's 16-B-ALIGNED window (64 chunks,
// lane l of instruction q takes chunk 8q + l: row q of the window lands as 128
// contiguous bytes at slot + 1024q + 128fg) plus the chunk after it, and each lane
// reads its 16-B pieces back at the byte offset (5 ds_read_b32 + 4 v_alignbyte).
// Ninth instruction, lane l of the group: 0 the window's chunk 64; 1-5 the frame's
// aligned last-stripe window (first step); 6 the aligned pair of stored checksums
// holding cs[f] (first step); 7 the walk-order frame record (vrec) of the frame
// four frames ahead in this group's sequence (first step), which the step's reader
// copies into the group's 8-entry record ring. So the next frames' positions are in
// LDS before their first block is issued, with no VGPR load in the loop (its only
// vector-memory operations are the 9 counted DMAs).
#ifndef IGGY_VD_SLOTS
#define IGGY_VD_SLOTS 2  // (build knobs for same-box A/B: ring slots, ring waves per workgroup)
#endif
#ifndef IGGY_VD_NDMA
#define IGGY_VD_NDMA 6
#endif
constexpr uint32_t kVdSlots = IGGY_VD_SLOTS;            // steps in flight + the one being read
// the record of a group's frame four ahead is copied into its ring at that frame's
// start, and the issue side runs kVdSlots steps ahead of the copy: at most 4 slots
static_assert(kVdSlots >= 2 && kVdSlots <= 4, "ring deeper than the record lookahead");
constexpr uint32_t kVdNdma = IGGY_VD_NDMA;              // ring waves: the last kVdNdma of a workgroup
constexpr uint32_t kVdFirst = 8 - kVdNdma;
constexpr uint32_t kVdStep = 9 * 1024;                  // 9 DMA instructions x 64 lanes x 16 B
constexpr uint32_t kVdMeta = 8 * 9 * 16;                // 8 groups x (8 frame records + a spare)
constexpr uint32_t kVdWave = kVdSlots * kVdStep + kVdMeta;
// WG 0's chain buffer (64 KiB) overlays the rings of its first ring waves; the ones
// after it (kVdWg0First..7) verify when WG 0 is alone
constexpr uint32_t kVdWg0First = kVdFirst + (2 * kChainChunk * 8 * 8 + kVdWave - 1) / kVdWave;
static_assert(kVdWg0First <= 6, "WG 0 keeps at least two ring waves");
constexpr uint32_t kVdRecOff = kVdNdma * kVdWave;       // the ring waves' rings; then
constexpr uint32_t kVdSecOff = kVdRecOff + kVdWg0First * 1024;  // the register loop's record slots (verify_frames_claimed),
constexpr uint32_t kGenLds = kVdSecOff + 24 * 8;         // and its stripe secrets
static_assert(kGenLds + 64 <= 160 * 1024, "LDS budget (with the kernel's static LDS words)");
#ifndef IGGY_VD_SHORT_SPLIT
#define IGGY_VD_SHORT_SPLIT 1  // (build knob for same-box A/B: 0 = short frames in every wave first)
#endif
#ifndef IGGY_VD_REGWAVES
#define IGGY_VD_REGWAVES 1  // (build knob for same-box A/B: 0 = the LDS-ring waves alone)
#endif
constexpr uint32_t kVdNone = 0xFFFFFFFFu;               // vrec frame index of "no frame"

__device__ __forceinline__ uint32_t vd_nsteps(bool valid, uint64_t L) {
    if (!valid || L <= 240) return 1;  // short frames: one empty step (verify_short hashes them)
    const uint64_t nbF = (L - 1) / 1024, ns = ((L - 1) - 1024 * nbF) / 64;
    return (uint32_t)(nbF + (ns > 0));
}
// the 16 bytes at byte offset rb of the 5 dwords d
__device__ __forceinline__ uint4 vd_align(const uint32_t d[5], uint32_t rb) {
    return make_uint4(__builtin_amdgcn_alignbyte(d[1], d[0], rb), __builtin_amdgcn_alignbyte(d[2], d[1], rb),
                      __builtin_amdgcn_alignbyte(d[3], d[2], rb), __builtin_amdgcn_alignbyte(d[4], d[3], rb));
}

__device__ inline void verify_frames_dma(const uint8_t *blob, const uint8_t *dummy, const GeneralScratch &gs,
                                         uint64_t nwalk, uint64_t fbase, uint64_t fstride, uint32_t *s_claim,
                                         uint8_t *smem, uint32_t lbase, uint32_t region, int lane, uint64_t t0) {
    // smem: the dynamic LDS (generic pointer, for ds reads and writes); lbase: its LDS
    // address, which the DMA's M0 needs (the static LDS variables come first)
    const uint32_t l = lane & 7, m = l >> 1, par = l & 1, fg = (uint32_t)lane >> 3;
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
    // Every secret is waited for here, before the first DMA: a first use inside the
    // loop (the rarely taken frame-end block) got a compiler vmcnt wait that also
    // drained the ring's in-flight steps.
    {
        uint64_t sink = key0 ^ key1 ^ init0 ^ init1 ^ last0 ^ last1 ^ mrg0 ^ mrg1;
#pragma unroll
        for (int q = 0; q < 8; ++q) sink ^= s0[q] ^ s1[q];
        asm volatile("" : "+v"(sink));
    }
    // frame sequence of this group: claims from the workgroup's LDS counter, frames
    // fbase + fstride k (the register loop of the other waves claims from the same one)
    auto claim = [&]() -> uint64_t {
        uint32_t k = 0;
        if (l == 0) k = atomicAdd(s_claim, 1u);
        k = (uint32_t)__shfl((int)k, lane & ~7);
        const uint64_t f = fbase + fstride * k;
        return f < nwalk ? f : nwalk;  // nwalk: none
    };
    auto succ = [&](uint64_t f) -> uint64_t { return f < nwalk ? claim() : nwalk; };
    region = __builtin_amdgcn_readfirstlane(region);  // wave-uniform: M0 from scalar registers
    lbase = __builtin_amdgcn_readfirstlane(lbase);
    const uint32_t meta = region + kVdSlots * kVdStep + 144 * fg;  // this group's record ring
    // records of the group's first four frames, straight from vrec (before the ring starts)
    uint64_t fa = claim();
    {
        uint64_t fo = fa;
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            if (l == k) *(uint4 *)(smem + meta + 16 * k) = *(const uint4 *)(gs.vrec + 2 * fo);
            fo = succ(fo);
        }
        fa = fo;  // the frame four ahead of the issue cursor
    }
    // issue cursor: frame ordinal ij, block ib. Branch-free per lane (the group
    // branches only at a frame start): divergent paths would run in turn for the
    // wave's eight groups, and a step's instruction count bounds the loop as much as
    // its bytes do.
    uint32_t ij = 0, ib = 0, i_nsteps = 1;
    // per-frame issue state, set at the frame's first block (a group-uniform branch):
    // the window base of block 0 for this lane, its alignment, the block counts, and
    // the ninth load's address for the first block
    const uint8_t *i_g = dummy, *i_x9 = dummy;
    uint32_t i_r = 0, i_nbF = 0, i_used = 0;
    bool i_lng = false;
    auto issue = [&](uint32_t slot_off) {
        const uint32_t slot = lbase + slot_off;  // the DMA's LDS address (M0) of the slot
        const bool first = ib == 0;
        if (first) {
            const uint4 rec = *(const uint4 *)(smem + meta + 16 * (ij & 7));
            const uint64_t p = (uint64_t)rec.x | ((uint64_t)rec.y << 32);
            const uint64_t L = rec.z;
            const uint32_t f = rec.w;
            const bool valid = f != kVdNone;
            i_nsteps = vd_nsteps(valid, L);
            i_lng = valid && L > 240;
            i_nbF = (uint32_t)((L - 1) >> 10);
            const uint8_t *H = blob + p + 8;
            i_r = (uint32_t)((uintptr_t)H & 15);
            i_g = H - i_r + 16 * l;
            // the partial block's bytes: [r, r + 64 ns) of its window
            i_used = i_lng ? (uint32_t)((((L - 1) & 1023) >> 6) << 6) + i_r : 0u;
            const uint8_t *Ls = H + L - 64;
            const uint32_t rl = (uint32_t)((uintptr_t)Ls & 15);
            const uint8_t *c0 = (i_lng && i_nbF > 0 && i_r) ? i_g + 1024 : dummy;  // (l == 0)
            const uint8_t *cl = (i_lng && (l < 5 || rl)) ? Ls - rl + 16 * (l - 1) : dummy;
            const uint8_t *c6 = valid ? (const uint8_t *)(gs.cs + (f & ~1u)) : dummy;
            const uint8_t *c7 = (const uint8_t *)(gs.vrec + 2 * fa);
            i_x9 = l == 0 ? c0 : l <= 5 ? cl : l == 6 ? c6 : c7;
            fa = succ(fa);
        }
        const uint8_t *g = i_g + ((uint64_t)ib << 10);
        const bool full = i_lng && ib < i_nbF;
        // window bytes this step needs: [r, r + 1024) of a full block, [r, r + 64 ns) of the
        // partial one; a chunk is loaded when it holds one of them
        const uint32_t used = full ? 1024u + i_r : i_used;
#pragma unroll
        for (uint32_t q = 0; q < 8; ++q) glds16(128 * q + 16 * l < used ? g + 128 * q : dummy, slot + 1024u * q);
        glds16(first ? i_x9 : ((l == 0 && full && i_r) ? g + 1024 : dummy), slot + 8u * 1024u);
        if (++ib == i_nsteps) {
            ib = 0;
            ++ij;
        }
    };
    // processing cursor: frame ordinal pj, block pb
    uint32_t pj = 0, pb = 0, p_nsteps = 1, p_f = kVdNone, rb = 0, rl = 0;
    uint64_t p_L = 0, stored = 0, bad = ~0ull, nbF = 0, ns = 0;
    bool lng = false;
    uint32_t o5[5] = {0, 0, 0, 0, 0};  // LDS offsets of a piece's 5 dwords from its row (this frame's r)
    uint64_t a0 = init0, a1 = init1;
    uint4 lastp = make_uint4(0, 0, 0, 0);
    for (uint32_t k = 0; k < kVdSlots; ++k) issue(region + k * kVdStep);
    for (uint32_t k = 0;; ++k) {
        if (pb == 0) {
            const uint4 rec = *(const uint4 *)(smem + meta + 16 * (pj & 7));
            const uint64_t p = (uint64_t)rec.x | ((uint64_t)rec.y << 32);
            p_L = rec.z;
            p_f = rec.w;
            p_nsteps = vd_nsteps(p_f != kVdNone, p_L);
            lng = p_f != kVdNone && p_L > 240;
            nbF = (p_L - 1) >> 10;
            ns = ((p_L - 1) & 1023) >> 6;
            const uint32_t r = (uint32_t)((uintptr_t)(blob + p + 8) & 15);
            rb = r & 3;
            const uint32_t e = (64 * par + 16 * m + r) >> 2;
#pragma unroll
            for (uint32_t j = 0; j < 5; ++j) o5[j] = 1024u * ((e + j) >> 5) + 4u * ((e + j) & 31);
            rl = (uint32_t)((uintptr_t)(blob + p + 8 + p_L - 64) & 15);
            a0 = init0;
            a1 = init1;
        }
        if (!__ballot(p_f != kVdNone)) break;
        wait_vm_const<9 * (kVdSlots - 1)>();  // step k landed; the later steps stay in flight
        const uint32_t slot = region + (k % kVdSlots) * kVdStep;
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
        {  // first step of a frame: its last-stripe piece, stored checksum, and the record of
           // the frame four ahead into the ring (elsewhere into the group's spare entry)
            uint32_t d[5];
            const uint8_t *ls = row + 8192 + 16 + ((rl + 16 * m) & ~3u);
#pragma unroll
            for (int j = 0; j < 5; ++j) d[j] = *(const uint32_t *)(ls + 4 * j);
            const uint4 lp = vd_align(d, rl & 3);
            const uint64_t sv = *(const uint64_t *)(row + 8192 + 96 + 8 * (p_f & 1));
            const uint4 rec = *(const uint4 *)(row + 8192 + 112);
            if (l == 7) *(uint4 *)(smem + meta + 16 * (first ? (pj + 4) & 7 : 8u)) = rec;
            // (component-wise: a select of the whole uint4 went through scratch memory,
            // whose vmcnt(0) drained the DMA ring every step)
            lastp.x = first ? lp.x : lastp.x;
            lastp.y = first ? lp.y : lastp.y;
            lastp.z = first ? lp.z : lastp.z;
            lastp.w = first ? lp.w : lastp.w;
            stored = first ? sv : stored;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot read out before it is refilled
        issue(slot);  // step k + 4
        {
            const bool full = lng && pb < nbF;
            uint64_t q0[4] = {0, 0, 0, 0}, q1[4] = {0, 0, 0, 0};
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint64_t w0 = (uint64_t)pc[q].x | ((uint64_t)pc[q].y << 32);
                const uint64_t w1 = (uint64_t)pc[q].z | ((uint64_t)pc[q].w << 32);
                // partial block: stripes < ns only (a mask, not a branch per piece)
                const uint64_t use = 0ull - (uint64_t)(full || (uint64_t)(2 * q + par) < ns);
                q0[q & 3] += (mul32x32(w0 ^ s0[q]) + w1) & use;
                q1[q & 3] += (mul32x32(w1 ^ s1[q]) + w0) & use;
            }
            a0 += (q0[0] + q0[1]) + (q0[2] + q0[3]);
            a1 += (q1[0] + q1[1]) + (q1[2] + q1[3]);
            // a full block ends with the pair fold and the scramble; the even lane keeps it
            const uint64_t f0 = a0 + gdpp64<0xB1>(a0), f1 = a1 + gdpp64<0xB1>(a1);
            a0 = full ? (par ? 0 : scramble1(f0, key0)) : a0;
            a1 = full ? (par ? 0 : scramble1(f1, key1)) : a1;
            const bool fin = pb + 1 == p_nsteps;
            if (__ballot(fin && lng)) {  // some group's frame ends here: last stripe, merge, compare
                uint64_t b0 = a0 + gdpp64<0xB1>(a0), b1 = a1 + gdpp64<0xB1>(a1);
                piece(b0, b1, lastp, last0, last1);
                uint64_t t = fold64(b0 ^ mrg0, b1 ^ mrg1);
                t += gdpp64<0x4E>(t);
                t += gswz_xor4(t);
                const uint64_t h = avalanche(p_L * P64_1 + t);
                bad = (fin && lng && h != stored && bad == ~0ull) ? p_f : bad;
            }
        }
        if (++pb == p_nsteps) {
            pb = 0;
            ++pj;
        }
    }
    wait_vm_const<0>();  // the dummy steps issued past the end land before the ring is reused
    if (l == 0 && bad != ~0ull) atomicMax((unsigned long long *)&gs.misc[2], (unsigned long long)~bad);
    uint64_t *vstat = (uint64_t *)(gs.small + 512) + 14;  // phase clock: [14] last / [15] sum of loop ends
    if (lane == 0) {
        const uint64_t d = rt_now() - t0;
        atomicMax((unsigned long long *)&vstat[0], (unsigned long long)d);
        atomicAdd((unsigned long long *)&vstat[1], (unsigned long long)d);
    }
}

// Register loop beside verify_frames_dma (claims mode), in the waves before the
// ring waves. A record
// (position, hashed length, index: vrec) only ever reaches a register through a
// step's load set that the wave has already waited for: each set carries the
// records of the two frames after the one it loads (and, on a frame's first block,
// its stored checksum); while it hashes that set the wave writes them to the group's
// LDS slots, where the frame switch reads them. A record loaded at the (divergent)
// frame switch itself made the wave wait for every outstanding load there (vmcnt(0)
// once per frame), and records kept in registers were merged through scratch.
struct VStepC {
    VStep s;
    uint64_t cs;     // stored checksum of this set's frame (its first block)
    uint32_t b, o;   // (not loaded) the block this set holds and its frame's ordinal
};
__device__ __forceinline__ VFrame vd_frame(uint4 r, uint64_t nwalk) {
    VFrame v;
    v.f = r.w == kVdNone ? nwalk : r.w;
    v.p = (uint64_t)r.x | ((uint64_t)r.y << 32);
    v.L = r.z;
    v.stored = 0;
    return v;
}
// recs: this lane group's 8 record slots in LDS (by frame ordinal mod 8), at LDS
// address rbase + 128 fg (the DMA's M0 base rbase is the wave's)
__device__ inline void verify_frames_claimed(const uint8_t *blob, const GeneralScratch &gs, uint64_t nwalk,
                                             uint64_t fbase, uint64_t fstride, uint32_t *s_claim,
                                             const uint4 *recs, uint32_t rbase, const uint64_t *sec, int lane,
                                             uint64_t t0) {
    // sec: the stripe secret words in LDS (one ds_read per piece keeps two load sets
    // and the accumulators in registers without spilling)
    const uint32_t l = lane & 7, m = l >> 1, par = l & 1;
    const uint32_t poff = 16 * (m + 4 * par);
    const uint32_t sbase = par + 2 * m;  // secret word of piece q: sbase + 2q (and + 1)
    rbase = __builtin_amdgcn_readfirstlane(rbase);
    const uint64_t key0 = kSecretW8[16 + 2 * m], key1 = kSecretW8[17 + 2 * m];
    const uint64_t init0 = par ? 0 : kAccInit[2 * m], init1 = par ? 0 : kAccInit[2 * m + 1];
    const uint64_t last0 = kSecretLast[2 * m], last1 = kSecretLast[2 * m + 1];
    const uint64_t mrg0 = kSecretMerge[2 * m], mrg1 = kSecretMerge[2 * m + 1];
    auto claim = [&]() -> uint64_t {
        uint32_t k = 0;
        if (l == 0) k = atomicAdd(s_claim, 1u);
        k = (uint32_t)__shfl((int)k, lane & ~7);
        const uint64_t f = fbase + fstride * k;
        return f < nwalk ? f : nwalk;
    };
    // issue cursor: frame icur (ordinal io, block ib), then the claimed frames n1, n2.
    // The records of frames 0 and 1 come straight from vrec, before the loop.
    const uint64_t f0 = claim();
    const uint64_t f1 = f0 < nwalk ? claim() : nwalk;
    if (l < 2) *(uint4 *)&recs[l] = *(const uint4 *)(gs.vrec + 2 * (l == 0 ? f0 : f1));
    VFrame icur = vd_frame(recs[0], nwalk);
    uint64_t n1 = f1, n2 = n1 < nwalk ? claim() : nwalk;
    // every prologue load is waited for here, before the loop: a first use inside it
    // (the merge at the loop head) drew a compiler vmcnt wait there on every iteration
    asm volatile("" ::"v"(key0), "v"(key1), "v"(init0), "v"(init1), "v"(last0), "v"(last1), "v"(mrg0), "v"(mrg1));
    asm volatile("" ::"v"(icur.p), "v"(icur.L), "v"(icur.f));
    uint32_t ib = 0, io = 0;
    bool sw = false;  // the next set starts frame n1
    auto issue = [&](VStepC &Y) {
        if (sw) {  // the next frame: its record was DMA'd by a set the wave has waited for
            icur = vd_frame(recs[(io + 1) & 7], nwalk);
            if (n1 >= nwalk) icur.f = nwalk;
            n1 = n2;
            n2 = n1 < nwalk ? claim() : nwalk;
            ib = 0;
            ++io;
        }
        vissue(blob, icur, nwalk, ib, par, poff, m, Y.s);
        Y.cs = gs.cs[(icur.f < nwalk && ib == 0) ? icur.f : 0];
        Y.b = ib;
        Y.o = io;
        {  // the records of the next two frames into their slots (lanes (io+1)&7, (io+2)&7)
            const uint32_t l1 = (io + 1) & 7, l2 = (io + 2) & 7;
            if (l == l1 || l == l2) glds16(gs.vrec + 2 * (l == l1 ? n1 : n2), rbase);
        }
        ++ib;
        sw = icur.f < nwalk && ib == vd_nsteps(true, icur.L);
    };
    uint64_t a0 = init0, a1 = init1, stored = 0, bad = ~0ull;
    uint4 lastp = make_uint4(0, 0, 0, 0);
    auto step = [&](VStepC &X, VStepC &Y) {
        issue(Y);
        // X has landed on every path (also the ones that skip the hashing): otherwise the
        // compiler waited for X at the next loop head, after Y was issued, i.e. for Y too
#pragma unroll
        for (int q = 0; q < 8; ++q)
            asm volatile("" ::"v"(X.s.v[q].x), "v"(X.s.v[q].y), "v"(X.s.v[q].z), "v"(X.s.v[q].w), "v"(X.s.nx[q]));
        asm volatile("" ::"v"(X.s.last.x), "v"(X.s.last.y), "v"(X.s.last.z), "v"(X.s.last.w), "v"(X.s.lnx), "v"(X.cs));
        const VFrame xf = vd_frame(recs[X.o & 7], nwalk);  // X's frame (its slot is not reused before ordinal + 8)
        if (xf.f >= nwalk) return;
        const uint64_t L = xf.L;
        const uint32_t b = X.b;
        const bool lng = L > 240;
        {  // a frame's first block: fresh accumulators, its stored checksum and last-stripe
           // piece (selects per component: a conditional uint4 went through scratch memory)
            const bool first = b == 0;
            const uint4 lp = realign(X.s.last, X.s.lnx, (uint32_t)((uintptr_t)(blob + xf.p + 8 + L) & 3));
            a0 = first ? init0 : a0;
            a1 = first ? init1 : a1;
            stored = first ? X.cs : stored;
            lastp.x = first ? lp.x : lastp.x;
            lastp.y = first ? lp.y : lastp.y;
            lastp.z = first ? lp.z : lastp.z;
            lastp.w = first ? lp.w : lastp.w;
        }
        if (!lng) return;
        const uint64_t nbF = (L - 1) / 1024, ns = ((L - 1) - 1024 * nbF) / 64;
        const uint32_t r = (uint32_t)((uintptr_t)(blob + xf.p + 8) & 3);
        uint4 pc[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) pc[q] = realign(X.s.v[q], X.s.nx[q], r);
        if (b < nbF) {
            uint64_t p0[4] = {0, 0, 0, 0}, p1[4] = {0, 0, 0, 0};
#pragma unroll
            for (int q = 0; q < 8; ++q) piece(p0[q & 3], p1[q & 3], pc[q], sec[sbase + 2 * q], sec[sbase + 2 * q + 1]);
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
                if (2 * q + par < ns) piece(a0, a1, pc[q], sec[sbase + 2 * q], sec[sbase + 2 * q + 1]);
        }
        if (b + 1 == vd_nsteps(true, L)) {
            a0 += gdpp64<0xB1>(a0);
            a1 += gdpp64<0xB1>(a1);
            piece(a0, a1, lastp, last0, last1);
            uint64_t t = fold64(a0 ^ mrg0, a1 ^ mrg1);
            t += gdpp64<0x4E>(t);
            t += gswz_xor4(t);
            const uint64_t h = avalanche(L * P64_1 + t);
            if (h != stored && bad == ~0ull) bad = xf.f;
        }
    };
    VStepC A, B;
    issue(A);
    bool more = true;
    while (more) {
        step(A, B);
        more = __ballot(vd_frame(recs[B.o & 7], nwalk).f < nwalk) != 0;
        if (!more) break;
        step(B, A);
        more = __ballot(vd_frame(recs[A.o & 7], nwalk).f < nwalk) != 0;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last record DMAs land before the LDS is reused
    if (l == 0 && bad != ~0ull) atomicMax((unsigned long long *)&gs.misc[2], (unsigned long long)~bad);
    uint64_t *vstat = (uint64_t *)(gs.small + 512) + 14;  // phase clock: [14] last / [15] sum of loop ends
    if (lane == 0) {
        const uint64_t d = rt_now() - t0;
        atomicMax((unsigned long long *)&vstat[0], (unsigned long long)d);
        atomicAdd((unsigned long long *)&vstat[1], (unsigned long long)d);
    }
}

// ------------------------------------------------------------------ kernel
template <bool VERIFY>
__global__ __launch_bounds__(kGenThreads) void k_decode_general(const uint8_t *__restrict__ body,
                                                        uint64_t len, uint64_t *frame_pos,
                                                        uint64_t cap, iggy_decode_result *result,
                                                        GeneralScratch gs) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // the uniform kernel of this decode has completed (stream order): re-arm its
        // sync words for the next decode, whether or not it finished cleanly
        __hip_atomic_store(gs.u_exited, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(gs.u_first_bad, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(gs.u_spec_fail, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // positions of a record the uniform kernel decoded by lane groups (kPosEpilogue):
    // frame i at i * S, one 8-B store per thread and pass, the whole grid
    // (both words loaded before either is tested: one memory latency for the common
    // early exit of a decode the uniform kernel finished, not two)
    const uint64_t npos = __hip_atomic_load(&gs.misc[kPosCountWord], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t ustatus = __hip_atomic_load(&result->status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (npos) {
        const uint64_t S = __hip_atomic_load(&gs.misc[kPosStrideWord], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
        for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < npos; i += nth) frame_pos[i] = i * S;
        return;
    }
    if (ustatus != kStatusNeedGeneral) return;
    const uint64_t t0 = rt_now();
    __shared__ uint32_t s_mem[3];
    // dynamic LDS (kGenLds, Verify only): the verify waves' rings (verify_frames_dma); in
    // WG 0 its first 64 KiB hold the chain's staged block sums instead
    extern __shared__ __attribute__((aligned(16))) uint8_t s_gdyn[];
    uint64_t *s_cbuf = (uint64_t *)s_gdyn;
    __shared__ uint32_t s_cflags[3];
    if (threadIdx.x < 3) s_cflags[threadIdx.x] = 0;  // (ordered by the barriers before phase D + F)
    join_members(gs, t0, s_mem);
    const uint32_t member = s_mem[0];
    if (member == kNotMember) return;  // registered after the close: the members do the work
    const uint32_t nwg = s_mem[1];     // members (all resident)
    const iggy_batch_header h = result->header;
    const uint8_t *blob = body + kHdr;
    const uint64_t bl = h.batch_length - kHdr;
    const uint64_t gtid = (uint64_t)member * blockDim.x + threadIdx.x;
    const uint64_t gthreads = (uint64_t)nwg * blockDim.x;
    const uint64_t T = tile_bytes(bl, h.message_count);
    const uint64_t ntiles = (bl + T - 1) / T;
    const uint64_t ngroups = (ntiles + kGrpTiles - 1) / kGrpTiles;
    const uint64_t lcap = tile_list_cap(T);
    const int lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    const uint64_t nwaves = gthreads >> 6;
    // wave ids interleaved across workgroups (wave-major): a phase with fewer work
    // items than lanes (locate: 68 K tiles for C3 against 131 K lanes) spreads over
    // every CU, one wave per SIMD first, instead of filling half the CUs two deep
    const uint64_t wid = (uint64_t)wave * nwg + member;
    uint32_t phase = 0;
    bool ok = true;

    // ---------------- A: locate
    if (threadIdx.x == 0) s_mem[2] = 0;  // the verify tail's claim counter (ordered by the barriers)
    for (uint64_t t = 64 * wid + lane; t < ntiles; t += gthreads) {
        const uint64_t lo = t * T, hi = min(lo + T, bl);
        uint32_t *list = gs.tile_list + t * lcap;
        uint64_t *lcs = VERIFY ? gs.tile_lcs + t * lcap : nullptr;
        uint64_t s = kNoStart, x = kNoStart;
        uint32_t cnt = 0;
        if (t == 0) {
            s = 0;
            cnt = walk_located(blob, bl, 0, hi, &x, list, 0, lcs);
        } else {
            pick_start(blob, bl, lo, hi, list, lcs, &s, &x, &cnt);
        }
        gs.tile_s[t] = s;
        gs.tile_cnt[t] = cnt;
        gs.tile_x[t] = x;
    }
    ok &= grid_barrier2(gs.bar2, member, nwg, ++phase, t0);
    gstamp(gs, member, 1, rt_now() - t0);
    gstamp(gs, member, 14, 0); gstamp(gs, member, 15, 0); gstamp(gs, member, 16, 0); gstamp(gs, member, 18, 0);  // verify / chain clock (below)

    // ---------------- B1: group summaries (one wave per 256 tiles, 4 per lane)
    for (uint64_t g = wid; g < ngroups; g += nwaves) {
        // lane-local fold over its 4 tiles, assuming the lane is entered at its first start
        const uint64_t tb = (uint64_t)kGrpTiles * g + 4 * lane;
        bool lhas = false, lok = true, lterm = false;
        uint64_t ls = kNoStart, lx = 0, lhi = 0;
        uint32_t lc = 0, pre[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint64_t t = tb + i;
            pre[i] = kNotLive;
            if (t >= ntiles || lterm) continue;
            const uint64_t s = gs.tile_s[t], x = gs.tile_x[t];
            const uint32_t c = gs.tile_cnt[t];
            const uint64_t hi_t = min((t + 1) * T, bl);
            lhi = hi_t;
            if (s != kNoStart && !(lhas && lx >= hi_t)) {  // else spanned by the running frame
                if (lhas) lok &= s == lx;
                else ls = s;
                lhas = true;
                pre[i] = lc;
                lc += c;
                lx = x;
                lterm = (x & kStopBit) || x >= bl;
            } else if (lhas) {
                lok &= lx >= hi_t;  // must be spanned by the frame that entered it
            }
        }
        const uint64_t termmask = __ballot(lhas && lterm);
        const int last = termmask ? __builtin_ctzll(termmask) : 63;
        const bool live = lhas && lane <= last;
        const uint64_t hasmask = __ballot(live);
        uint64_t S = kNoStart, X = 0, CNT = 0, flags = kGrpOk;
        uint32_t lpre = 0;
        if (hasmask) {
            const int f0 = __builtin_ctzll(hasmask);
            const int lh = 63 - __builtin_clzll(hasmask);
            uint64_t pm = live ? lx : 0;  // max exit over live lanes up to this one
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint64_t o = __shfl_up(pm, d);
                if (lane >= d) pm = max(pm, o);
            }
            const uint64_t pred = __shfl_up(pm, 1);
            const bool okl = lane < f0 || lane > last || lhi == 0 ||
                             (lok && (lane == f0 || (lhas ? ls == pred : pred >= lhi)));
            if (__ballot(!okl)) flags = 0;
            const uint64_t c = live ? lc : 0;
            uint64_t inc = c;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint64_t o = __shfl_up(inc, d);
                if (lane >= d) inc += o;
            }
            lpre = (uint32_t)(inc - c);
            S = __shfl(ls, f0);
            X = __shfl(lx, lh);
            CNT = __shfl(inc, 63);
            if (termmask) flags |= kGrpTerm;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint64_t t = tb + i;
            if (t < ntiles) gs.tile_pre[t] = (live && pre[i] != kNotLive) ? lpre + pre[i] : kNotLive;
        }
        if (lane == 0) {
            uint64_t *q = gs.grp + kGrpWords * g;
            q[0] = S; q[1] = X; q[2] = CNT; q[3] = flags;
        }
    }
    ok &= grid_barrier2(gs.bar2, member, nwg, ++phase, t0);
    gstamp(gs, member, 2, rt_now() - t0);

    // ---------------- B2: link (one wave)
    if (member == 0 && wave == 0) {
        uint64_t e = 0;      // true entry into the next group
        uint64_t total = 0;  // frames accepted so far
        bool ended = false;  // the walk stopped (stop bit) or reached the blob end
        uint64_t nfast = 0, nsum = 0, nspan = 0, nrep = 0;  // diagnostics
        uint64_t G0 = 0;
        while (G0 < ngroups) {
            const uint64_t g = G0 + lane;
            const bool in = g < ngroups;
            uint64_t *q = gs.grp + kGrpWords * g;
            if (ended) {
                if (in) q[5] = 0;
                G0 += 64;
                continue;
            }
            const uint64_t S = in ? q[0] : kNoStart, X = in ? q[1] : 0, CNT = in ? q[2] : 0;
            const uint64_t flags = in ? q[3] : 0;
            const bool has = S != kNoStart;
            const uint64_t ghi = min(min((uint64_t)kGrpTiles * (g + 1), ntiles) * T, bl);
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
            const bool okl = !in || lane > last || ((flags & kGrpOk) && (has ? S == pred : pred >= ghi));
            const uint64_t badmask = __ballot(!okl);
            // lanes before the first failing one are accepted as summarised
            const int nacc = badmask ? __builtin_ctzll(badmask) : 64;
            if (nacc > 0) {
                const bool acc = in && lane < nacc;
                const uint64_t c = (acc && has && lane <= last) ? CNT : 0;
                uint64_t inc = c;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint64_t o = __shfl_up(inc, d);
                    if (lane >= d) inc += o;
                }
                if (acc) {
                    q[4] = total + inc - c;
                    q[5] = (has && lane <= last) ? 1 : 0;
                }
                total += __shfl(inc, 63);
                ++nfast;
                if (termmask && last < nacc) {
                    e = __shfl(X, last);
                    ended = true;
                } else {
                    e = max(e, __shfl(pm, nacc - 1));
                }
            }
            if (nacc == 64 || ended) {
                G0 += 64;
                continue;
            }
            // group G0 + nacc, exactly
            const uint64_t gg = G0 + nacc;
            if (gg >= ngroups) break;
            const uint64_t Sl = __shfl(S, nacc), Xl = __shfl(X, nacc), Cl = __shfl(CNT, nacc);
            const uint64_t Fl = __shfl(flags, nacc), ghl = __shfl(ghi, nacc);
            uint64_t *ql = gs.grp + kGrpWords * gg;
            G0 = gg + 1;
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
            // tile by tile: lane l holds tiles 4l..4l+3 of the group
            uint64_t ts[4], tx[4];
            uint32_t tc[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint64_t t = (uint64_t)kGrpTiles * gg + 4 * lane + i;
                const bool tin = t < ntiles;
                ts[i] = tin ? gs.tile_s[t] : kNoStart;
                tx[i] = tin ? gs.tile_x[t] : 0;
                tc[i] = tin ? gs.tile_cnt[t] : 0;
            }
            // Parallel repair. From tile k0 (true entry e), every lane folds its 4
            // tiles twice: as B1 assumed (its first start entered, later tiles entered
            // at their start unless the running exit spans them) and as the true walk
            // does given the exits of the lanes before it. The first tile where the
            // two disagree (or the true walk finds no start at its entry) is the first
            // break in sequential order: every tile before it is accepted as listed,
            // that tile is re-walked from its true entry, and the next pass starts
            // after it. One scan + one walk per break.
            const uint64_t gt0 = (uint64_t)kGrpTiles * gg;
            uint32_t k0 = 0;
            while (!ended && k0 < kGrpTiles && gt0 + k0 < ntiles) {
                // pass 1: the lane's exit as B1 assumed it
                bool seen = false, lterm = false;
                uint64_t lx = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t k = 4 * lane + i;
                    const uint64_t t = gt0 + k;
                    if (k < k0 || t >= ntiles || lterm || ts[i] == kNoStart) continue;
                    const uint64_t hi = min((t + 1) * T, bl);
                    if (seen && lx >= hi) continue;  // spanned
                    seen = true;
                    lx = tx[i];
                    lterm = (lx & kStopBit) || lx >= bl;
                }
                const uint64_t tm = __ballot(seen && lterm);
                const int tl = tm ? __builtin_ctzll(tm) : 63;
                uint64_t pm = (seen && lane <= tl) ? lx : 0;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint64_t o = __shfl_up(pm, d);
                    if (lane >= d) pm = max(pm, o);
                }
                uint64_t r = __shfl_up(pm, 1);
                if (lane == 0) r = 0;
                r = max(r, e);
                // pass 2: the true walk through the lane vs the assumption
                uint32_t kbad = kGrpTiles;
                uint64_t ebad = 0;
                bool aseen = false, stop = false;
                uint64_t ax = 0;
                uint32_t live = 0;  // bit i: tile i entered at its start by the true walk
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t k = 4 * lane + i;
                    const uint64_t t = gt0 + k;
                    if (k < k0 || t >= ntiles || stop || kbad != kGrpTiles || lane > tl) continue;
                    const uint64_t hi = min((t + 1) * T, bl);
                    const bool has = ts[i] != kNoStart;
                    const bool assumed = has && (!aseen || ax < hi);
                    bool fail;
                    if (r >= hi) {
                        fail = assumed;  // truly spanned
                    } else {
                        fail = !has || ts[i] != r || !assumed;
                    }
                    if (fail) {
                        kbad = k;
                        ebad = r;
                        continue;
                    }
                    if (assumed) {
                        aseen = true;
                        ax = tx[i];
                        live |= 1u << i;
                        r = tx[i];
                        stop = (r & kStopBit) || r >= bl;
                    }
                }
                uint32_t kb = kbad;
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) kb = min(kb, (uint32_t)__shfl_xor((int)kb, d));
                // accept tiles [k0, kb)
                uint64_t c = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (((live >> i) & 1) && 4 * (uint32_t)lane + i < kb) c += tc[i];
                uint64_t inc = c;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint64_t o = __shfl_up(inc, d);
                    if (lane >= d) inc += o;
                }
                uint64_t run = total + inc - c;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t k = 4 * lane + i;
                    const uint64_t t = gt0 + k;
                    if (k < k0 || k >= kb || t >= ntiles) continue;
                    const bool lv = (live >> i) & 1;
                    gs.tile_e[t] = lv ? ts[i] : ~0ull;
                    if (lv) {
                        gs.tile_base[t] = run;
                        run += tc[i];
                    }
                }
                total += __shfl(inc, 63);
                if (kb == kGrpTiles) {  // the rest of the group agreed
                    if (tm) {
                        e = __shfl(lx, tl);
                        ended = true;
                    } else {
                        e = max(e, __shfl(pm, 63));
                    }
                    k0 = kGrpTiles;
                    break;
                }
                // re-walk tile kb from its true entry (no frames when the entry spans it)
                const uint32_t owner = kb >> 2;
                const uint64_t eb = __shfl(ebad, (int)owner);
                const uint64_t t = gt0 + kb;
                const uint64_t lo = t * T, hi = min(lo + T, bl);
                uint64_t x2 = 0;
                uint32_t c2 = 0;
#ifdef IGGY_CODEC_DIAG
                if (lane == 0 && nrep < 2) {  // what the first repairs re-walked (scripts/diag_general.py)
                    uint64_t *st = (uint64_t *)(gs.small + 512) + 20 + 6 * nrep;
                    st[0] = t; st[1] = eb - lo; st[2] = gs.tile_s[t] - lo;
                    st[3] = gs.tile_cnt[t]; st[4] = gs.tile_x[t] - lo;
                }
#endif
                if (lane == 0) {
                    c2 = walk(blob, bl, eb, hi, &x2, gs.tile_list + t * lcap, lo, VERIFY ? gs.tile_lcs + t * lcap : nullptr);
                    gs.tile_cnt[t] = c2;
                    gs.tile_e[t] = eb;
                    gs.tile_base[t] = total;
#ifdef IGGY_CODEC_DIAG
                    if (nrep < 2) ((uint64_t *)(gs.small + 512))[25 + 6 * nrep] = c2 | ((x2 - lo) << 32);
#endif
                }
                x2 = __shfl(x2, 0);
                c2 = (uint32_t)__shfl((int)c2, 0);
                total += c2;
                e = x2;
                if ((e & kStopBit) || e >= bl) ended = true;
                k0 = kb + 1;
            }
            // the walk ended inside the group: later tiles start no frames
            if (ended) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t k = 4 * lane + i;
                    if (k >= k0 && gt0 + k < ntiles) gs.tile_e[gt0 + k] = ~0ull;
                }
            }
            if (lane == 0) ql[5] = 2;
            ++nrep;
        }
        if (lane == 0) {
            uint64_t *st = (uint64_t *)(gs.small + 512);
            st[8] = nfast; st[9] = nsum; st[10] = nspan; st[11] = nrep; st[12] = ntiles; st[13] = T;
            __hip_atomic_store(&gs.misc[0], total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&gs.misc[1], e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    ok &= grid_barrier2(gs.bar2, member, nwg, ++phase, t0);
    gstamp(gs, member, 3, rt_now() - t0);

    const uint64_t nwalk = __hip_atomic_load(&gs.misc[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // ---------------- C: scatter the accepted tiles' lists (walk order): frame positions
    // and the stored checksums locate listed beside them. Sixteen lanes per tile, four
    // tiles per wave; each pass takes kScatU tile quads and issues each load round
    // (group word -> tile prefix and count -> list entries) for all of them together,
    // since the phase is a chain of dependent load rounds.
    {
        constexpr int kScatU = 4, kScatK = 2;  // quads per pass; list entries per lane before the remainder loop
        const uint32_t sub = (uint32_t)lane >> 4, k0 = (uint32_t)lane & 15;
        const uint64_t nquads = (ntiles + 3) / 4;
        for (uint64_t q0 = wid; q0 < nquads; q0 += (uint64_t)kScatU * nwaves) {
            uint64_t t[kScatU], mode[kScatU], g4[kScatU], base[kScatU], te[kScatU], tb[kScatU];
            uint32_t pre[kScatU], cnt[kScatU];
#pragma unroll
            for (int u = 0; u < kScatU; ++u) {
                t[u] = (q0 + (uint64_t)u * nwaves) * 4 + sub;
                const uint64_t tt = t[u] < ntiles ? t[u] : 0;
                const uint64_t *q = gs.grp + kGrpWords * (tt / kGrpTiles);
                mode[u] = t[u] < ntiles ? q[5] : 0;
                g4[u] = q[4];
                pre[u] = gs.tile_pre[tt];
                te[u] = gs.tile_e[tt];  // (read for every mode, used by repaired groups only)
                tb[u] = gs.tile_base[tt];
                cnt[u] = gs.tile_cnt[tt];
            }
#pragma unroll
            for (int u = 0; u < kScatU; ++u) {
                bool live = false;
                base[u] = 0;
                if (mode[u] == 1) {
                    live = pre[u] != kNotLive;
                    base[u] = g4[u] + pre[u];
                } else if (mode[u] == 2) {
                    live = te[u] != ~0ull;
                    base[u] = tb[u];
                }
                if (!live) cnt[u] = 0;
            }
            uint32_t off[kScatU][kScatK];
            uint64_t lc[kScatU][kScatK];
#pragma unroll
            for (int u = 0; u < kScatU; ++u)
#pragma unroll
                for (int j = 0; j < kScatK; ++j) {
                    const uint32_t k = k0 + 16 * j;
                    const uint64_t li = k < cnt[u] ? t[u] * lcap + k : 0;
                    off[u][j] = gs.tile_list[li];
                    lc[u][j] = VERIFY ? gs.tile_lcs[li] : 0;
                }
#pragma unroll
            for (int u = 0; u < kScatU; ++u) {
                const uint64_t lo = t[u] * T;
#pragma unroll
                for (int j = 0; j < kScatK; ++j) {
                    const uint32_t k = k0 + 16 * j;
                    if (k >= cnt[u]) continue;
                    const uint64_t p = lo + off[u][j], i = base[u] + k;
                    gs.fpos[i] = p;
                    if (VERIFY) gs.cs[i] = lc[u][j];
                    if (frame_pos && i < cap) frame_pos[i] = p;
                }
                // tiles of more than 16 * kScatK frames (small frames): the rest a round at a time
                for (uint32_t k = k0 + 16 * kScatK; k < cnt[u]; k += 16) {
                    const uint64_t li = t[u] * lcap + k;
                    const uint64_t p = lo + gs.tile_list[li], i = base[u] + k;
                    gs.fpos[i] = p;
                    if (VERIFY) gs.cs[i] = gs.tile_lcs[li];
                    if (frame_pos && i < cap) frame_pos[i] = p;
                }
            }
        }
    }
    ok &= grid_barrier2(gs.bar2, member, nwg, ++phase, t0);
    gstamp(gs, member, 4, rt_now() - t0);

    // ---------------- E: checksum-input block sums (one wave per block)
    const uint64_t n = 44 + 8 * nwalk;
    const bool long_cs = VERIFY && n > 240;
    uint64_t nb = 0, Mreg = 0;
    if (long_cs) {
        nb = (n - 1) / 1024;
        const uint64_t ns = ((n - 1) - 1024 * nb) / 64;
        Mreg = 8 * (16 * nb + ns);
        const uint64_t sec[2] = {block_word_secret(0, lane), block_word_secret(1, lane)};
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
                    y += v;
                    x += mul32x32(v ^ sec[half]);
                }
            }
            x += __shfl_xor(x, 8); y += __shfl_xor(y, 8);
            x += __shfl_xor(x, 16); y += __shfl_xor(y, 16);
            x += __shfl_xor(x, 32); y += __shfl_xor(y, 32);
            const uint64_t t8 = x + __shfl_xor(y, 1);
            if (lane < 8) gs.bsums[b * 8 + lane] = t8;
        }
    }
    // walk-order frame records for verify_frames_dma (vrec), and the "none" record after them
    const bool vdma = VERIFY && bl < (1ull << 32) && !(kDiagMask && (gs.dbg & 0x200000));
    if (vdma) {
        if (threadIdx.x < 24) ((uint64_t *)(s_gdyn + kVdSecOff))[threadIdx.x] = kSecretW8[threadIdx.x];
        const uint64_t wend = __hip_atomic_load(&gs.misc[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ~kStopBit;
        // kVrecU records per pass, their loads issued before any store (a store ahead
        // of the next record's loads would make them wait for its acknowledgement)
        for (uint64_t f0 = gtid; f0 <= nwalk; f0 += (uint64_t)kVrecU * gthreads) {
            uint64_t pa[kVrecU], pb[kVrecU];
#pragma unroll
            for (int u = 0; u < kVrecU; ++u) {
                const uint64_t f = f0 + (uint64_t)u * gthreads;
                pa[u] = f < nwalk ? gs.fpos[f] : 0;
                pb[u] = f + 1 < nwalk ? gs.fpos[f + 1] : wend;  // frames tile the walk
            }
#pragma unroll
            for (int u = 0; u < kVrecU; ++u) {
                const uint64_t f = f0 + (uint64_t)u * gthreads;
                if (f > nwalk) continue;
                uint4 v = make_uint4(0, 0, 0, kVdNone);
                if (f < nwalk) {
                    const uint64_t p = pa[u], L = pb[u] - p - 8;
                    v = make_uint4((uint32_t)p, (uint32_t)(p >> 32), (uint32_t)L, (uint32_t)f);
                }
                *(uint4 *)(gs.vrec + 2 * f) = v;
            }
        }
    }
    // (a grid barrier, not a block-sum count only the chain wave waits for: with the
    // verify waves going straight on, the C3 decode measured 15-25 us slower)
    ok &= grid_barrier2(gs.bar2, member, nwg, ++phase, t0);
    gstamp(gs, member, 5, rt_now() - t0);

    // ---------------- D + F: chain (wave 0 of WG 0) beside frame verification
    uint64_t computed = 0;
    // WG 0: wave 0 chains, wave 1 stages its block sums through LDS (chain_stager);
    // every other wave verifies
    if (member == 0 && wave == 0) {
        if (long_cs) {
            const int j = lane & 7;
            uint64_t acc = 0;
            if (!chain_staged(nb, s_cbuf, s_cflags, lane, t0, acc)) ok = false;
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
            if (lane == 0) ((uint64_t *)(gs.small + 512))[18] = rt_now() - t0;  // phase clock: chain done
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
    } else if (member == 0 && wave == 1 && long_cs) {
        chain_stager(gs.bsums, nb, s_cbuf, s_cflags, lane, t0);
    } else if (VERIFY && vdma) {
        // Frames of <= 240 B first, a slice per wave of every WG. Then the long frames,
        // claimed one per lane group from the workgroup's LDS counter (WG member m of
        // the verifying set takes frames m + nv k, a chip-wide front) by two loops side
        // by side: the last kVdNdma waves (4..7) stream through LDS rings
        // (verify_frames_dma), the others run the register loop (verify_frames_claimed);
        // the counter balances the two. WG 0 runs the chain and only verifies when it
        // is alone (its first ring waves' space holds the chain buffer).
        const uint32_t ws = long_cs ? 2 : 1;  // WG 0's waves below ws chain (and stage)
        const uint64_t wend = __hip_atomic_load(&gs.misc[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ~kStopBit;
        const bool alone = nwg == 1;
        if (IGGY_VD_SHORT_SPLIT) {
            // the short frames go to the waves that do not stream through rings (WG 0's
            // idle waves, the register-loop waves), so the rings start at once
            const bool ring = wave >= (member == 0 ? kVdWg0First : kVdFirst) && (alone || member > 0);
            if (!ring) {
                const uint32_t n0 = alone ? kVdWg0First - ws : 8 - ws;  // WG 0's share
                const uint32_t sw = member == 0 ? wave - ws : n0 + kVdFirst * (member - 1) + wave;
                const uint32_t nsw = n0 + kVdFirst * (nwg - 1);
                verify_short(blob, gs, nwalk, wend, sw, nsw, lane);
            }
        } else {
            verify_short(blob, gs, nwalk, wend, member * 8 + wave - ws, nwg * 8 - ws, lane);
        }
        if (lane == 0)  // phase clock [16]: the short frames' end
            atomicMax((unsigned long long *)((uint64_t *)(gs.small + 512) + 16), (unsigned long long)(rt_now() - t0));
        if (alone || member > 0) {
            const uint64_t fbase = alone ? 0 : member - 1, fstride = alone ? 1 : nwg - 1;
            if (wave >= (member == 0 ? kVdWg0First : kVdFirst)) {
                typedef __attribute__((address_space(3))) uint8_t lds_u8;
                const uint32_t lbase = (uint32_t)(uintptr_t)(lds_u8 *)s_gdyn;
                verify_frames_dma(blob, body, gs, nwalk, fbase, fstride, &s_mem[2], s_gdyn, lbase,
                                  (wave - kVdFirst) * kVdWave, lane, t0);
            } else if (IGGY_VD_REGWAVES) {
                if (member == 1 && wave == 0 && lane == 0) ((uint64_t *)(gs.small + 512))[17] = 8 * (nwg - 1);
                typedef __attribute__((address_space(3))) uint8_t lds_u8;
                const uint32_t lbase = (uint32_t)(uintptr_t)(lds_u8 *)s_gdyn;
                verify_frames_claimed(blob, gs, nwalk, fbase, fstride, &s_mem[2],
                                      (const uint4 *)(s_gdyn + kVdRecOff + 1024 * wave + 128 * ((uint32_t)lane >> 3)),
                                      lbase + kVdRecOff + 1024 * wave, (const uint64_t *)(s_gdyn + kVdSecOff), lane, t0);
            }
        }
    } else if (VERIFY) {
        // (records of 4 GiB and more, whose frame lengths need not fit vrec's 32 bits;
        // diagnostic bit 0x200000 forces it): the register loop in every other wave
        const uint32_t ws = long_cs ? 2 : 1;  // WG 0's waves below ws chain (and stage)
        const uint32_t vw = member * (blockDim.x >> 6) + wave - ws;
        const uint32_t nvw = nwg * (blockDim.x >> 6) - ws;
        if (vw == 0 && lane == 0) ((uint64_t *)(gs.small + 512))[17] = nvw;
        const uint64_t wend = __hip_atomic_load(&gs.misc[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ~kStopBit;
        verify_frames(blob, gs, nwalk, wend, vw, nvw, member, nwg, &s_mem[2], lane, t0, blob + bl);
    }
    ok &= grid_barrier2(gs.bar2, member, nwg, ++phase, t0);
    gstamp(gs, member, 6, rt_now() - t0);

    // ---------------- resolution (wave 0 of WG 0)
    if (member == 0 && wave == 0 && lane == 0) {
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
    // barrier, registration and misc[2] are re-armed by the next decode's uniform kernel
    (void)len;
}

template __global__ void k_decode_general<true>(const uint8_t *__restrict__, uint64_t, uint64_t *,
                                                uint64_t, iggy_decode_result *, GeneralScratch);
template __global__ void k_decode_general<false>(const uint8_t *__restrict__, uint64_t, uint64_t *,
                                                 uint64_t, iggy_decode_result *, GeneralScratch);

}  // namespace iggy

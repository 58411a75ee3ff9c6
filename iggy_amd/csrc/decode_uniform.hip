// decode_uniform.hip — decode_batch_slice_with (core/binary_protocol/src/batch.rs:391-506)
// for records whose frames share one stride S (every frame 48 + payload + user
// headers bytes long). The reference walk is a serial pointer chase
// (batch.rs:288-355); here it is replaced by speculation + parallel proof:
// frame i is assumed at i*S and EVERY frame's header is checked to have size S
// and zero reserved bytes. When all checks hold, the chain from offset 0 is
// exactly those frames, so the result is bit-identical to the serial walk.
// When a check fails, the first failing index decides whether the real walk
// stops there (result still exact) or continues with another size (status
// kStatusNeedGeneral: the general walk in decode_general.hip takes over).
//
// Work layout (MI355X: 256 CUs, wave64, 160 KiB LDS):
//  * grid = 1 consumer WG + NPROD producer WGs (one per CU, 256 threads,
//    ~154 KiB LDS). Producer g handles chunks g, g+NPROD, ... statically.
//  * a chunk = 256 consecutive frames [256c-6, 256c+250); the -6 aligns the
//    chunk with two 1024-B blocks of the batch-checksum input
//    (44 header bytes + 8 bytes per frame => word m = frame + 6).
//  * each wave owns 64 frames (one per lane) and streams them through a
//    double-buffered 16 KiB LDS image with global_load_lds_dwordx4: one
//    wave-instruction moves 4 frames x 256 contiguous bytes (full lines),
//    the image is XOR-swizzled so every lane's ds_read_b128 is conflict-free.
//  * XXH3 per lane: stripe words accumulate in registers, scramble at block
//    ends, last stripe from a per-lane side copy, merge.
//  * batch checksum: each chunk reduces its 256 checksum-input words to the
//    8 accumulator sums of its two XXH3 blocks and publishes them
//    (write-through sc1 stores + flag); the consumer WG runs the serial
//    8192-step scramble chain concurrently, fed through an LDS ring.
#include "codec_common.hpp"

#include <utility>

namespace iggy {

struct DecodeScratch {
    uint32_t *exited;     // producer WGs that finished (reset by consumer)
    uint64_t *first_bad;  // ~index of first checksum mismatch (max-encoded), 0 = none
    uint64_t *spec_fail;  // ~index of first frame whose header breaks the stride
    uint32_t *flags;      // [max_chunks] = epoch when the chunk's sums are published
    uint64_t *sums;       // [2*max_chunks][8] per-block accumulator sums
    uint64_t *errslot;    // [max_chunks*4][2] (stored, computed) per wave
    uint8_t *small;       // >= 512 B: short batch-checksum inputs
    uint64_t max_chunks;
};

// ---- LDS map of a producer WG (dynamic LDS only, base offset 0) ----------
constexpr uint32_t kWaveBuf = 16384;                  // one phase: 64 lanes x 16 chunks x 16 B
constexpr uint32_t kSideOff = 4 * 2 * kWaveBuf;      // 131072
constexpr uint32_t kSideLane = 96;                    // 6 chunks per lane
constexpr uint32_t kXchgOff = kSideOff + 4 * 64 * kSideLane;  // 155648
constexpr uint32_t kRedOff = kXchgOff + 256 * 8;      // 157696
constexpr uint32_t kLdsBytes = kRedOff + 4 * 8 * 8;   // 157952
// consumer WG reuses the space: ring of per-chunk sums + control words
constexpr uint32_t kRing = 1024;                      // chunks (128 B each) = 128 KiB
constexpr uint32_t kCtrlOff = kRing * 128;            // 131072
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");


struct UPlan {
    uint32_t state;  // 0 run, 1 result known early, 2 need general
    uint32_t nck, nph, q_side0;
    uint64_t S, N, L, nchunks;
    uint64_t nbF, Kreg;          // per-frame hash: full blocks, regular words
    uint64_t n, nb, Mreg;        // batch checksum input: bytes, full blocks, regular words
    uint32_t ekind, ereason;
    uint64_t ea, eb, ec;
    bool long_frames, long_cs;
    bool tail_unsafe;  // last frame's last 16-B chunk would read past the caller's buffer
};

__device__ inline void make_plan(const HeaderInfo &hi, const uint8_t *blob, uint64_t len,
                                 bool verify, uint64_t max_chunks, bool allow_unaligned, UPlan &p) {
    p.state = 2;
    p.tail_unsafe = false;
    p.ekind = IGGY_OK; p.ereason = 0; p.ea = p.eb = p.ec = 0;
    p.S = p.N = p.L = p.nchunks = 0;
    p.nck = p.nph = p.q_side0 = 0;
    p.nbF = p.Kreg = p.n = p.nb = p.Mreg = 0;
    p.long_frames = p.long_cs = false;
    if (hi.err_kind != IGGY_OK) {
        p.state = 1; p.ekind = hi.err_kind; p.ereason = hi.err_reason;
        p.ea = hi.ea; p.eb = hi.eb; p.ec = hi.ec;
        return;
    }
    const uint64_t bl = hi.blob_len;
    if (bl == 0) {  // zero frames walked
        p.state = 1;
        if (hi.h.message_count != 0) { p.ekind = IGGY_ERR_VALIDATION; p.ereason = IGGY_V_FRAMES_DO_NOT_TILE; }
        return;
    }
    if (bl < kFrameHdr || ld64_any(blob + 40) != 0) {  // walk stops at frame 0
        p.state = 1; p.ekind = IGGY_ERR_VALIDATION; p.ereason = IGGY_V_FRAMES_DO_NOT_TILE;
        return;
    }
    uint64_t S = kFrameHdr + (uint64_t)ld32_any(blob + 36) + (uint64_t)ld32_any(blob + 32);
    if (S > bl) {
        p.state = 1; p.ekind = IGGY_ERR_VALIDATION; p.ereason = IGGY_V_FRAMES_DO_NOT_TILE;
        return;
    }
    if (bl % S != 0 || S > (1u << 20)) return;  // not a single-stride record
    if (!allow_unaligned && ((((uintptr_t)blob) | S) & 15)) return;
    p.S = S;
    p.N = bl / S;
    p.L = S - 8;
    p.nchunks = (p.N + 6 + 255) / 256;
    if (p.nchunks > max_chunks) return;
    if (verify) {
        p.nck = (uint32_t)((S + 15) / 16);
        p.long_frames = p.L > 240;
        if (p.long_frames) {
            p.nbF = (p.L - 1) / 1024;
            uint64_t ns = ((p.L - 1) - 1024 * p.nbF) / 64;
            p.Kreg = 8 * (16 * p.nbF + ns);
            p.q_side0 = (uint32_t)((S - 64) >> 4);
        }
        p.n = 44 + 8 * p.N;
        p.long_cs = p.n > 240;
        if (p.long_cs) {
            p.nb = (p.n - 1) / 1024;
            uint64_t ns = ((p.n - 1) - 1024 * p.nb) / 64;
            p.Mreg = 8 * (16 * p.nb + ns);
        }
    } else {
        p.nck = 3;  // header bytes 0..47 only
    }
    p.nph = (p.nck + 15) / 16;
    p.tail_unsafe = hi.h.batch_length + (16ull * p.nck - S) > len;
    p.state = 0;
}

// ------------------------------------------------------------ primitives
__device__ __forceinline__ void glds16(const void *gsrc, uint32_t lds_addr) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds_addr)
        : "memory");
}
__device__ __forceinline__ void wait_vm16() { asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); }
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void lds_fence_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ uint64_t funnel64(uint64_t lo, uint64_t hi, uint32_t t) {
    return t ? ((lo >> (8 * t)) | (hi << (64 - 8 * t))) : lo;
}

// issue one phase (16 chunks per frame) for the wave's 64 frames of chunk c:
// instruction k moves frames 4k..4k+3 (16 lanes each = 256 contiguous bytes)
__device__ __forceinline__ void issue_phase(const uint8_t *blob, const UPlan &pl, int64_t iw0,
                                            uint32_t p, uint32_t lds_buf, int lane) {
    const int fsub = lane >> 4;
    int64_t i = iw0 + fsub;
    const uint8_t *fb = blob + (uint64_t)i * pl.S;  // frame base (maybe bogus if i invalid)
    const uint64_t step = 4 * pl.S;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int f = 4 * k + fsub;
        const uint32_t cidx = (uint32_t)((lane & 15) ^ (f & 15));
        const uint32_t q = 16 * p + cidx;
        const bool ok = (i >= 0) && ((uint64_t)i < pl.N) && (q < pl.nck) &&
                        !(pl.tail_unsafe && (uint64_t)i == pl.N - 1 && 16ull * q + 16 > pl.S);
        const uint8_t *src = ok ? fb + 16ull * q : blob;
        glds16(src, lds_buf + 1024u * k);
        i += 4;
        fb += step;
    }
}

// ------------------------------------------------------------- phase body
struct PhaseState {
    Acc8 acc;
    uint64_t stored, resv;
    uint32_t uh, plen;
};

// chunk C (compile-time) of phase p (p % 4 == P4) for this lane's frame.
// Returns true when the frame has no chunk C (end of the phase loop).
template <int P4, bool CHECKED, bool VERIFY, int C>
__device__ __forceinline__ bool chunk_step(const uint8_t *lbase, uint32_t sw, uint8_t *side,
                                           uint32_t p, const UPlan &pl, PhaseState &st) {
    const uint32_t q = 16 * p + C;
    if (CHECKED && q >= pl.nck) return true;
    const uint4 D = *(const uint4 *)(lbase + 16u * ((uint32_t)C ^ sw));
    const uint64_t u0 = (uint64_t)D.x | ((uint64_t)D.y << 32);
    const uint64_t u1 = (uint64_t)D.z | ((uint64_t)D.w << 32);
    if (P4 == 0 && C == 0 && CHECKED) {
        if (p == 0) st.stored = u0;
    }
    if (P4 == 0 && C == 2 && CHECKED) {
        if (p == 0) { st.uh = D.x; st.plen = D.y; st.resv = u1; }
    }
    if (!VERIFY || !pl.long_frames) return false;
    if (CHECKED && q >= pl.q_side0) *(uint4 *)(side + 16u * (q - pl.q_side0)) = D;
    // unit 2q -> hashed word k = 2q-1 ; unit 2q+1 -> word 2q
    constexpr int J0 = (2 * C - 1) & 7;
    constexpr int SIB0 = (4 * P4 + ((2 * C - 1) >> 3)) & 15;
    constexpr int J1 = (2 * C) & 7;
    constexpr int SIB1 = (4 * P4 + ((2 * C) >> 3)) & 15;
    {
        const int64_t k0 = 2 * (int64_t)q - 1;
        const bool reg0 = CHECKED ? (k0 >= 0 && (uint64_t)k0 < pl.Kreg) : true;
        if (reg0) st.acc.word<J0>(u0, Secret::w(8 * (SIB0 + J0)));
        if (C == 0 && P4 == 0) {
            if (p >= 4 && (uint64_t)(p / 4 - 1) < pl.nbF) st.acc.scramble();
        }
    }
    {
        const uint64_t k1 = 2 * (uint64_t)q;
        const bool reg1 = CHECKED ? (k1 < pl.Kreg) : true;
        if (reg1) st.acc.word<J1>(u1, Secret::w(8 * (SIB1 + J1)));
    }
    return false;
}

template <int P4, bool CHECKED, bool VERIFY, int... Cs>
__device__ __forceinline__ void phase_chunks(std::integer_sequence<int, Cs...>, const uint8_t *lbase,
                                             uint32_t sw, uint8_t *side, uint32_t p,
                                             const UPlan &pl, PhaseState &st) {
    (void)(chunk_step<P4, CHECKED, VERIFY, Cs>(lbase, sw, side, p, pl, st) || ...);
}

// Processes the 16 chunks of phase p for this lane's frame.
// CHECKED: some word of the phase may be non-regular / need side capture /
// be the frame header (p == 0).
template <int P4, bool CHECKED, bool VERIFY>
__device__ __forceinline__ void phase_body(const uint8_t *buf, uint8_t *side, int lane, uint32_t p,
                                           const UPlan &pl, PhaseState &st) {
    phase_chunks<P4, CHECKED, VERIFY>(std::make_integer_sequence<int, 16>{},
                                      buf + (uint32_t)lane * 256u, (uint32_t)(lane & 15), side, p,
                                      pl, st);
}

template <bool VERIFY>
__device__ __forceinline__ void run_phase(const uint8_t *buf, uint8_t *side, int lane, uint32_t p,
                                          const UPlan &pl, PhaseState &st) {
    // a phase is "full" when all its words are regular and none needs side capture
    const bool full = VERIFY && pl.long_frames && p > 0 && (16 * p + 15 < pl.nck) &&
                      (32ull * p + 30 < pl.Kreg) && (16 * p + 15 < pl.q_side0);
    switch (p & 3) {
        case 0:
            if (full) phase_body<0, false, VERIFY>(buf, side, lane, p, pl, st);
            else phase_body<0, true, VERIFY>(buf, side, lane, p, pl, st);
            break;
        case 1:
            if (full) phase_body<1, false, VERIFY>(buf, side, lane, p, pl, st);
            else phase_body<1, true, VERIFY>(buf, side, lane, p, pl, st);
            break;
        case 2:
            if (full) phase_body<2, false, VERIFY>(buf, side, lane, p, pl, st);
            else phase_body<2, true, VERIFY>(buf, side, lane, p, pl, st);
            break;
        default:
            if (full) phase_body<3, false, VERIFY>(buf, side, lane, p, pl, st);
            else phase_body<3, true, VERIFY>(buf, side, lane, p, pl, st);
            break;
    }
}

// short frames (hashed length 40..240): random access inside phase 0 image
__device__ inline uint64_t short_hash(const uint8_t *buf0, int lane, uint64_t L) {
    const uint32_t sw = (uint32_t)(lane & 15);
    const uint8_t *lbase = buf0 + (uint32_t)lane * 256u;
    auto unit = [&](uint32_t u) -> uint64_t {
        return *(const uint64_t *)(lbase + 16u * ((u >> 1) ^ sw) + 8u * (u & 1));
    };
    auto rd = [&](uint64_t hoff) -> uint64_t {  // hashed offset -> stream offset 8 + hoff
        uint64_t o = 8 + hoff;
        uint32_t u = (uint32_t)(o >> 3), t = (uint32_t)(o & 7);
        uint64_t lo = unit(u);
        return t ? funnel64(lo, unit(u + 1), t) : lo;
    };
    auto mix16 = [&](uint64_t off, uint64_t s0, uint64_t s1) {
        return fold64(rd(off) ^ s0, rd(off + 8) ^ s1);
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

// ------------------------------------------------------------- consumer
template <bool VERIFY>
__device__ void consumer_wg(const uint8_t *body, const HeaderInfo &hi, const UPlan &pl,
                            uint64_t *frame_pos, iggy_decode_result *result,
                            const DecodeScratch &sc, uint32_t epoch, uint32_t nprod,
                            uint8_t *smem, uint32_t dbg) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const uint8_t *blob = body + kHdr;
    uint64_t *ring = (uint64_t *)smem;
    uint32_t *ctrl = (uint32_t *)(smem + kCtrlOff);  // [0]=ready [1]=consumed [2]=alldone [3]=timeout
    if (threadIdx.x == 0) { ctrl[0] = 0; ctrl[1] = 0; ctrl[2] = 0; ctrl[3] = 0; }
    __syncthreads();
    if (wave >= 2) return;

    if (pl.state != 0) {
        if (wave != 0) return;
        // result known without producers (header errors, empty / broken first frame)
        uint32_t kind = pl.ekind, reason = pl.ereason;
        uint64_t a = pl.ea, b = pl.eb, c = pl.ec, computed = 0;
        uint32_t status = kStatusDone;
        if (pl.state == 2) {
            status = kStatusNeedGeneral;
        } else if (kind == IGGY_OK && VERIFY) {
            // zero frames: checksum over the 44 header bytes (batch.rs:452-458)
            if (lane == 0) {
                uint8_t *s = sc.small;
                uint64_t w[5] = {hi.h.partition_id, hi.h.base_offset, hi.h.base_timestamp,
                                 hi.h.origin_timestamp, hi.h.batch_length};
                for (int i = 0; i < 5; ++i)
                    for (int k = 0; k < 8; ++k) s[8 * i + k] = (uint8_t)(w[i] >> (8 * k));
                for (int k = 0; k < 4; ++k) s[40 + k] = (uint8_t)(hi.h.message_count >> (8 * k));
                computed = xxh3_64_lane(s, 44);
                if (computed != hi.h.batch_checksum) {
                    kind = IGGY_ERR_INVALID_BATCH_CHECKSUM; reason = 0;
                    a = hi.h.batch_checksum; b = computed; c = hi.h.base_offset;
                }
            }
        }
        if (lane == 0)
            write_result(result, hi, kind, reason, a, b, c, 0, computed, 1, status, 0);
        return;
    }

    const uint64_t t_start = rt_now();
    if (wave == 1) {
        // ---------------- feeder: flags -> LDS ring (sc1 loads, Guideline 16 R1)
        const uint64_t need = (VERIFY && pl.long_cs && !(dbg & 1)) ? (pl.nb >> 1) + 1 : 0;
        uint64_t c = 0;
        bool timed_out = false;
        while (c < need) {
            const uint32_t consumed = __hip_atomic_load(&ctrl[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            const uint64_t space = kRing - (c - consumed);
            uint64_t win = need - c;
            if (win > 64) win = 64;
            if (win > space) win = space;
            bool ready = false;
            if ((uint64_t)lane < win) {
                const uint64_t cc = c + lane;
                ready = cc >= pl.nchunks ||
                        __hip_atomic_load(&sc.flags[cc], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
            }
            const uint64_t mask = __ballot(ready);
            const uint32_t r = (~mask == 0) ? 64u : (uint32_t)__builtin_ctzll(~mask);  // consecutive ready
            if (r == 0) {
                __builtin_amdgcn_s_sleep(2);
                if (rt_now() - t_start > kSpinLimitTicks) { timed_out = true; break; }
                continue;
            }
            // 16 sums per chunk; + the chunk-boundary checksum word m = 256cc+255
            for (uint32_t idx = lane; idx < ((dbg & 4) ? 0u : 16 * r); idx += 64) {
                const uint64_t cc = c + idx / 16;
                const uint32_t e = idx % 16;
                uint64_t v = 0;
                if (cc < pl.nchunks)
                    v = __hip_atomic_load(&sc.sums[(2 * cc) * 8 + e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (e >= 14) {
                    const uint64_t m = 256 * cc + 255;
                    const uint64_t ia = 256 * cc + 249;  // frame whose hi32 starts word m
                    if (m < pl.Mreg && ia + 1 < pl.N) {
                        const uint64_t csa = ld64_any(blob + ia * pl.S);
                        const uint64_t csb = ld64_any(blob + (ia + 1) * pl.S);
                        const uint64_t wv = (csa >> 32) | (csb << 32);
                        // word j = 7 of stripe 15: acc[6] += v, acc[7] += mul(v ^ sec[15+7])
                        if (e == 14) v += wv;
                        else v += mul32x32(wv ^ Secret::w(8 * 22));
                    }
                }
                ring[(cc % kRing) * 16 + e] = v;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0)
                __hip_atomic_store(&ctrl[0], (uint32_t)(c + r), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            c += r;
        }
        // every producer done => every chunk's stores / atomics are visible
        while (!timed_out &&
               __hip_atomic_load(sc.exited, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != nprod) {
            __builtin_amdgcn_s_sleep(4);
            if (rt_now() - t_start > kSpinLimitTicks) timed_out = true;
        }
        if (lane == 0) {
            if (timed_out) __hip_atomic_store(&ctrl[3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_store(&ctrl[2], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        return;
    }

    // ---------------- wave 0: serial batch-checksum chain + resolution
    uint64_t computed = 0;
    bool timed_out = false;
    if (VERIFY && pl.long_cs && !(dbg & 1)) {
        const int j = lane & 7;
        uint64_t acc = kAccInit[j];
        const uint64_t key = kSecretW8[16 + j];
        // words 0..5 of stripe 0: header fields, then count | lo32(cs_0)
        {
            const uint64_t cs0 = ld64_any(blob);
            const uint64_t w6[6] = {hi.h.partition_id, hi.h.base_offset, hi.h.base_timestamp,
                                    hi.h.origin_timestamp, hi.h.batch_length,
                                    (uint64_t)hi.h.message_count | (cs0 << 32)};
#pragma unroll
            for (int m = 0; m < 6; ++m) {
                if (j == (m ^ 1)) acc += w6[m];
                if (j == m) acc += mul32x32(w6[m] ^ Secret::w(8 * m));
            }
        }
        uint32_t ready = 0;
        uint64_t b = 0;
        while (b <= pl.nb) {
            const uint64_t cc = b >> 1;
            if (cc >= ready) {
                ready = __hip_atomic_load(&ctrl[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (cc >= ready) {
                    if (__hip_atomic_load(&ctrl[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                        timed_out = true;  // feeder gave up
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
            }
            // run every block that is ready without re-polling
            uint64_t bend = 2 * (uint64_t)ready;
            if (bend > pl.nb + 1) bend = pl.nb + 1;
            for (; b < bend; ++b) {
                acc += ring[((b >> 1) % kRing) * 16 + (b & 1) * 8 + j];
                if (b < pl.nb) acc = scramble1(acc, key);
                if ((b & 1) && lane == 0)
                    __hip_atomic_store(&ctrl[1], (uint32_t)((b >> 1) + 1), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        if (!timed_out) {
            // last stripe = stored checksums of frames N-8 .. N-1 (secret offset 121)
            const uint64_t v = ld64_any(blob + (pl.N - 8 + j) * pl.S);
            const uint64_t vx = __shfl_xor(v, 1);
            acc += vx;
            acc += mul32x32(v ^ kSecretLast[j]);
            uint64_t a[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) a[i] = __shfl(acc, i);
            uint64_t r = pl.n * P64_1;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                r += fold64(a[2 * i] ^ Secret::w(11 + 16 * i), a[2 * i + 1] ^ Secret::w(19 + 16 * i));
            computed = avalanche(r);
        }
    } else if (VERIFY && !pl.long_cs) {
        // short checksum input (N <= 24): hash it directly
        if (lane == 0) {
            uint8_t *s = sc.small;
            uint64_t w[5] = {hi.h.partition_id, hi.h.base_offset, hi.h.base_timestamp,
                             hi.h.origin_timestamp, hi.h.batch_length};
            for (int i = 0; i < 5; ++i)
                for (int k = 0; k < 8; ++k) s[8 * i + k] = (uint8_t)(w[i] >> (8 * k));
            for (int k = 0; k < 4; ++k) s[40 + k] = (uint8_t)(hi.h.message_count >> (8 * k));
            for (uint64_t i = 0; i < pl.N; ++i) {
                const uint64_t cs = ld64_any(blob + i * pl.S);
                for (int k = 0; k < 8; ++k) s[44 + 8 * i + k] = (uint8_t)(cs >> (8 * k));
            }
            computed = xxh3_64_lane(s, pl.n);
        }
    }
    // last frame when its final chunk could not be staged
    uint64_t tail_stored = 0, tail_computed = 0;
    bool tail_bad = false;
    if (VERIFY && pl.tail_unsafe && lane == 0) {
        const uint8_t *f = blob + (pl.N - 1) * pl.S;
        tail_stored = ld64_any(f);
        tail_computed = xxh3_64_lane(f + 8, pl.L);
        tail_bad = tail_stored != tail_computed;
    }
    // wait for the feeder's "all producers done"
    while (!__hip_atomic_load(&ctrl[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP))
        __builtin_amdgcn_s_sleep(2);
    if (__hip_atomic_load(&ctrl[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) timed_out = true;
    if (lane != 0) return;
    if (timed_out) {
        write_result(result, hi, IGGY_ERR_TIMEOUT, 0, 0, 0, 0, 0, 0, 1, kStatusDone, 0);
        return;  // scratch left dirty on purpose: the host re-initialises it
    }
    uint64_t fb_enc = __hip_atomic_load(sc.first_bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tail_bad && fb_enc == 0) fb_enc = ~(pl.N - 1);  // producers only report smaller indices
    const uint64_t sf_enc = __hip_atomic_load(sc.spec_fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool has_fb = fb_enc != 0, has_sf = sf_enc != 0;
    const uint64_t fb = ~fb_enc, sf = ~sf_enc;
    uint32_t kind = IGGY_OK, reason = 0, status = kStatusDone;
    uint64_t a = 0, b = 0, c = 0, nframes = pl.N;
    auto msg_err = [&](uint64_t idx) {
        const uint64_t slot = ((idx + 6) >> 8) * 4 + (((idx + 6) >> 6) & 3);
        kind = IGGY_ERR_INVALID_MESSAGE_CHECKSUM;
        if (tail_bad && idx == pl.N - 1) {
            a = tail_stored;
            b = tail_computed;
        } else {
            a = __hip_atomic_load(&sc.errslot[2 * slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            b = __hip_atomic_load(&sc.errslot[2 * slot + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        c = sat_add(hi.h.base_offset, ld32_any(blob + idx * pl.S + 24));
    };
    if (has_sf) {
        // the true walk reaches frame sf at sf*S (all earlier frames have size S)
        const uint64_t pos = sf * pl.S, bl = hi.blob_len;
        bool stops = (bl - pos < kFrameHdr) || ld64_any(blob + pos + 40) != 0;
        if (!stops) {
            const uint64_t end = pos + kFrameHdr + ld32_any(blob + pos + 36) + ld32_any(blob + pos + 32);
            stops = end > bl;
        }
        nframes = sf;
        if (!stops) status = kStatusNeedGeneral;
        else if (VERIFY && has_fb && fb < sf) msg_err(fb);
        else { kind = IGGY_ERR_VALIDATION; reason = IGGY_V_FRAMES_DO_NOT_TILE; }
    } else if (VERIFY && has_fb) {
        msg_err(fb);
    } else if (pl.N != (uint64_t)hi.h.message_count) {
        kind = IGGY_ERR_VALIDATION; reason = IGGY_V_FRAMES_DO_NOT_TILE;
    } else if (VERIFY && computed != hi.h.batch_checksum) {
        kind = IGGY_ERR_INVALID_BATCH_CHECKSUM;
        a = hi.h.batch_checksum; b = computed; c = hi.h.base_offset;
    }
    write_result(result, hi, kind, reason, a, b, c, nframes, computed, 1, status, nframes * pl.S);
    // re-arm the scratch for the next call on this stream
    __hip_atomic_store(sc.exited, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(sc.first_bad, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(sc.spec_fail, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------- kernel
template <bool VERIFY>
__global__ __launch_bounds__(256, 1) void k_decode_uniform(const uint8_t *__restrict__ body,
                                                           uint64_t len, uint64_t *frame_pos,
                                                           uint64_t cap, iggy_decode_result *result,
                                                           DecodeScratch sc, uint32_t epoch,
                                                           uint32_t allow_unaligned, uint32_t dbg) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const uint32_t nprod = gridDim.x - 1;
    HeaderInfo hi;
    parse_header(body, len, hi);
    UPlan pl;
    make_plan(hi, body + kHdr, len, VERIFY, sc.max_chunks, allow_unaligned != 0, pl);

    if (blockIdx.x == 0) {
        consumer_wg<VERIFY>(body, hi, pl, frame_pos, result, sc, epoch, nprod, smem, dbg);
        return;
    }
    if (pl.state != 0) return;  // nothing for producers; consumer resolves

    const uint8_t *blob = body + kHdr;
    const uint32_t g = blockIdx.x - 1;
    const uint32_t wave_u = (uint32_t)__builtin_amdgcn_readfirstlane(wave);
    const uint32_t buf0 = wave_u * 2 * kWaveBuf;
    uint8_t *side = smem + kSideOff + wave_u * 64 * kSideLane + (uint32_t)lane * kSideLane;
    uint64_t *xchg = (uint64_t *)(smem + kXchgOff);
    uint64_t *red = (uint64_t *)(smem + kRedOff);

    // per-thread constant of the checksum-input word it owns in every chunk
    const uint32_t tid = threadIdx.x;
    const uint64_t cs_sec = kSecretW8[((tid >> 3) & 15) + (tid & 7)];

    uint64_t c = g;
    uint32_t bi = 0;
    bool have_prev = false;
    uint64_t c_prev = 0;
    if (c < pl.nchunks) issue_phase(blob, pl, (int64_t)(256 * c) - 6 + 64 * wave, 0, buf0, lane);

    for (; c < pl.nchunks; c += nprod) {
        const uint64_t cn = c + nprod;
        const int64_t iw0 = (int64_t)(256 * c) - 6 + 64 * wave;
        const int64_t i = iw0 + lane;
        const bool fvalid = i >= 0 && (uint64_t)i < pl.N;
        PhaseState st;
        st.acc.init();
        st.stored = 0;
        st.resv = 0;
        st.uh = 0;
        st.plen = 0;
        for (uint32_t p = 0; p < pl.nph; ++p) {
            const uint32_t nb_ = buf0 + (bi ^ 1) * kWaveBuf;
            bool issued = true;
            if (p + 1 < pl.nph) issue_phase(blob, pl, iw0, p + 1, nb_, lane);
            else if (cn < pl.nchunks) issue_phase(blob, pl, (int64_t)(256 * cn) - 6 + 64 * wave, 0, nb_, lane);
            else issued = false;
            if (issued) wait_vm16(); else wait_vm0();
            if (p == 0) {
                // everything older than the phase just issued has landed in every
                // wave, including the previous chunk's sc1 stores: publish it
                lds_fence_barrier();
                if (have_prev && threadIdx.x == 0)
                    __hip_atomic_store(&sc.flags[c_prev], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (dbg & 2) run_phase<false>(smem + buf0 + bi * kWaveBuf, side, lane, p, pl, st);
            else run_phase<VERIFY>(smem + buf0 + bi * kWaveBuf, side, lane, p, pl, st);
            bi ^= 1;
        }
        // ---- per-frame result
        uint64_t h = 0;
        if (VERIFY) {
            if (pl.long_frames) {
                // last stripe: hashed bytes [L-64, L) = stream [S-64, S) from the side copy
                const uint64_t o = pl.S - 64;
                const uint32_t t = (uint32_t)(o & 7);
                const uint32_t u0 = (uint32_t)(o >> 3) - 2 * pl.q_side0;
                uint64_t U[9];
#pragma unroll
                for (int k = 0; k < 9; ++k) {
                    if (k < 8 || t) U[k] = *(const uint64_t *)(side + 8u * (u0 + k));
                    else U[k] = 0;
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const uint64_t w = funnel64(U[k], U[k + 1], t);
                    switch (k) {
                        case 0: st.acc.word<0>(w, Secret::w(121)); break;
                        case 1: st.acc.word<1>(w, Secret::w(129)); break;
                        case 2: st.acc.word<2>(w, Secret::w(137)); break;
                        case 3: st.acc.word<3>(w, Secret::w(145)); break;
                        case 4: st.acc.word<4>(w, Secret::w(153)); break;
                        case 5: st.acc.word<5>(w, Secret::w(161)); break;
                        case 6: st.acc.word<6>(w, Secret::w(169)); break;
                        default: st.acc.word<7>(w, Secret::w(177)); break;
                    }
                }
                h = st.acc.merge(pl.L);
            } else {
                // single phase; its image is buffer (bi ^ 1) now
                h = short_hash(smem + buf0 + (bi ^ 1) * kWaveBuf, lane, pl.L);
            }
        }
        const uint64_t stored = st.stored;
        const bool spec_bad = fvalid && (st.resv != 0 || (uint64_t)kFrameHdr + st.plen + st.uh != pl.S);
        // the last frame of a record that ends at the buffer end is verified by the
        // consumer from exact-extent reads (its last chunk was not staged)
        const bool mism = VERIFY && fvalid && h != stored &&
                          !(pl.tail_unsafe && (uint64_t)i == pl.N - 1);
        if (frame_pos && fvalid && (uint64_t)i < cap) frame_pos[i] = (uint64_t)i * pl.S;
        const uint64_t mb = __ballot(mism);
        if (mb) {
            const int leader = __builtin_ctzll(mb);
            if (lane == leader) {
                atomicMax((unsigned long long *)sc.first_bad, (unsigned long long)~(uint64_t)i);
                const uint64_t slot = c * 4 + wave;
                __hip_atomic_store(&sc.errslot[2 * slot], stored, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&sc.errslot[2 * slot + 1], h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        const uint64_t sb = __ballot(spec_bad);
        if (sb) {
            const int leader = __builtin_ctzll(sb);
            if (lane == leader) atomicMax((unsigned long long *)sc.spec_fail, (unsigned long long)~(uint64_t)i);
        }
        // ---- batch-checksum words of this chunk: m = 256c + tid (tid < 255)
        if (VERIFY && pl.long_cs) {
            xchg[tid] = stored;
            lds_fence_barrier();
            const uint64_t m = 256 * c + tid;
            uint64_t x = 0, y = 0;  // x -> acc[j], y -> acc[j^1]
            if (tid < 255 && m >= 6 && m < pl.Mreg) {
                const uint64_t v = (stored >> 32) | (xchg[tid + 1] << 32);
                y = v;
                x = mul32x32(v ^ cs_sec);
            }
            // sum lanes with equal (lane & 7): xor 8, 16, 32
            x += __shfl_xor(x, 8); y += __shfl_xor(y, 8);
            x += __shfl_xor(x, 16); y += __shfl_xor(y, 16);
            x += __shfl_xor(x, 32); y += __shfl_xor(y, 32);
            const uint64_t t8 = x + __shfl_xor(y, 1);  // lane t (<8): acc[t] sum
            if (lane < 8) red[wave * 8 + lane] = t8;
            lds_fence_barrier();
            if (wave == 0 && lane < 16) {
                const int half = lane >> 3, t = lane & 7;
                const uint64_t s = red[(2 * half) * 8 + t] + red[(2 * half + 1) * 8 + t];
                __hip_atomic_store(&sc.sums[(2 * c + half) * 8 + t], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        have_prev = true;
        c_prev = c;
    }
    // drain every wave's stores, then publish the last chunk and retire
    wait_vm0();
    lds_fence_barrier();
    if (threadIdx.x == 0) {
        if (have_prev)
            __hip_atomic_store(&sc.flags[c_prev], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(sc.exited, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template __global__ void k_decode_uniform<true>(const uint8_t *__restrict__, uint64_t, uint64_t *,
                                                uint64_t, iggy_decode_result *, DecodeScratch,
                                                uint32_t, uint32_t, uint32_t);
template __global__ void k_decode_uniform<false>(const uint8_t *__restrict__, uint64_t, uint64_t *,
                                                 uint64_t, iggy_decode_result *, DecodeScratch,
                                                 uint32_t, uint32_t, uint32_t);

}  // namespace iggy

// decode_records.hip — decode_batch_slice_with (core/binary_protocol/src/batch.rs:391-506)
// over MANY records in ONE launch: the walks that visit a sequence of batches (a
// 1 MiB disk-poll chunk, poll_plan.rs:484/950-1011; boot recovery of a segment,
// segment_recovery.rs:425-530; a transferred segment, state_transfer.rs:715-833;
// a poll response body, poll_messages.rs:95-165 / polled_messages.rs:95-150)
// mostly carry C1-sized batches (1 000 x 256 B = 304 KB, core/bench
// defaults.rs:33). The persistent single-record decode (decode_uniform.hip) sizes a
// whole-chip grid per record; here every record's 128-frame checksum blocks are
// workgroups of ONE grid, so a chunk or a segment of small batches fills the chip
// with one dispatch.
//
// Per record (uniform stride S taken from frame 0, as decode_uniform.hip
// speculates and proves): WG (record, b) checks and hashes frames
// [128b - 6, 128b + 122) -- exactly the frames whose stored checksums form words
// 128b .. 128b + 127 of the batch-checksum input -- and stores that block's 8
// XXH3 accumulator sums. 8 lanes per frame (lane-group XXH3, 16-B pieces, pairs
// folded by DPP) for hashed lengths > 240 B; one lane per frame otherwise and
// under LayoutOnly. The LAST workgroup of a record to finish (a per-record
// counter; the block sums handed over as sc1 stores and loads) runs the record's
// serial scramble chain over its block sums and resolves precedence exactly as the
// uniform kernel's consumer does. A record whose stride speculation breaks without the walk stopping is
// left with status kStatusNeedGeneral; the host re-decodes it with the general
// walk (decode_general.hip).
//
// Optional fused outputs (both written speculatively by the block workgroups,
// valid when the record decodes):
//  * frame positions at frame_pos[pos_base + i];
//  * polled message descriptors (poll.hip's k_poll_fill) at msgs[msg_base + i].
#include "codec_common.hpp"

namespace iggy {

struct RecTask {
    uint64_t off, len;            // record start in the device buffer, bytes available from there
    uint64_t pos_base, pos_cap;   // frame positions: frame_pos[pos_base + i], i < pos_cap
    uint64_t msg_base;            // polled messages: msgs[msg_base + i] (when msgs != nullptr)
    uint64_t bsum_base;           // block sums of this record: bsums[8 * (bsum_base + b) + j]
    uint32_t wg0, nwg;            // its workgroups in the grid
};
// The general kernel's barrier / registration words (DecodeScratch gbar, gbar2, gmisc),
// re-armed by a launch that runs in the uniform kernel's place before a k_decode_general
// (the asynchronous single-stride decode); all null otherwise.
struct GenRearm {
    uint32_t *gbar, *gbar2;
    uint64_t *gmisc;
};

// k_decode_general's barrier words re-armed on their own (before a general walk that no
// uniform or records launch directly precedes)
__global__ void k_general_rearm(GenRearm rearm) {
    if (threadIdx.x == 0) {
        __hip_atomic_store(&rearm.gbar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&rearm.gbar[2], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&rearm.gbar[3], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&rearm.gmisc[2], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&rearm.gmisc[kPosCountWord], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x < kBar2Words)
        __hip_atomic_store(&rearm.gbar2[32 * threadIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

typedef uint32_t rec_g2 __attribute__((ext_vector_type(2)));

struct RecState {  // zero between launches: zeroed when allocated, reset by the record's resolver
    uint64_t first_bad;  // ~min index of a frame whose checksum mismatches (max-encoded), 0 = none
    uint64_t spec_fail;  // ~min index of a frame that breaks the stride
    uint32_t done;       // block workgroups finished
    uint32_t _pad;
};

constexpr uint32_t kRecThreads = 256;
constexpr uint32_t kRecFrames = 128;  // frames per workgroup: one checksum block

__host__ __device__ __forceinline__ uint64_t rec_blocks(uint64_t N) { return (N + 5) / kRecFrames + 1; }

__device__ __forceinline__ void rec_fill_msg(const uint8_t *rec, uint64_t rec_off, uint64_t p, uint64_t base_offset,
                                             uint64_t base_ts, uint64_t origin, iggy_polled_message *out) {
    const uint8_t *f = rec + kHdr + p;
    iggy_polled_message m;
    m.checksum = ld64_any(f);
    m.id_lo = ld64_any(f + 8);
    m.id_hi = ld64_any(f + 16);
    m.offset = base_offset + ld32_any(f + 24);  // wrapping, as in release Rust
    m.timestamp = base_ts;                      // flat per batch
    m.origin_timestamp = origin + ld32_any(f + 28);
    m.user_headers_length = ld32_any(f + 32);
    m.payload_length = ld32_any(f + 36);
    m.payload_pos = rec_off + kHdr + p + kFrameHdr;
    m.user_headers_pos = m.payload_pos + m.payload_length;
    m._pad = 0;
    *out = m;
}

// lane l's 64-bit value, wave-uniform (v_readlane)
__device__ __forceinline__ uint64_t rdlane64(uint64_t v, int l) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32);
}

// minima over the WG of two per-thread candidates (~0 = none), via wave minima in LDS
// (s8: 2 per wave). A wave without a candidate (a clean block: every wave) skips its
// shuffle ladder, six dependent 64-bit shuffles of ~0.3 us each pair; the two ladders of
// a wave that has one run interleaved, and the two minima share one pair of barriers.
__device__ __forceinline__ void wg_min2(uint64_t &v1, uint64_t &v2, uint64_t *s8) {
    if (__ballot(v1 != ~0ull || v2 != ~0ull)) {
        for (int d = 32; d; d >>= 1) {
            const uint64_t o1 = __shfl_xor(v1, d), o2 = __shfl_xor(v2, d);
            v1 = o1 < v1 ? o1 : v1;
            v2 = o2 < v2 ? o2 : v2;
        }
    }
    if ((threadIdx.x & 63) == 0) {
        s8[2 * (threadIdx.x >> 6)] = v1;
        s8[2 * (threadIdx.x >> 6) + 1] = v2;
    }
    __syncthreads();
    uint64_t m1 = s8[0], m2 = s8[1];
#pragma unroll
    for (int w = 1; w < (int)(kRecThreads / 64); ++w) {
        m1 = s8[2 * w] < m1 ? s8[2 * w] : m1;
        m2 = s8[2 * w + 1] < m2 ? s8[2 * w + 1] : m2;
    }
    __syncthreads();
    v1 = m1;
    v2 = m2;
}

// Launch completion for host callers that spin instead of synchronising the stream:
// every workgroup arrives on a device counter once its writes are fenced at system
// scope; the last one re-arms the counter and stores `value` into the host-mapped
// flag (a plain launch boundary would otherwise need a stream sync, ~3 us more, or
// a D2H copy of the results, ~5 us more; scripts/latency_micro.cpp).
__device__ __forceinline__ void launch_done(uint32_t *counter, uint32_t *host_flag, uint32_t value) {
    if (!host_flag) return;
#ifndef IGGY_REC_K1
    __threadfence_system();  // every wave: its own host-visible writes (a fence orders only its wave's)
#endif
    __syncthreads();
    if (threadIdx.x == 0) {
        if (atomicAdd(counter, 1u) == gridDim.x - 1) {
            __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifndef IGGY_REC_K2
            __threadfence_system();
            __hip_atomic_store(host_flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
#else
            __hip_atomic_store(host_flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#endif
        }
    }
}

// The resident service's block hand-off (k_decode_service; units == nullptr elsewhere):
// block b > 0 of the post stores its record -- 8 partial sums and the low words of its
// first-bad and stride-fail encodings, 18 dwords -- as 9 16-B units of two 8-B granules
// {the post's number, one dword} each, and block 0 resolves once one load round has seen
// the number in every granule. Each 8-B half of a 16-B sc1 store is observed untorn,
// the whole 16 B is not (MI355X_MICROARCH.md: granules): a unit {number, 12 B} let a
// load see the new number beside a stale second half -- the previous post's first-bad
// word, a corrupt frame passed as clean. No counter, no sum buffer read after it: one
// host-visible round trip fewer on a small record's path.
constexpr uint32_t kSvcRecUnits = 9;
constexpr uint32_t kSvcWgs_ = 8;  // (k_decode_service's kSvcWgs)
struct SvcHand {
    uint4 *units;  // [(block - 1) * kSvcRecUnits + u] (device memory, sc1)
    uint32_t seq;
    uint64_t *bdiag = nullptr;  // (diagnostic build) [2 b]: block b's entry / hashed clocks
};

template <bool VERIFY>
__device__ __forceinline__ void decode_record_block(const RecTask &inl, const uint8_t *__restrict__ base,
                                                    const RecTask *__restrict__ tasks,
                                                    const uint32_t *__restrict__ wg_task, RecState *st,
                                                    uint64_t *bsums, uint64_t *frame_pos, iggy_polled_message *msgs,
                                                    iggy_decode_result *results, uint32_t vblock = ~0u,
                                                    const uint8_t *pre_head = nullptr, uint64_t *stamp = nullptr,
                                                    SvcHand hand = SvcHand{nullptr, 0}) {
    // (diagnostic build: stage times of thread 0 into stamp[k], the service's LDS)
    auto mark = [&](int k) {
        if (kDiagMask && stamp && threadIdx.x == 0) stamp[k] = rt_now();
    };
    mark(1);
    __shared__ uint64_t s_cs[kRecFrames + 2];  // stored checksums of frames 128b - 6 + k
    __shared__ uint64_t s_min[2 * (kRecThreads / 64)];
    __shared__ uint32_t s_last;
    __shared__ uint8_t s_small[256];  // short checksum inputs (N <= 24): 44 + 8 N bytes
    // one record: its task comes in the kernel arguments (tasks == nullptr), not from a
    // table in host-mapped memory (two dependent PCIe reads before anything else)
    // vblock: the workgroup's block when a resident service workgroup runs it (k_decode_service)
    const uint32_t wg = vblock != ~0u ? vblock : blockIdx.x;
    const uint32_t t = tasks ? wg_task[wg] : 0u;
    const RecTask tk = tasks ? tasks[t] : inl;
    const uint32_t blk = wg - tk.wg0;
    const uint8_t *body = base + tk.off;
    const uint8_t *blob = body + kHdr;
    const int lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    // the batch header and the first frame header (304 B) staged in LDS with one load
    // round, so the header parse and the plan cost no further memory round trips (each
    // one is microseconds for a registered record read in place over the host link)
    // (pre_head: the same 304 B already in LDS, the resident service's relay)
    __shared__ __attribute__((aligned(16))) uint8_t s_head[kHdr + kFrameHdr];
    const bool staged = tk.len >= kHdr + kFrameHdr;
    if (staged && !pre_head) {
        if (threadIdx.x < (kHdr + kFrameHdr) / 16)
            *(uint4 *)(s_head + 16 * threadIdx.x) = ld128_any(body + 16 * threadIdx.x);
        __syncthreads();
    }
    const uint8_t *head = pre_head ? pre_head : s_head;
    HeaderInfo hi;
    parse_header(staged ? head : body, tk.len, hi);
    UPlan pl;
    make_plan(hi, staged ? head + kHdr : blob, tk.len, VERIFY, ~0ull, true, pl);
    iggy_decode_result *res = results + t;

    if (pl.state != 0 || tk.nwg < rec_blocks(pl.N)) {
        // result known without the frames (header errors, empty record, broken first
        // frame), or not a single-stride record: the general walk (host re-decodes)
        if (blk != 0 || wave != 0) return;
        uint32_t kind = pl.ekind, reason = pl.ereason, status = kStatusDone;
        uint64_t a = pl.ea, b = pl.eb, c = pl.ec, computed = 0;
        if (pl.state != 1) {
            status = kStatusNeedGeneral;
        } else if (kind == IGGY_OK && VERIFY && lane == 0) {
            // zero frames: the checksum over the 44 header bytes (batch.rs:452-458)
            const uint64_t w[5] = {hi.h.partition_id, hi.h.base_offset, hi.h.base_timestamp,
                                   hi.h.origin_timestamp, hi.h.batch_length};
            for (int i = 0; i < 5; ++i) st64_any(s_small + 8 * i, w[i]);
            *(u32_ua *)(s_small + 40) = hi.h.message_count;
            computed = xxh3_64_lane(s_small, 44);
            if (computed != hi.h.batch_checksum) {
                kind = IGGY_ERR_INVALID_BATCH_CHECKSUM; reason = 0;
                a = hi.h.batch_checksum; b = computed; c = hi.h.base_offset;
            }
        }
        if (lane == 0) write_result(res, hi, kind, reason, a, b, c, 0, computed, 1, status, 0);
        return;
    }
    const uint64_t S = pl.S, N = pl.N, L = pl.L;
    const uint64_t nblk = rec_blocks(N);
    if (blk >= nblk) return;
    const int64_t i0v = (int64_t)kRecFrames * blk - 6;
    auto store_positions = [&]() {
        if (!frame_pos) return;
        for (uint32_t k = threadIdx.x; k < kRecFrames; k += kRecThreads) {
            const int64_t i = i0v + k;
            if (i >= 0 && (uint64_t)i < pl.N && (uint64_t)i < tk.pos_cap) frame_pos[tk.pos_base + i] = (uint64_t)i * pl.S;
        }
    };
    // (service: the positions go out before the frame loads; their host-link acks are
    // long in by the time the block fences them before handing over its record)
    if (hand.units) store_positions();
    // the resolver's per-lane constants, loaded now rather than on its critical path
    const uint64_t rc_init = kAccInit[lane & 7], rc_key = kSecretW8[16 + (lane & 7)], rc_last = kSecretLast[lane & 7];
    // and the block's partial sums' (wave 0, after the hashes: a constant-table load there
    // waited out a cache miss behind the frames' stream)
    const uint64_t ps_key0 = kSecretW8[(lane >> 3) + (lane & 7)], ps_key1 = kSecretW8[8 + (lane >> 3) + (lane & 7)];
    const int64_t i0 = (int64_t)kRecFrames * blk - 6;
    const uint64_t base_offset = hi.h.base_offset, base_ts = hi.h.base_timestamp, origin = hi.h.origin_timestamp;
    uint64_t mybad = ~0ull, mysf = ~0ull;
    // frame 128b + 122's stored checksum (its low half closes word 128b + 127), loaded
    // beside the frames
    uint64_t cs_next = 0;
    if (threadIdx.x == 0) {
        const int64_t i = i0 + kRecFrames;
        if (i >= 0 && (uint64_t)i < N) cs_next = ld64_any(blob + (uint64_t)i * S);
    }
    // the resolver's inputs from the record (frame 0's stored checksum, the last eight
    // frames' ones: lane j of wave 0), loaded now by every workgroup so the one that
    // resolves does not wait for them afterwards
    uint64_t r_cs0 = 0, r_lv = 0;
    if (VERIFY && pl.long_cs && threadIdx.x < 8) {
        r_cs0 = ld64_any(blob);
        r_lv = ld64_any(blob + (N - 8 + threadIdx.x) * S);
    }

    if (VERIFY && pl.long_frames) {
        // lane groups: group g = 8 wave + (lane >> 3) takes frames i0 + g + 32 k, k = 0..3
        const uint32_t l = lane & 7, m = l >> 1, par = l & 1, g = 8 * wave + ((uint32_t)lane >> 3);
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
        const uint64_t nbF = pl.nbF, ns = pl.ns;
        // one frame's hash from its loaded pieces (the last, partial block and the last
        // stripe), the header checks and the outputs
        // (QT: the pieces pc holds, 2 or 8; a frame needs piece q when 2 q + par < ns)
        auto finish = [&](auto QT, uint32_t k, int64_t i, bool valid, uint4 hdr, uint64_t stored, uint64_t a0,
                          uint64_t a1, const uint4 *pc, uint4 lastp) {
            constexpr int Q = decltype(QT)::value;
#pragma unroll
            for (int q = 0; q < Q; ++q)
                if (2 * (uint64_t)q + par < ns) piece(a0, a1, pc[q], s0[q], s1[q]);
            a0 += gdpp64<0xB1>(a0);
            a1 += gdpp64<0xB1>(a1);
            piece(a0, a1, lastp, last0, last1);  // odd lanes: never used
            uint64_t tt = fold64(a0 ^ mrg0, a1 ^ mrg1);
            tt += gdpp64<0x4E>(tt);
            tt += gswz_xor4(tt);
            const uint64_t h = avalanche(L * P64_1 + tt);
            if (l == 0) {
                if (valid) {
                    if (hdr.z | hdr.w || (uint64_t)kFrameHdr + hdr.x + hdr.y != S) mysf = min(mysf, (uint64_t)i);
                    if (h != stored) mybad = min(mybad, (uint64_t)i);
                }
                s_cs[g + 32 * k] = valid ? stored : 0;
            }
        };
        if (nbF == 0) {
            // frames of at most one block (C1: 296 B): the four frames' loads first, then
            // the hashes -- one memory round trip instead of four (a registered record
            // is read in place over the host link, where each round trip is microseconds)
            constexpr uint32_t K = kRecFrames / 32;
            // Buffer loads over the block's own frames, a piece a lane does not need given an
            // offset past the range (the load returns zeros and fetches nothing: a small
            // record read in place does not fetch frame 0 again over the host link for every
            // slot past its end). No branch around any load, and frames of at most 4 stripes
            // (C1's 296 B) hold 2 pieces a lane, not 8, so the loads land in VGPRs: the
            // compiler then waits for each frame's own pieces (vmcnt(n)) and frame k's hash
            // runs while frames k + 1.. are still on the way. Loads behind branches had been
            // waited for all at once before the first hash.
            const int64_t f0 = i0 < 0 ? 0 : i0;
            const int64_t f1 = min<int64_t>(i0 + (int64_t)kRecFrames, (int64_t)N);
            const __amdgpu_buffer_rsrc_t frs = __builtin_amdgcn_make_buffer_rsrc(
                (void *)(blob + (uint64_t)f0 * S), 0, (int)((uint64_t)(f1 - f0) * S), 0x00020000);
            constexpr uint32_t kOff = 0x80000000u;  // (past any block's range)
            auto frames = [&](auto QT) {
                constexpr int Q = decltype(QT)::value;
                uint4 hdr[K], pc[K][Q], lastp[K];
                uint64_t stored[K];
#pragma unroll
                for (uint32_t k = 0; k < K; ++k) {
                    const int64_t i = i0 + g + 32 * k;
                    const bool valid = i >= 0 && (uint64_t)i < N;
                    const uint32_t fo = valid ? (uint32_t)((uint64_t)(i - f0) * S) : kOff;
                    const uint32_t ho = fo + 8 + poff;
                    const g4 h4 = __builtin_amdgcn_raw_buffer_load_b128(frs, l == 0 ? fo + 32 : kOff, 0, 0);
                    hdr[k] = make_uint4(h4.x, h4.y, h4.z, h4.w);
                    const rec_g2 s2 = __builtin_amdgcn_raw_buffer_load_b64(frs, l == 0 ? fo : kOff, 0, 0);
                    stored[k] = (uint64_t)s2.x | ((uint64_t)s2.y << 32);
#pragma unroll
                    for (int q = 0; q < Q; ++q) {
                        const g4 p4 = __builtin_amdgcn_raw_buffer_load_b128(
                            frs, (2 * (uint64_t)q + par < ns) ? ho + 128 * q : kOff, 0, 0);
                        pc[k][q] = make_uint4(p4.x, p4.y, p4.z, p4.w);
                    }
                    const g4 l4 = __builtin_amdgcn_raw_buffer_load_b128(
                        frs, !par ? fo + 8 + (uint32_t)L - 64 + 16 * m : kOff, 0, 0);
                    lastp[k] = make_uint4(l4.x, l4.y, l4.z, l4.w);
                }
#pragma unroll
                for (uint32_t k = 0; k < K; ++k) {
                    const int64_t i = i0 + g + 32 * k;
                    finish(QT, k, i, i >= 0 && (uint64_t)i < N, hdr[k], stored[k], init0, init1, pc[k], lastp[k]);
                }
            };
            if (ns <= 4)
                frames(std::integral_constant<int, 2>{});
            else
                frames(std::integral_constant<int, 8>{});
        } else
#pragma unroll 1
        for (uint32_t k = 0; k < kRecFrames / 32; ++k) {
            const int64_t i = i0 + g + 32 * k;
            const bool valid = i >= 0 && (uint64_t)i < N;
            const uint8_t *fb = blob + (valid ? (uint64_t)i : 0) * S;
            const uint8_t *hb = fb + 8 + poff;
            uint4 hdr = make_uint4(0, 0, 0, 0);
            uint64_t stored = 0;
            if (valid && l == 0) {
                hdr = ld128_any(fb + 32);  // user_headers_length, payload_length, reserved
                stored = ld64_any(fb);
            }
            uint64_t a0 = init0, a1 = init1;
            for (uint64_t b = 0; b < (valid ? nbF : 0); ++b) {
                uint4 pc[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) pc[q] = ld128_any(hb + 1024 * b + 128 * q);
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
            }
            uint4 pc[8];
#pragma unroll
            for (int q = 0; q < 8; ++q)
                pc[q] = valid && (2 * (uint64_t)q + par < ns) ? ld128_any(hb + 1024 * nbF + 128 * q)
                                                              : make_uint4(0, 0, 0, 0);
            const uint4 lastp = valid && !par ? ld128_any(fb + 8 + L - 64 + 16 * m) : make_uint4(0, 0, 0, 0);
            finish(std::integral_constant<int, 8>{}, k, i, valid, hdr, stored, a0, a1, pc, lastp);
        }
    } else if (threadIdx.x < kRecFrames) {
        // one lane per frame: header checks, short-frame hashes (<= 240 B), positions
        const uint32_t k = threadIdx.x;
        const int64_t i = i0 + k;
        const bool valid = i >= 0 && (uint64_t)i < N;
        uint64_t stored = 0;
        if (valid) {
            const uint8_t *fb = blob + (uint64_t)i * S;
            const uint4 hdr = ld128_any(fb + 32);
            stored = ld64_any(fb);
            if (hdr.z | hdr.w || (uint64_t)kFrameHdr + hdr.x + hdr.y != S) mysf = (uint64_t)i;
            if (VERIFY && xxh3_64_lane(fb + 8, L) != stored) mybad = (uint64_t)i;
        }
        s_cs[k] = stored;
    }
    if (msgs) {  // poll-side descriptors (poll.hip), written whether or not the record decodes
        for (uint32_t k = threadIdx.x; k < kRecFrames; k += kRecThreads) {
            const int64_t i = i0 + k;
            if (i >= 0 && (uint64_t)i < N)
                rec_fill_msg(body, tk.off, (uint64_t)i * S, base_offset, base_ts, origin, msgs + tk.msg_base + i);
        }
    }
    if (threadIdx.x == 0) s_cs[kRecFrames] = cs_next;
    // the resolver's inputs from the record have landed by now (without this use the
    // compiler sank their loads to the resolver, one host-link round trip on its path)
    asm volatile("" ::"v"(r_cs0), "v"(r_lv));
    mark(2);  // (thread 0's own frames hashed)
    uint64_t wbad = mybad, wsf = mysf;
    wg_min2(wbad, wsf, s_min);  // (its barriers also publish s_cs)
    if (threadIdx.x == 0 && nblk > 1 && !hand.units) {  // (a one-block record's own minima are final)
        if (wbad != ~0ull) atomicMax((unsigned long long *)&st[t].first_bad, (unsigned long long)~wbad);
        if (wsf != ~0ull) atomicMax((unsigned long long *)&st[t].spec_fail, (unsigned long long)~wsf);
    }
    uint64_t t8 = 0;  // (wave 0 lane j < 8: this block's partial sum j)
    if (VERIFY && pl.long_cs && wave == 0) {
        // words m = 128b + j of the checksum input, j = lane, lane + 64
        const uint64_t mb = (uint64_t)kRecFrames * blk;
        uint64_t x = 0, y = 0;
        word_contrib_s(pl.Mreg, mb + lane, s_cs[lane], s_cs[lane + 1], true, ps_key0, x, y);
        word_contrib_s(pl.Mreg, mb + 64 + lane, s_cs[64 + lane], s_cs[65 + lane], true, ps_key1, x, y);
        t8 = reduce_acc8(x, y);
        // (sc1: written through, for the resolver's sc1 loads on another CU)
        if (lane < 8 && nblk > 1 && !hand.units)
            __hip_atomic_store(&bsums[8 * (tk.bsum_base + blk) + lane], t8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // The last block workgroup of the record resolves it (a one-block record: its only
    // workgroup, with no counter). The hand-off needs no fence (round 6): the block sums
    // are sc1 stores of wave 0 and the minima are atomics of its lane 0, which waits for
    // all of them (vmcnt) before its counter add; the resolver is the wave whose add came
    // last and reads them with sc1 loads after its add has returned
    // (MI355X_MICROARCH.md, hand-off table, first row). A __threadfence() on each side
    // (an L2 write-back and an L1 invalidate, microseconds each) was on every small
    // record's critical path.
    __syncthreads();
    // Frame positions (i * S; valid when the record decodes) are stored after the
    // counter add: ahead of it, a store to host-mapped positions would put a host-link
    // round trip into the wait before it. (The service's blocks store them first of all,
    // see store_positions' definition.)
    // (service) every block's record, block 0 first: [8 sums, first-bad, stride-fail]
    __shared__ uint64_t s_recs[kSvcWgs_ * 10];
    bool svc_ok = true;
    if (hand.units && nblk > 1) {
        // (blocks > 0, every wave, when the post asked for positions in host memory: they
        // are host-visible before the block's units go out; block 0's are ordered before
        // the flag by its completion fence. A vmcnt wait alone was measured not to be
        // enough: positions of other blocks read back as zeros after the flag. The host's
        // own posts ask for none, see svc_post_wait.)
        if (blk != 0 && frame_pos) __threadfence_system();
        if (wave == 0) {
            uint64_t *mine = s_recs + 10 * (blk == 0 ? 0 : 1);  // (a block > 0 stages its own record in slot 1)
            if (lane < 8) mine[lane] = t8;
            if (lane == 8) mine[8] = wbad != ~0ull ? ~wbad : 0ull;
            if (lane == 9) mine[9] = wsf != ~0ull ? ~wsf : 0ull;
        }
        __syncthreads();
        if (blk != 0) {
            if (kDiagMask && stamp && hand.bdiag && threadIdx.x == 0) {  // (diagnostic build)
                __hip_atomic_store(&hand.bdiag[2 * blk], stamp[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&hand.bdiag[2 * blk + 1], stamp[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (wave == 0 && lane < (int)kSvcRecUnits) {  // (LDS reads: dwords 2 lane, 2 lane + 1)
                const uint32_t *r32 = (const uint32_t *)(s_recs + 10);
                // (unit 8: the low words of the first-bad and stride-fail encodings; a frame
                // index < 2^32 leaves their high words all ones, and none encodes as 0)
                const uint32_t d0 = lane < 8 ? r32[2 * lane] : r32[16], d1 = lane < 8 ? r32[2 * lane + 1] : r32[18];
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                    (void *)hand.units, 0, (int)(16 * kSvcRecUnits * (kSvcWgs_ - 1)), 0x00020000);
                const g4 w = {hand.seq, d0, hand.seq, d1};
                __builtin_amdgcn_raw_buffer_store_b128(w, rs, 16u * (kSvcRecUnits * (blk - 1) + (uint32_t)lane), 0,
                                                       kAuxSc1);
            }
            return;
        }
        if (wave != 0) return;
        // block 0 resolves: one sc1 load round per poll over every other block's units
        const uint32_t nu = kSvcRecUnits * (uint32_t)(nblk - 1);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)hand.units, 0, (int)(16 * kSvcRecUnits * (kSvcWgs_ - 1)), 0x00020000);
        const uint64_t tw = rt_now();
        for (;;) {
            const g4 v = (uint32_t)lane < nu ? __builtin_amdgcn_raw_buffer_load_b128(rs, 16u * (uint32_t)lane, 0, kAuxSc1)
                                             : g4{hand.seq, 0, hand.seq, 0};
            if (__ballot(v.x != hand.seq || v.z != hand.seq) == 0) {
                if ((uint32_t)lane < nu) {  // unit u of block b + 1 into slot b + 1
                    const uint32_t b = (uint32_t)lane / kSvcRecUnits, u = (uint32_t)lane % kSvcRecUnits;
                    uint64_t *slot = s_recs + 10 * (b + 1);
                    if (u < 8) {
                        slot[u] = (uint64_t)v.y | ((uint64_t)v.w << 32);
                    } else {
                        slot[8] = v.y ? (0xFFFFFFFF00000000ull | v.y) : 0ull;
                        slot[9] = v.w ? (0xFFFFFFFF00000000ull | v.w) : 0ull;
                    }
                }
                break;
            }
            if (rt_now() - tw > kSpinLimitTicks) {  // (bug guard: a block never arrived)
                svc_ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_s_waitcnt(0);  // (the slots' LDS writes, before the chain reads them)
    } else if (nblk > 1) {
        if (threadIdx.x == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // wave 0's block sums and minima
            const uint32_t old = __hip_atomic_fetch_add(&st[t].done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_last = old + 1 == (uint32_t)nblk;
        }
        store_positions();
        __syncthreads();
        if (!s_last || wave != 0) return;
    } else {
        if (!hand.units) store_positions();  // (the service's went out first)
        if (wave != 0) return;
    }

    // the record's first-bad / stride-fail words: final now, loaded beside the chain's
    // block sums (one memory round trip, not two)
    mark(3);
    // (one block: this workgroup's own minima and partial sums, no memory round trip)
    uint64_t fb_enc = 0, sf_enc = 0;
    if (hand.units && nblk > 1) {  // (service) the blocks' records, max-encoded minima
        // (lane b reads block b's pair, one LDS round; then v_readlane, not one LDS round
        // trip per block)
        const uint64_t f = (uint64_t)lane < nblk ? s_recs[10 * lane + 8] : 0ull;
        const uint64_t g = (uint64_t)lane < nblk ? s_recs[10 * lane + 9] : 0ull;
        for (uint32_t b = 0; b < (uint32_t)nblk; ++b) {
            fb_enc = max(fb_enc, rdlane64(f, (int)b));
            sf_enc = max(sf_enc, rdlane64(g, (int)b));
        }
    } else {
        fb_enc = nblk > 1 ? __hip_atomic_load(&st[t].first_bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                          : (wbad != ~0ull ? ~wbad : 0ull);
        sf_enc = nblk > 1 ? __hip_atomic_load(&st[t].spec_fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                          : (wsf != ~0ull ? ~wsf : 0ull);
    }
    uint64_t computed = 0;
    if (VERIFY && pl.long_cs) {
        const int j = lane & 7;
        uint64_t acc = rc_init;
        const uint64_t key = rc_key;
        const uint32_t klo = (uint32_t)key, khi = (uint32_t)(key >> 32);
        {  // words 0..5: header fields, then count | lo32(cs_0)
            const uint64_t cs0 = rdlane64(r_cs0, 0);
            const uint64_t w6[6] = {hi.h.partition_id, hi.h.base_offset, hi.h.base_timestamp,
                                    hi.h.origin_timestamp, hi.h.batch_length,
                                    (uint64_t)hi.h.message_count | (cs0 << 32)};
#pragma unroll
            for (int mm = 0; mm < 6; ++mm) {
                if (j == (mm ^ 1)) acc += w6[mm];
                if (j == mm) acc += mul32x32(w6[mm] ^ Secret::w(8 * mm));
            }
        }
        // y = acc + S_0; y = scramble(y) + S_b for b = 1 .. nb (the partial block nb only adds)
        // (the block sums of other workgroups: sc1 loads, see the hand-off above)
        // (buffer loads with the sc1 policy: schedulable, so a group of 16 is one round)
        const uint64_t nb = pl.nb;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(bsums + 8 * tk.bsum_base), 0, (int)min<uint64_t>(64 * (nb + 1), 1u << 30), 0x00020000);
        const bool from_lds = hand.units != nullptr;  // (service: the records the poll staged)
        auto sum_at = [&](uint64_t b) -> uint64_t {  // (lane j: sum j of block b)
            if (from_lds) return s_recs[10 * b + j];
            const rec_g2 r = __builtin_amdgcn_raw_buffer_load_b64(rs, (uint32_t)(64 * b + 8 * j), 0, kAuxSc1);
            return (uint64_t)r.x | ((uint64_t)r.y << 32);
        };
        uint64_t y = acc + (nblk > 1 ? sum_at(0) : t8);  // (one block: pl.nb == 0; lane j < 8 holds sum j)
        uint64_t b = 1;
        uint64_t v[16];
        for (; b <= nb; b += 16) {  // groups of up to 16 blocks: the group's loads, then its steps
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = b + q <= nb ? sum_at(b + q) : 0;
#pragma unroll
            for (int q = 0; q < 16; ++q)
                if (b + q <= nb) y = chain_step(y, v[q], klo, khi);
        }
        acc = y;
#ifdef IGGY_DIAG_CHAIN
        mark(5);  // (diagnostic bisect build, -DIGGY_DIAG_CHAIN: the chain done, not the result written)
#endif
        // last stripe = stored checksums of frames N-8 .. N-1 (secret offset 121)
        const uint64_t lv = r_lv;  // (lane j < 8 loaded frame N - 8 + j's; only lanes 0..7 carry on)
        acc += gdpp64<0xB1>(lv);   // (lane j ^ 1's)
        acc += mul32x32(lv ^ rc_last);
        uint64_t a[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = rdlane64(acc, i);  // (v_readlane: no LDS round trip)
        uint64_t r = pl.n * P64_1;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            r += fold64(a[2 * i] ^ Secret::w(11 + 16 * i), a[2 * i + 1] ^ Secret::w(19 + 16 * i));
        computed = avalanche(r);
    } else if (VERIFY && lane == 0) {
        // short checksum input (N <= 24): hash it directly
        const uint64_t w[5] = {hi.h.partition_id, hi.h.base_offset, hi.h.base_timestamp, hi.h.origin_timestamp,
                               hi.h.batch_length};
        for (int i = 0; i < 5; ++i) st64_any(s_small + 8 * i, w[i]);
        *(u32_ua *)(s_small + 40) = hi.h.message_count;
        // (the stored checksums are in s_cs already: frame i at s_cs[i + 6] of the one block)
        for (uint64_t i = 0; i < N; ++i) st64_any(s_small + 44 + 8 * i, s_cs[i + 6]);
        computed = xxh3_64_lane(s_small, pl.n);
    }
    if (lane != 0) return;
    mark(4);
    // precedence, as the uniform kernel's consumer (batch.rs:395-421, 461-506)
    // every block workgroup of the record has arrived: re-arm its state for the next launch
    if (nblk > 1 && !hand.units) {
        __hip_atomic_store(&st[t].first_bad, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&st[t].spec_fail, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&st[t].done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const bool has_fb = fb_enc != 0, has_sf = sf_enc != 0;
    const uint64_t fbi = ~fb_enc, sf = ~sf_enc;
    uint32_t kind = IGGY_OK, reason = 0, status = kStatusDone;
    uint64_t a = 0, b = 0, c = 0, nframes = N;
    auto msg_err = [&](uint64_t idx) {
        const uint8_t *f = blob + idx * S;
        kind = IGGY_ERR_INVALID_MESSAGE_CHECKSUM;
        a = ld64_any(f);
        b = xxh3_64_lane(f + 8, L);
        c = sat_add(hi.h.base_offset, ld32_any(f + 24));
    };
    if (has_sf) {
        // the true walk reaches frame sf at sf*S (all earlier frames have size S)
        const uint64_t pos = sf * S, bl = hi.blob_len;
        bool stops = (bl - pos < kFrameHdr) || ld64_any(blob + pos + 40) != 0;
        if (!stops) {
            const uint64_t end = pos + kFrameHdr + ld32_any(blob + pos + 36) + ld32_any(blob + pos + 32);
            stops = end > bl;
        }
        nframes = sf;
        if (!stops) status = kStatusNeedGeneral;
        else if (VERIFY && has_fb && fbi < sf) msg_err(fbi);
        else { kind = IGGY_ERR_VALIDATION; reason = IGGY_V_FRAMES_DO_NOT_TILE; }
    } else if (VERIFY && has_fb) {
        msg_err(fbi);
    } else if (N != (uint64_t)hi.h.message_count) {
        kind = IGGY_ERR_VALIDATION; reason = IGGY_V_FRAMES_DO_NOT_TILE;
    } else if (VERIFY && computed != hi.h.batch_checksum) {
        kind = IGGY_ERR_INVALID_BATCH_CHECKSUM;
        a = hi.h.batch_checksum; b = computed; c = hi.h.base_offset;
    }
    if (!svc_ok) {  // (service: a block's record never arrived -- the bug guard)
        kind = IGGY_ERR_TIMEOUT; reason = 0; a = b = c = 0; status = kStatusDone;
    }
    write_result(res, hi, kind, reason, a, b, c, nframes, computed, 1, status, nframes * S);
#ifndef IGGY_DIAG_CHAIN
    mark(5);
#endif
}

// tasks / wg_task may live in host-mapped pinned memory (read once per workgroup);
// results and frame_pos may too (plain stores); st, bsums and counter are device memory.
template <bool VERIFY>
__global__ __launch_bounds__(kRecThreads) void k_decode_records(const uint8_t *__restrict__ base,
                                                                const RecTask *__restrict__ tasks,
                                                                const uint32_t *__restrict__ wg_task,
                                                                RecState *st, uint64_t *bsums, uint64_t *frame_pos,
                                                                iggy_polled_message *msgs,
                                                                iggy_decode_result *results, uint32_t *counter,
                                                                uint32_t *host_flag, uint32_t flag_value,
                                                                GenRearm rearm, RecTask inl) {
    if (rearm.gbar && blockIdx.x == 0) {  // as k_decode_uniform's prologue
        if (threadIdx.x == 0) {
            __hip_atomic_store(&rearm.gbar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&rearm.gbar[2], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&rearm.gbar[3], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&rearm.gmisc[2], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&rearm.gmisc[kPosCountWord], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (threadIdx.x < kBar2Words)
            __hip_atomic_store(&rearm.gbar2[32 * threadIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    decode_record_block<VERIFY>(inl, base, tasks, wg_task, st, bsums, frame_pos, msgs, results);
    launch_done(counter, host_flag, flag_value);
}

// ------------------------------------------------------------ resident service
// A synchronous host decode of a small single-stride record (iggy_codec_decode_batch
// at C1, the reference's own call shape, batch.rs:391) spends most of its time on the
// launch: the host's launch call and the dispatch before the first wave runs (a
// 4-message record: ≈ 18 µs from the launch returning to its completion flag, of which
// the kernel is a few). k_decode_service keeps kSvcWgs workgroups resident instead. The
// leader (workgroup 0) polls a host-mapped mailbox and relays each post through a
// device-memory control block; every workgroup then decodes block b = its index of the
// posted record with the same block code as k_decode_records, the last one raising the
// host flag. Only the leader decides to stop (the mailbox's stop word, kSvcIdleTicks
// without a post, or the bug guard), and the followers stop on its word, so a post is
// decoded by all of its workgroups or by none (the host relaunches and re-posts it
// then). On its way out the leader clears the mailbox's `alive` word.
constexpr uint32_t kSvcWgs = kSvcWgs_;                // records of <= 8 blocks (C1: 1 000 frames)
constexpr uint32_t kSvcPre = 26;                      // 12-B pieces of the record's first 304 B
constexpr uint64_t kSvcIdleTicks = 100000ull * 20;    // 20 ms without a post: exit
constexpr uint64_t kSvcBackoffTicks = 100ull * 200;   // 200 us without a post: poll every ~4 us
// Host-mapped mailbox: 8 chunks of 16 B, read by the leader's wave in ONE round of loads
// (lane c takes chunk c). Chunks 0-5 hold the post and carry its sequence number in
// their first word, written by the host after the chunk's other words, so a load
// round that sees the same new number in all six saw the whole post.
struct SvcMailbox {
    uint32_t seq0, integrity; uint64_t len;                   // chunk 0
    uint32_t seq1, nwg; uint64_t pos_cap;                     // 1
    uint32_t seq2, flag_value; const uint8_t *base;           // 2: the record (device-visible)
    uint32_t seq3, _r3; uint64_t *frame_pos;                  // 3: positions (device-visible, nullable)
    uint32_t seq4, _r4; iggy_decode_result *result;           // 4: device-visible
    uint32_t seq5, _r5; uint32_t *host_flag;                  // 5: raised to flag_value when done
    uint32_t stop, alive, _r6[2];                             // 6: host: 1 = exit now; alive: see below
    uint64_t _r7[2];                                          // 7
    // 8..33: the record's first 304 B (batch header + frame 0's header) in 12-B pieces,
    // each after its own copy of the sequence number, so the post's load round also
    // stages what every block workgroup would otherwise fetch over the host link first
    struct { uint32_t seq; uint8_t b[12]; } pre[kSvcPre];
    uint64_t diag[8];  // (diagnostic build: stage times of the post, ticks after the leader saw it)
};
static_assert(sizeof(SvcMailbox) == 128 + 16 * kSvcPre + 64, "mailbox layout");
// Every workgroup keeps the post in LDS as kSvcPost dwords: the record's first 304 B
// (dwords 0-75, the block code's pre_head), then chunks 0-5's words y, z, w (76-93).
// The leader relays them to the followers as 47 16-B units of two 8-B granules
// {the post's sequence number, one dword} each. A follower's poll is one round of sc1
// loads of all of them (and the exit word): a round that sees one new number in all 94
// granules saw the whole relay. Each 8-B half of a 16-B sc1 store is observed untorn,
// the whole 16 B is not (see kSvcRecUnits). Round 6: the relay had been a go word
// behind a release, read behind an acquire and re-checked behind a second one, ~1.9 us
// from the leader seeing the post to the followers starting.
constexpr uint32_t kSvcPost = 76 + 18;
#ifndef IGGY_SVC_DIRECT
#define IGGY_SVC_DIRECT 1
#endif
#ifndef IGGY_SVC_INFLIGHT
#define IGGY_SVC_INFLIGHT 1
#endif
constexpr bool kSvcDirect = IGGY_SVC_DIRECT;      // followers poll the mailbox themselves (no relay)
constexpr int kSvcInflight = IGGY_SVC_INFLIGHT;   // mailbox polls in flight per poller: 1, 2 or 4
constexpr uint32_t kSvcUnits = kSvcPost / 2;
struct SvcCtl {                        // device memory, zeroed before every launch
    uint4 unit[kSvcUnits];             // the relayed post (tagged granules, see above)
    uint32_t exit, _e[3];              // unit kSvcUnits: the leader's exit word (1 = exit)
    uint32_t diag[4];                  // (diagnostic build) when the leader saw the post
    uint4 rec[kSvcRecUnits * (kSvcWgs - 1)];  // blocks 1.. of the current post hand their records to block 0 (SvcHand)
    uint64_t bdiag[2 * kSvcWgs];       // (diagnostic build) every block's entry / hashed clocks
};
static_assert(sizeof(SvcCtl) == 16 * kSvcUnits + 32 + 16 * kSvcRecUnits * (kSvcWgs - 1) + 16 * kSvcWgs,
              "control block layout");
constexpr int kAuxSys = 17;  // buffer-load cache policy sc0 | sc1: system-coherent (host-mapped memory)

__device__ __forceinline__ uint4 svc_chunk_sys(const SvcMailbox *mb, uint32_t c) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)mb, 0, sizeof(SvcMailbox), 0x00020000);
    const g4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, 16u * c, 0, kAuxSys);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint4 svc_unit_dev(const SvcCtl *ctl, uint32_t c) {  // c: 16-B unit, kSvcUnits: exit
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)ctl, 0, sizeof(SvcCtl), 0x00020000);
    const g4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, 16u * c, 0, kAuxSc1);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void svc_unit_store(SvcCtl *ctl, uint32_t c, uint4 v) {  // sc1: written through
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)ctl, 0, sizeof(SvcCtl), 0x00020000);
    const g4 w = {v.x, v.y, v.z, v.w};
    __builtin_amdgcn_raw_buffer_store_b128(w, rs, 16u * c, 0, kAuxSc1);
}

// (diagnostic build) ticks from the leader seeing the post to the flag store, into the
// mailbox's chunk 7 (the host reads it beside the flag); stamps 6 / 7: the latest
// follower's entry / hashed clock
__device__ __forceinline__ void svc_stamp(SvcMailbox *mb, SvcCtl *ctl, uint64_t *stamp, uint32_t nwg) {
    uint64_t e = stamp[1], h = stamp[2];
    for (uint32_t b = 1; b < nwg; ++b) {
        e = max(e, __hip_atomic_load(&ctl->bdiag[2 * b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        h = max(h, __hip_atomic_load(&ctl->bdiag[2 * b + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
    stamp[6] = e;
    stamp[7] = h;
    const uint64_t t0 = (uint64_t)__hip_atomic_load(&ctl->diag[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) |
                        ((uint64_t)__hip_atomic_load(&ctl->diag[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) << 32);
    for (int k = 1; k < 8; ++k)
        __hip_atomic_store(&mb->diag[k], stamp[k] - t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&mb->_r7[0], rt_now() - t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(kRecThreads) void k_decode_service(SvcMailbox *mb, uint32_t start_seq, SvcCtl *ctl,
                                                                RecState *st, uint64_t *bsums) {
    __shared__ uint32_t s_cmd;
    __shared__ __attribute__((aligned(16))) uint32_t s_post[kSvcPost + 2];  // (see kSvcPost; [kSvcPost]: its number)
    __shared__ uint64_t s_stamp[8];  // (diagnostic build)
    const int lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    uint32_t seen = start_seq;  // the last post taken (posts are numbered from 1; 0 is never one)
    uint64_t t_idle = rt_now();
    const uint64_t t_guard = t_idle;
    for (;;) {
        if (wave == 0) {  // (wave-uniform control flow: every decision comes from a shuffle)
            uint32_t cmd = 2;
            const bool leader = blockIdx.x == 0;
            if (leader || kSvcDirect) {
                // The host's mailbox, one load round per poll (kSvcInflight polls in
                // flight, each waiting only for the oldest). The leader decides stop and
                // idle exit; a follower (kSvcDirect) polls the mailbox too, so it starts
                // with the leader instead of a device hand-off later, and stops on the
                // leader's exit word, which its lane 34 loads beside the chunks.
                const uint32_t cidx = (uint32_t)min(lane, 8 + (int)kSvcPre - 1);
                const bool tagged = lane < 6 || (lane >= 8 && lane < 8 + (int)kSvcPre);
                const int xl = leader ? 6 : 34;  // (the stop word / the leader's exit word)
                const uint64_t t0 = rt_now();
                auto poll = [&]() -> uint4 {
                    return !leader && lane == 34 ? svc_unit_dev(ctl, kSvcUnits) : svc_chunk_sys(mb, cidx);
                };
                // returns true when the poll v decides (a new post: cmd 1; stop, idle, the
                // leader's exit or the bug guard: cmd 2)
                auto take = [&](const uint4 &v) -> bool {
                    if (__shfl((int)v.x, xl)) return true;
                    const uint32_t s0 = (uint32_t)__shfl((int)v.x, 0);
                    if (s0 != 0 && s0 != seen && __ballot(tagged && v.x != s0) == 0) {  // a whole new post
                        if (lane < 6) {  // chunk lane's words
                            uint32_t *d = s_post + 76 + 3u * (uint32_t)lane;
                            d[0] = v.y; d[1] = v.z; d[2] = v.w;
                        }
                        if (lane >= 8 && lane < 8 + (int)kSvcPre) {  // 12-B piece lane - 8 of the prefix
                            uint32_t *d = s_post + 3u * (uint32_t)(lane - 8);  // (76 dwords)
                            d[0] = v.y;
                            if (lane < 8 + (int)kSvcPre - 1) { d[1] = v.z; d[2] = v.w; }
                        }
                        if (lane == 0) s_post[kSvcPost] = s0;
                        if (leader && !kSvcDirect) {
                            const bool relay = (uint32_t)__shfl((int)v.y, 1) > 1;  // (a one-block post is the leader's alone)
                            // (this wave's own LDS writes have landed; the memory clobber
                            // keeps the reads below after them)
                            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                            if (relay && lane < (int)kSvcUnits)
                                svc_unit_store(ctl, (uint32_t)lane,
                                               make_uint4(s0, s_post[2 * lane], s0, s_post[2 * lane + 1]));
                        }
                        if (kDiagMask && leader && lane == 0) {  // (diagnostic build: when the post was seen)
                            const uint64_t t = rt_now();
                            ctl->diag[0] = (uint32_t)t;
                            ctl->diag[1] = (uint32_t)(t >> 32);
                        }
                        seen = s0;
                        cmd = 1;
                        return true;
                    }
                    const uint64_t now = rt_now();
                    if (!leader) return now - t0 > kSpinLimitTicks * 16;  // bug guard (the leader always ends with exit)
                    return now - t_idle > kSvcIdleTicks || now - t_guard > kSpinLimitTicks * 16;
                };
                if (kSvcInflight == 1) {
                    for (;;) {
                        if (take(poll())) break;
                        // (idle for kSvcBackoffTicks: ~4 us between polls, so a service
                        // alive between sparse posts reads ~0.8 GB/s over the host link,
                        // not ~3 GB/s; back-to-back posts never get here)
                        if (rt_now() - t_idle > kSvcBackoffTicks) __builtin_amdgcn_s_sleep(127);
                    }
                } else if (kSvcInflight == 2) {
                    uint4 p0 = poll();
                    __builtin_amdgcn_s_sleep(8);
                    uint4 p1 = poll();
                    for (;;) {
                        if (take(p0)) break;
                        p0 = poll();
                        if (take(p1)) break;
                        p1 = poll();
                    }
                } else {
                    uint4 p0 = poll();
                    __builtin_amdgcn_s_sleep(2);
                    uint4 p1 = poll();
                    __builtin_amdgcn_s_sleep(2);
                    uint4 p2 = poll();
                    for (;;) {
                        __builtin_amdgcn_s_sleep(2);
                        uint4 p3 = poll();
                        if (take(p0)) break;
                        __builtin_amdgcn_s_sleep(2);
                        p0 = poll();
                        if (take(p1)) break;
                        __builtin_amdgcn_s_sleep(2);
                        p1 = poll();
                        if (take(p2)) break;
                        __builtin_amdgcn_s_sleep(2);
                        p2 = poll();
                        if (take(p3)) break;
                    }
                }
                __builtin_amdgcn_s_waitcnt(0);  // the polls still in flight, the relay stores and the LDS writes
                if (leader && cmd != 1 && lane == 0)  // the followers stop on this word
                    __hip_atomic_store(&ctl->exit, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (lane == 0) s_cmd = cmd;
            } else {  // a follower: the leader's latest relay (one sc1 load round per poll)
                const uint64_t t0 = rt_now();
                for (;;) {
                    const uint4 v = lane <= (int)kSvcUnits ? svc_unit_dev(ctl, (uint32_t)lane) : make_uint4(0, 0, 0, 0);
                    if (__shfl((int)v.x, kSvcUnits)) break;  // the leader exits
                    const uint32_t s0 = (uint32_t)__shfl((int)v.x, 0);
                    if (s0 != 0 && s0 != seen && __ballot(lane < (int)kSvcUnits && (v.x != s0 || v.z != s0)) == 0) {
                        if (lane < (int)kSvcUnits) {
                            s_post[2 * lane] = v.y;
                            s_post[2 * lane + 1] = v.w;
                        }
                        if (lane == 0) s_post[kSvcPost] = s0;
                        seen = s0;
                        cmd = 1;
                        break;
                    }
                    if (rt_now() - t0 > kSpinLimitTicks * 16) break;  // bug guard (the leader always ends with exit)
                    __builtin_amdgcn_s_sleep(1);
                }
                if (lane == 0) s_cmd = cmd;
            }
        }
        __syncthreads();
        if (s_cmd != 1) break;
        t_idle = rt_now();
        // chunk k's words: y = s_post[76 + 3k], z | w << 32 = u64(k)
        const uint32_t *cw = s_post + 76;
        const uint32_t integ = cw[0], nwg = cw[3], flag_value = cw[6];
        auto u64 = [&](int k) { return (uint64_t)cw[3 * k + 1] | ((uint64_t)cw[3 * k + 2] << 32); };
        if (blockIdx.x < nwg && nwg <= kSvcWgs) {
            RecTask tk;
            tk.off = 0; tk.len = u64(0); tk.pos_base = 0; tk.pos_cap = u64(1); tk.msg_base = 0;
            tk.bsum_base = 0; tk.wg0 = 0; tk.nwg = nwg;
            // (made a global-space pointer first: a plain pointer out of LDS words is
            // loaded through with flat loads, which count on lgkmcnt too, and the frames'
            // whole load round was then waited for with vmcnt(0) lgkmcnt(0) before the
            // first frame's hash; global loads let each frame's hash start when its own
            // bytes have landed)
            const uint8_t *base = (const uint8_t *)(const __attribute__((address_space(1))) uint8_t *)u64(2);
            uint64_t *fpos = (uint64_t *)u64(3);
            iggy_decode_result *res = (iggy_decode_result *)u64(4);
            uint32_t *flag = (uint32_t *)u64(5);
            const uint8_t *s_pre = (const uint8_t *)s_post;
            const SvcHand hand{ctl->rec, s_post[kSvcPost], kDiagMask ? ctl->bdiag : nullptr};  // (the post's number tags its blocks' records)
            if (integ == IGGY_INTEGRITY_VERIFY)
                decode_record_block<true>(tk, base, nullptr, nullptr, st, bsums, fpos, nullptr, res, blockIdx.x, s_pre,
                                          kDiagMask ? s_stamp : nullptr, hand);
            else
                decode_record_block<false>(tk, base, nullptr, nullptr, st, bsums, fpos, nullptr, res, blockIdx.x, s_pre,
                                           kDiagMask ? s_stamp : nullptr, hand);
            // Completion: block 0 resolved the post after every other block had fenced its
            // host-visible writes at system scope and handed over its record, so its own
            // fence orders the verdict, and with it every position, before the flag.
            if (blockIdx.x == 0) {
                __threadfence_system();
                if (kDiagMask && threadIdx.x == 0) s_stamp[6] = rt_now();
                __syncthreads();
                if (kDiagMask && threadIdx.x == 0) {
                    svc_stamp(mb, ctl, s_stamp, nwg);
                    __threadfence_system();
                }
                if (threadIdx.x == 0) __hip_atomic_store(flag, flag_value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        // Every workgroup drops what its caches hold of the record before the next post:
        // the host rewrites its buffers between calls (a pageable record goes through the
        // same mapped staging every time), and the next post's in-place loads would hit
        // this one's lines -- a corrupt frame judged on the clean bytes of the call before
        // (measured). The launch path gets this from every launch's acquire. Here it comes
        // after the flag (block 0) or the hand-over (the others): off the post's path.
        // (System scope: L1 and L2. Agent scope, the L1 alone, passed the service tests
        // and saved 0.27 us per call, but nothing shows the L2 holds no host lines.)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        __syncthreads();  // (s_cmd / s_post are rewritten by the next relay)
    }
    if (blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(&mb->alive, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template __global__ void k_decode_records<true>(const uint8_t *__restrict__, const RecTask *__restrict__,
                                                const uint32_t *__restrict__, RecState *, uint64_t *, uint64_t *,
                                                iggy_polled_message *, iggy_decode_result *, uint32_t *, uint32_t *,
                                                uint32_t, GenRearm, RecTask);
template __global__ void k_decode_records<false>(const uint8_t *__restrict__, const RecTask *__restrict__,
                                                 const uint32_t *__restrict__, RecState *, uint64_t *, uint64_t *,
                                                 iggy_polled_message *, iggy_decode_result *, uint32_t *, uint32_t *,
                                                 uint32_t, GenRearm, RecTask);

}  // namespace iggy

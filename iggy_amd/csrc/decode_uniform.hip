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
// Work layout (MI355X: 256 CUs in 8 XCDs, wave64, 160 KiB LDS per CU):
//  * one persistent grid of ncu - 1 WGs of 320 threads (one CU stays free for a
//    pipelined decode's chain). Block 0 is the consumer WG; blocks 1.. produce.
//  * checksum blocks: 128 consecutive frames [128b - 6, 128b + 122) cover exactly
//    the 1024-B block b of the batch-checksum input (44 header bytes + 8 bytes per
//    frame => checksum word m = frame + 6); a 32-frame "unit" is a quarter block.
//  * Long frames under Verify (hashed length > 240 B, the C2 path): 4 lane-group
//    producer waves + 1 publisher wave per WG. Producer WG g sweeps blocks g,
//    g + NP, ...; at step j its wave w takes 8-frame group w of unit j & 3 of its
//    block j >> 2. 8 lanes per frame, 8 frames per wave-instruction: each step is
//    exactly 9 global_load_lds_dwordx4 (8 pieces of a 1-KiB block, then the last-
//    stripe piece in even lanes / the stored checksum in odd lanes) into a 4-slot
//    LDS ring per wave with a constant vmcnt (3 steps in flight). XXH3 accumulator
//    pairs stay lane-local, folded by DPP at block ends. The producers deposit each
//    group's 8 stored checksums in LDS; the publisher wave reduces each block's
//    127 interior checksum words to 8 accumulator sums and stores ONE epoch-tagged
//    128-B block record (no flag, no fence).
//  * Short frames (hashed <= 240 B) and LayoutOnly: LDS-staged producers (waves
//    0-3, 64 frames per wave per 256-frame chunk, XOR-swizzled rings, bank-balanced
//    ds_read_b128); odd/even wave pairs join their halves of a block in LDS and the
//    even wave publishes the same block record.
//  * Consumer WG: 2 gatherer waves load block records (coherent sc1 buffer loads,
//    tags checked), add each block's last word and stage 16 sums per 256-frame
//    chunk into a 64 KiB LDS ring; the chain wave (raised priority, a SIMD of its
//    own) runs the serial one-scramble-per-block batch-checksum chain beside the
//    producers, then resolves precedence (batch.rs:395-421, 461-506).
//  DESIGN.md section 4.1 has the measurements behind each choice.
#include "codec_common.hpp"

#include <utility>

namespace iggy {

struct DecodeScratch {
    uint32_t *exited;     // producer waves that finished (reset by consumer)
    uint64_t *first_bad;  // ~index of first checksum mismatch (max-encoded), 0 = none
    uint64_t *spec_fail;  // ~index of first frame whose header breaks the stride
    uint64_t *sums;       // block records: one 128-B line (16 epoch-tagged granules) per
                          // 128-frame checksum block, 2 per chunk; see publish_block
    uint64_t *errslot;    // [max_chunks*32][2] (stored, computed) of the first mismatch per 8-frame group
    uint8_t *small;       // >= 512 B: short batch-checksum inputs
    uint64_t *sink;       // 64 x u64: the lane-group producers' frame-position stores that
                          // have no frame (past N or the caller's capacity) land here
    uint32_t *gbar2;      // the general kernel's two-level barrier counters (kBar2Words, 128-B stride)
    uint32_t *gbar;       // the general kernel's barrier / registration words and its
    uint64_t *gmisc;      // first-bad slot: re-armed here (see k_decode_general); [8] stride and
                          // [9] count of the frame positions k_decode_general writes (kPosEpilogue)
    uint64_t max_chunks;
};

// ---- LDS map of a producer WG (dynamic LDS only, base offset 0) ----------
constexpr uint32_t kWaveRing = 32768;                          // per wave: 4 x 8 KiB or 2 x 16 KiB
constexpr uint32_t kSideOff = 4 * kWaveRing;                   // 131072
constexpr uint32_t kSideLane = 96;                             // 6 chunks per lane
constexpr uint32_t kLdsBytes = kSideOff + 4 * 64 * kSideLane;  // 155648
// consumer WG: ring of kRing batches of 64 chunks' block sums (16 x u64 per chunk),
// filled by kGatherWaves gatherer waves, drained by the chain wave
constexpr uint32_t kBatch = 64;
constexpr uint32_t kRing = 8;
// consumer WG waves 1..2 gather; wave 0 runs the chain at raised priority. Waves 3, 4
// idle, so only the chain wave issues on its SIMD: with 4 gatherers one shared it, and
// C2 decodes measured 0.2363-0.2402 ms against 0.2296-0.2314 ms (same box, with the
// poll-free passes below); 2 gatherers still outpace the chain when it is the bound
// (8 M x 64 B records: 1.43 ms either way)
constexpr uint32_t kGatherWaves = 2;
constexpr uint32_t kUniformThreads = 320;  // 4 producer waves + 1 publisher wave per WG (consumer: chain + 4 gatherers)
constexpr uint32_t kCtlOff = kRing * kBatch * 16 * 8;  // 64 KiB
struct ChainCtl {
    uint32_t staged[kRing];  // (batch index + 1) << 7 | leading chunks of the slot staged so far
    uint32_t consumed;      // batches the chain wave has finished
    uint32_t abort;         // a gatherer or the chain wave gave up (spin limit)
};
constexpr uint32_t kConsumerLds = kCtlOff + 64;
static_assert(kCtlOff + sizeof(ChainCtl) <= kConsumerLds, "consumer LDS");
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");

struct UPlan {
    uint32_t state;  // 0 run, 1 result known early, 2 need general
    uint32_t nck, nph, q_side0, ph;
    uint64_t S, N, L, nchunks;
    uint64_t nbF, Kreg, ns;      // per-frame hash: full blocks, regular words, partial stripes
    uint64_t n, nb, Mreg;        // batch checksum input: bytes, full blocks, regular words
    uint32_t ekind, ereason;
    uint64_t ea, eb, ec;
    bool long_frames, long_cs;
    bool nt;           // diagnostics: non-temporal LDS-DMA loads
    bool nopub;        // diagnostics (dbg bit 128): lane-group producers publish nothing
    bool tail_unsafe;  // last frame's last 16-B chunk would read past the caller's buffer
};

__device__ inline void make_plan(const HeaderInfo &hi, const uint8_t *blob, uint64_t len,
                                 bool verify, uint64_t max_chunks, bool allow_unaligned, UPlan &p) {
    p.state = 2;
    p.tail_unsafe = false;
    p.nt = false;
    p.nopub = false;
    p.ekind = IGGY_OK; p.ereason = 0; p.ea = p.eb = p.ec = 0;
    p.S = p.N = p.L = p.nchunks = 0;
    p.nck = p.nph = p.q_side0 = 0;
    p.ph = 16;
    p.nbF = p.Kreg = p.ns = p.n = p.nb = p.Mreg = 0;
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
    const uint64_t S = kFrameHdr + (uint64_t)ld32_any(blob + 36) + (uint64_t)ld32_any(blob + 32);
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
            p.ph = 8;
            p.nbF = (p.L - 1) / 1024;
            p.ns = ((p.L - 1) - 1024 * p.nbF) / 64;
            p.Kreg = 8 * (16 * p.nbF + p.ns);
            p.q_side0 = (uint32_t)((S - 64) >> 4);
        }
        p.n = 44 + 8 * p.N;
        p.long_cs = p.n > 240;
        if (p.long_cs) {
            p.nb = (p.n - 1) / 1024;
            const uint64_t ns = ((p.n - 1) - 1024 * p.nb) / 64;
            p.Mreg = 8 * (16 * p.nb + ns);
        }
    } else {
        p.nck = 3;  // header bytes 0..47 only
    }
    p.nph = (p.nck + p.ph - 1) / p.ph;
    p.tail_unsafe = hi.h.batch_length + (16ull * p.nck - S) > len;
    p.state = 0;
}

// ------------------------------------------------------------ primitives
__device__ __forceinline__ void wait_vm(uint32_t n) {
    // n = glds instructions allowed to stay in flight (multiples of 8)
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
        case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
        case 30: asm volatile("s_waitcnt vmcnt(30)" ::: "memory"); break;
        case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
        case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}


__device__ __forceinline__ uint64_t funnel64(uint64_t lo, uint64_t hi, uint32_t t) {
    return t ? ((lo >> (8 * t)) | (hi << (64 - 8 * t))) : lo;
}

// one XXH3 block step on the carried value y = acc + S_b: returns scramble(y) + S_{b+1}.
// The form measured fastest on gfx950 (26 ns/step: v_lshl_add_u64, v_xor, v_mul_lo_u32,
// v_mad_u64_u32; scripts/chain_micro.hip); the mad's 64-bit addend form is slower.
__device__ __forceinline__ uint64_t chain_step(uint64_t y, uint64_t s, uint32_t klo, uint32_t khi) {
    const uint32_t hi = (uint32_t)(y >> 32);
    const uint32_t lo = (uint32_t)y ^ (hi >> 15) ^ klo;
    const uint32_t h2 = hi ^ khi;
    uint64_t t = (uint64_t)lo * P32_1 + ((uint64_t)(h2 * P32_1) << 32);
    asm volatile("" : "+v"(t));  // keep s out of the mad's addend (that form is 1.8x slower)
    return t + s;
}

// A span of 16 * n16 chain steps over block sums staged in LDS (lane j: block k's sum at
// LDS byte address addr + 64 k), in one asm statement: y = f(y) + S_k per step, f the
// XXH3 scramble. The split form: the next sum is the 64-bit addend of the mad and the high
// word's product is added after it, so the multiply of the high word runs beside the
// mad instead of feeding it; two 8-sum register buffers are refilled by ds_read2_b64 two
// groups ahead, with constant lgkmcnt waits. The step's own latency is ~12 ns
// (scripts/lat_micro.hip, sums in registers: 12.3 ns; the compiler's form 15.8), against
// ~22 ns for the C++ loop over LDS reads that the compiler waited for group by group.
// Reads run up to 31 blocks past the span (inside the consumer's LDS; never used).
#ifndef IGGY_CHAIN_ASM
#define IGGY_CHAIN_ASM 1  // (build knob for a same-box A/B: 0 = the C++ chain loop only)
#endif
#define IGGY_CH_STEP(S)                                      \
    "v_lshrrev_b32 v42, 15, v41\n\t"                         \
    "v_xor_b32 v43, v41, %[khi]\n\t"                         \
    "v_bitop3_b32 v42, v40, v42, %[klo] bitop3:0x96\n\t"     \
    "v_mul_lo_u32 v43, v43, %[pr]\n\t"                       \
    "v_mad_u64_u32 v[40:41], s[20:21], v42, %[pr], " S "\n\t" \
    "v_add_u32 v41, v41, v43\n\t"
__device__ __forceinline__ uint64_t chain_span(uint64_t y, uint32_t addr, uint32_t n16, uint32_t klo, uint32_t khi) {
    uint32_t cnt = __builtin_amdgcn_readfirstlane(n16);
    const uint32_t pr = P32_1;
    asm volatile(
        "s_waitcnt lgkmcnt(0)\n\t"
        "ds_read2_b64 v[48:51], %[ad] offset0:0 offset1:8\n\t"
        "ds_read2_b64 v[52:55], %[ad] offset0:16 offset1:24\n\t"
        "ds_read2_b64 v[56:59], %[ad] offset0:32 offset1:40\n\t"
        "ds_read2_b64 v[60:63], %[ad] offset0:48 offset1:56\n\t"
        "ds_read2_b64 v[64:67], %[ad] offset0:64 offset1:72\n\t"
        "ds_read2_b64 v[68:71], %[ad] offset0:80 offset1:88\n\t"
        "ds_read2_b64 v[72:75], %[ad] offset0:96 offset1:104\n\t"
        "ds_read2_b64 v[76:79], %[ad] offset0:112 offset1:120\n\t"
        "v_lshl_add_u64 v[40:41], %[y], 0, 0\n\t"
        "L_chain_%=:\n\t"
        "s_waitcnt lgkmcnt(4)\n\t"
        IGGY_CH_STEP("v[48:49]") IGGY_CH_STEP("v[50:51]") IGGY_CH_STEP("v[52:53]") IGGY_CH_STEP("v[54:55]")
        IGGY_CH_STEP("v[56:57]") IGGY_CH_STEP("v[58:59]") IGGY_CH_STEP("v[60:61]") IGGY_CH_STEP("v[62:63]")
        "ds_read2_b64 v[48:51], %[ad] offset0:128 offset1:136\n\t"
        "ds_read2_b64 v[52:55], %[ad] offset0:144 offset1:152\n\t"
        "ds_read2_b64 v[56:59], %[ad] offset0:160 offset1:168\n\t"
        "ds_read2_b64 v[60:63], %[ad] offset0:176 offset1:184\n\t"
        "s_waitcnt lgkmcnt(4)\n\t"
        IGGY_CH_STEP("v[64:65]") IGGY_CH_STEP("v[66:67]") IGGY_CH_STEP("v[68:69]") IGGY_CH_STEP("v[70:71]")
        IGGY_CH_STEP("v[72:73]") IGGY_CH_STEP("v[74:75]") IGGY_CH_STEP("v[76:77]") IGGY_CH_STEP("v[78:79]")
        "ds_read2_b64 v[64:67], %[ad] offset0:192 offset1:200\n\t"
        "ds_read2_b64 v[68:71], %[ad] offset0:208 offset1:216\n\t"
        "ds_read2_b64 v[72:75], %[ad] offset0:224 offset1:232\n\t"
        "ds_read2_b64 v[76:79], %[ad] offset0:240 offset1:248\n\t"
        "v_add_u32 %[ad], 0x400, %[ad]\n\t"
        "s_sub_u32 %[cnt], %[cnt], 1\n\t"
        "s_cmp_lg_u32 %[cnt], 0\n\t"
        "s_cbranch_scc1 L_chain_%=\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_lshl_add_u64 %[y], v[40:41], 0, 0\n\t"
        : [y] "+v"(y), [ad] "+v"(addr), [cnt] "+s"(cnt)
        : [klo] "v"(klo), [khi] "v"(khi), [pr] "v"(pr)
        : "memory", "scc", "s20", "s21", "v40", "v41", "v42", "v43", "v48", "v49", "v50", "v51", "v52", "v53",
          "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68",
          "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79");
    return y;
}

// issue phase p of this wave's 64 frames of chunk c: instruction k moves frames
// (64/PH)k .. (64/PH)k + 64/PH - 1, PH lanes x 16 B = PH*16 contiguous bytes each
template <int PH>
__device__ __forceinline__ void issue_phase(const uint8_t *blob, const UPlan &pl, int64_t iw0,
                                            uint32_t p, uint32_t lds_slot, int lane) {
    constexpr int FPI = 64 / PH;  // frames per instruction
    const int fsub = lane / PH;
    int64_t i = iw0 + fsub;
    const uint8_t *fb = blob + (uint64_t)i * pl.S;
    const uint64_t step = (uint64_t)FPI * pl.S;
#pragma unroll
    for (int k = 0; k < PH; ++k) {
        const int f = FPI * k + fsub;
        const uint32_t cidx = (uint32_t)((lane % PH) ^ (f % PH));
        const uint32_t q = PH * p + cidx;
        const bool ok = (i >= 0) && ((uint64_t)i < pl.N) && (q < pl.nck) &&
                        !(pl.tail_unsafe && (uint64_t)i == pl.N - 1 && 16ull * q + 16 > pl.S);
        const uint8_t *src = ok ? fb + 16ull * q : blob;
        glds16(src, lds_slot + 1024u * k, pl.nt);
        i += FPI;
        fb += step;
    }
}

// ------------------------------------------------------------- phase body
struct PhaseState {
    Acc8 acc;
    uint64_t stored, resv;
    uint32_t uh, plen;
};

// chunk C (compile-time) of phase p (p % (64/PH) == PM) for this lane's frame.
// Returns true when the frame has no chunk C (end of the phase loop).
template <int PH, int PM, bool CHECKED, bool VERIFY, int C>
__device__ __forceinline__ bool chunk_step(const uint8_t *lbase, uint32_t sw, uint8_t *side,
                                           uint32_t p, const UPlan &pl, PhaseState &st) {
    const uint32_t q = PH * p + C;
    if (CHECKED && q >= pl.nck) return true;
    const uint4 D = *(const uint4 *)(lbase + 16u * ((uint32_t)C ^ sw));
    const uint64_t u0 = (uint64_t)D.x | ((uint64_t)D.y << 32);
    const uint64_t u1 = (uint64_t)D.z | ((uint64_t)D.w << 32);
    if (PM == 0 && C == 0 && CHECKED) {
        if (p == 0) st.stored = u0;
    }
    if (PM == 0 && C == 2 && CHECKED) {
        if (p == 0) { st.uh = D.x; st.plen = D.y; st.resv = u1; }
    }
    if (!VERIFY || PH != 8) return false;  // hashing here only for long frames (PH == 8)
    if (CHECKED && q >= pl.q_side0) *(uint4 *)(side + 16u * (q - pl.q_side0)) = D;
    // unit 2q -> hashed word k = 2q-1 ; unit 2q+1 -> word 2q
    constexpr int J0 = (2 * C - 1) & 7;
    constexpr int SIB0 = ((PH / 4) * PM + ((2 * C - 1) >> 3)) & 15;
    constexpr int J1 = (2 * C) & 7;
    constexpr int SIB1 = ((PH / 4) * PM + ((2 * C) >> 3)) & 15;
    {
        const int64_t k0 = 2 * (int64_t)q - 1;
        const bool reg0 = CHECKED ? (k0 >= 0 && (uint64_t)k0 < pl.Kreg) : true;
        if (reg0) st.acc.word<J0>(u0, Secret::w(8 * (SIB0 + J0)));
        if (C == 0 && PM == 0) {  // word 128b+127 closes block b = p*PH/64 - 1
            if (p > 0 && (uint64_t)(p * PH / 64 - 1) < pl.nbF) st.acc.scramble();
        }
    }
    {
        const uint64_t k1 = 2 * (uint64_t)q;
        const bool reg1 = CHECKED ? (k1 < pl.Kreg) : true;
        if (reg1) st.acc.word<J1>(u1, Secret::w(8 * (SIB1 + J1)));
    }
    return false;
}

template <int PH, int PM, bool CHECKED, bool VERIFY, int... Cs>
__device__ __forceinline__ void phase_chunks(std::integer_sequence<int, Cs...>, const uint8_t *lbase,
                                             uint32_t sw, uint8_t *side, uint32_t p,
                                             const UPlan &pl, PhaseState &st) {
    (void)(chunk_step<PH, PM, CHECKED, VERIFY, Cs>(lbase, sw, side, p, pl, st) || ...);
}

template <int PH, int PM, bool CHECKED, bool VERIFY>
__device__ __forceinline__ void phase_body(const uint8_t *slot, uint8_t *side, int lane, uint32_t p,
                                           const UPlan &pl, PhaseState &st) {
    phase_chunks<PH, PM, CHECKED, VERIFY>(std::make_integer_sequence<int, PH>{},
                                          slot + (uint32_t)lane * (PH * 16u),
                                          (uint32_t)(lane % PH), side, p, pl, st);
}

template <int PH, bool VERIFY, int... PMs>
__device__ __forceinline__ void run_phase_impl(std::integer_sequence<int, PMs...>, const uint8_t *slot,
                                               uint8_t *side, int lane, uint32_t p, const UPlan &pl,
                                               PhaseState &st) {
    constexpr uint32_t NPM = 64 / PH;
    // a phase is "full" when all its words are regular and none needs side capture
    const bool full = VERIFY && PH == 8 && p > 0 && (PH * p + PH - 1 < pl.nck) &&
                      (2ull * (PH * p + PH - 1) < pl.Kreg) && (PH * p + PH - 1 < pl.q_side0);
    const uint32_t pm = p % NPM;
    (void)((pm == (uint32_t)PMs
                ? (full ? phase_body<PH, PMs, false, VERIFY>(slot, side, lane, p, pl, st)
                        : phase_body<PH, PMs, true, VERIFY>(slot, side, lane, p, pl, st),
                   true)
                : false) ||
           ...);
}

template <int PH, bool VERIFY>
__device__ __forceinline__ void run_phase(const uint8_t *slot, uint8_t *side, int lane, uint32_t p,
                                          const UPlan &pl, PhaseState &st) {
    run_phase_impl<PH, VERIFY>(std::make_integer_sequence<int, 64 / PH>{}, slot, side, lane, p, pl, st);
}

// short frames (hashed length 40..240): random access inside the 16-chunk image
__device__ inline uint64_t short_hash(const uint8_t *slot, int lane, uint64_t L) {
    const uint32_t sw = (uint32_t)(lane & 15);
    const uint8_t *lbase = slot + (uint32_t)lane * 256u;
    auto unit = [&](uint32_t u) -> uint64_t {
        return *(const uint64_t *)(lbase + 16u * ((u >> 1) ^ sw) + 8u * (u & 1));
    };
    auto rd = [&](uint64_t hoff) -> uint64_t {  // hashed offset -> stream offset 8 + hoff
        const uint64_t o = 8 + hoff;
        const uint32_t u = (uint32_t)(o >> 3), t = (uint32_t)(o & 7);
        const uint64_t lo = unit(u);
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

// ---- block records: what the producers hand the batch-checksum chain
// The chain consumes, per 1024-B block b of the checksum input (words m = 128b ..
// 128b + 127, word m = hi32(cs_{m-6}) | lo32(cs_{m-5}) << 32 for the stored frame
// checksums cs), the block's 8 accumulator partial sums. Block b is summed by the
// producer WG that hashed its frames 128b - 6 .. 128b + 121 and published as ONE
// 128-B line: 16 granules [data32 | spare8 << 32 | tag24 << 40], granule t = half
// (t & 1) of acc[t >> 1] over words 128b .. 128b + 126; the spare bytes of granules
// 0-3 carry lo32(cs_{128b-6}), of 4-7 hi32(cs_{128b+121}), from which the gatherer
// forms the block's last word (it spans into block b + 1). No flag, no fence: each
// 8-B store is single-copy atomic and the gatherer checks every tag.
// Why lines: the gatherer's CU gets ~1/256 of HBM bandwidth under the producers'
// full read stream (~20 GB/s), so it must read few bytes -- 1 MiB for C2. (32-frame
// unit records, 144 B each, read 8 MiB: the chain waited ~200 us on them; 8-B
// column-major granules written by many CUs cost ~100 us of partial-line writes.)
constexpr uint32_t kBlockWords = 16;                     // granules per block record
constexpr uint32_t kChunkSumWords = 2 * kBlockWords;     // u64 per 256-frame chunk
constexpr uint32_t kUnitsPerChunk = 8;                   // 32-frame lane-group units
constexpr uint32_t kEpochMask = 0xFFFFFF;                // host: tags wrap -> sums re-zeroed
__device__ __forceinline__ uint64_t *block_rec(const DecodeScratch &sc, uint64_t b) {
    return sc.sums + b * kBlockWords;
}
// word m's contribution: acc[m & 7] += mul32x32(v ^ secret), acc[(m & 7) ^ 1] += v
__device__ __forceinline__ void word_contrib(uint64_t Mreg, uint64_t m, uint64_t cur, uint64_t nxt, bool use,
                                             uint64_t &x, uint64_t &y) {
    if (use && m >= 6 && m < Mreg) {
        const uint64_t v = (cur >> 32) | (nxt << 32);
        y += v;
        x += mul32x32(v ^ kSecretW8[((m >> 3) & 15) + (m & 7)]);
    }
}
// the same with the word's secret already in a register
__device__ __forceinline__ void word_contrib_s(uint64_t Mreg, uint64_t m, uint64_t cur, uint64_t nxt, bool use,
                                               uint64_t sec, uint64_t &x, uint64_t &y) {
    if (use && m >= 6 && m < Mreg) {
        const uint64_t v = (cur >> 32) | (nxt << 32);
        y += v;
        x += mul32x32(v ^ sec);
    }
}
// lanes hold words with m & 7 == lane & 7: returns acc[j] on lanes j < 8
__device__ __forceinline__ uint64_t reduce_acc8(uint64_t x, uint64_t y) {
    x += __shfl_xor(x, 8); y += __shfl_xor(y, 8);
    x += __shfl_xor(x, 16); y += __shfl_xor(y, 16);
    x += __shfl_xor(x, 32); y += __shfl_xor(y, 32);
    return x + __shfl_xor(y, 1);
}
// t8: acc[j] on lanes j < 8 (all lanes call); first_lo / last_hi wave-uniform
__device__ __forceinline__ void publish_block(const DecodeScratch &sc, uint32_t epoch, uint64_t b, int lane,
                                              uint64_t t8, uint32_t first_lo, uint32_t last_hi) {
    const uint32_t t = (uint32_t)lane & 15;
    const uint64_t a = __shfl(t8, (int)(t >> 1));
    const uint32_t data = (t & 1) ? (uint32_t)(a >> 32) : (uint32_t)a;
    const uint32_t sp = t < 4 ? (first_lo >> (8 * t)) & 0xffu : t < 8 ? (last_hi >> (8 * (t - 4))) & 0xffu : 0u;
    if (lane < 16)
        __hip_atomic_store(block_rec(sc, b) + t, (uint64_t)data | ((uint64_t)sp << 32) | ((uint64_t)epoch << 40),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// LDS-staged producers: waves 2k and 2k+1 hold the two halves of block 2c + k; the
// odd wave hands its partial sums over in LDS (after the producer rings)
constexpr uint32_t kXchOff = kLdsBytes;
constexpr uint32_t kXchBytes = 512;  // [2][128 B] partials + first_lo|last_hi, then full[2], taken[2]
__device__ __forceinline__ uint32_t *xch_flags(uint8_t *smem) { return (uint32_t *)(smem + kXchOff + 256); }

// ------------------------------------------------------------- producer
// One wave's whole life: every chunk of this WG, streamed through its ring.
template <int PH, int NSLOT, int DEPTH, bool VERIFY>
__device__ __forceinline__ void produce(const uint8_t *blob, const UPlan &pl, uint64_t *frame_pos, uint64_t cap,
                        const DecodeScratch &sc, uint32_t epoch, uint32_t g, uint32_t nprod,
                        uint32_t wave, int lane, uint8_t *smem, uint32_t dbg) {
    constexpr uint32_t kSlot = 64u * PH * 16u;
    static_assert(NSLOT * kSlot <= kWaveRing, "ring");
    const uint32_t ring = wave * kWaveRing;
    uint8_t *side = smem + kSideOff + wave * 64 * kSideLane + (uint32_t)lane * kSideLane;
    const uint32_t tid = wave * 64 + (uint32_t)lane;
    // secret words of this wave's checksum words m = 256 c + 64 wave + lane (any chunk
    // c) and of its joining word m = 256 c + 64 wave + 63: wave and lane only
    const uint64_t cs_sec = kSecretW8[((tid >> 3) & 15) + (tid & 7)];
    const uint64_t join_sec = kSecretW8[((8 * wave + 7) & 15) + 7];

    // flat stream of steps (chunk, phase) issued DEPTH ahead of the compute side
    uint64_t ic = g;
    uint32_t ip = 0, iss = 0, k = 0;
    auto issue_next = [&]() {
        if (ic >= pl.nchunks) return;
        issue_phase<PH>(blob, pl, (int64_t)(256 * ic) - 6 + 64 * (int64_t)wave, ip,
                        ring + (iss % NSLOT) * kSlot, lane);
        ++iss;
        if (++ip == pl.nph) { ip = 0; ic += nprod; }
    };
    for (int d = 0; d < DEPTH; ++d) issue_next();

    const uint64_t t_start = rt_now();
    uint32_t it = 0;  // chunks done (the wave pair's exchange generation)
    for (uint64_t c = g; c < pl.nchunks; c += nprod) {
        const int64_t i = (int64_t)(256 * c) - 6 + 64 * (int64_t)wave + lane;
        const bool fvalid = i >= 0 && (uint64_t)i < pl.N;
        PhaseState st;
        st.acc.init();
        st.stored = 0; st.resv = 0; st.uh = 0; st.plen = 0;
        uint32_t slot_last = 0;
        for (uint32_t p = 0; p < pl.nph; ++p) {
            issue_next();
            wait_vm(PH * (iss - 1 - k));  // step k landed; later steps may stay in flight
            slot_last = ring + (k % NSLOT) * kSlot;
            if (dbg & 8) { ++k; continue; }  // diagnostics: loads only
            if (dbg & 2) run_phase<PH, false>(smem + slot_last, side, lane, p, pl, st);
            else run_phase<PH, VERIFY>(smem + slot_last, side, lane, p, pl, st);
            ++k;
        }
        if (dbg & 8) { ++it; continue; }
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
                for (int x = 0; x < 9; ++x) U[x] = (x < 8 || t) ? *(const uint64_t *)(side + 8u * (u0 + x)) : 0;
                st.acc.word<0>(funnel64(U[0], U[1], t), Secret::w(121));
                st.acc.word<1>(funnel64(U[1], U[2], t), Secret::w(129));
                st.acc.word<2>(funnel64(U[2], U[3], t), Secret::w(137));
                st.acc.word<3>(funnel64(U[3], U[4], t), Secret::w(145));
                st.acc.word<4>(funnel64(U[4], U[5], t), Secret::w(153));
                st.acc.word<5>(funnel64(U[5], U[6], t), Secret::w(161));
                st.acc.word<6>(funnel64(U[6], U[7], t), Secret::w(169));
                st.acc.word<7>(funnel64(U[7], U[8], t), Secret::w(177));
                h = st.acc.merge(pl.L);
            } else {
                h = short_hash(smem + slot_last, lane, pl.L);
            }
        }
        const uint64_t stored = st.stored;
        const bool spec_bad = fvalid && (st.resv != 0 || (uint64_t)kFrameHdr + st.plen + st.uh != pl.S);
        // the last frame of a record that ends at the buffer end is verified by the
        // consumer from exact-extent reads (its last chunk was not staged)
        const bool mism = VERIFY && fvalid && h != stored && !(pl.tail_unsafe && (uint64_t)i == pl.N - 1);
        if (frame_pos && fvalid && (uint64_t)i < cap) frame_pos[i] = (uint64_t)i * pl.S;
        const uint64_t mb = __ballot(mism);
        if (mb) {
            const int leader = __builtin_ctzll(mb);
            if (lane == leader) {
                atomicMax((unsigned long long *)sc.first_bad, (unsigned long long)~(uint64_t)i);
                const uint64_t slot = (uint64_t)(i + 6) >> 3;  // the frame's 8-frame group
                __hip_atomic_store(&sc.errslot[2 * slot], stored, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&sc.errslot[2 * slot + 1], h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        const uint64_t sb = __ballot(spec_bad);
        if (sb) {
            const int leader = __builtin_ctzll(sb);
            if (lane == leader) atomicMax((unsigned long long *)sc.spec_fail, (unsigned long long)~(uint64_t)i);
        }
        if (VERIFY && pl.long_cs) {
            // words m = i + 6 of this wave's 64 frames; lane 63's word spans into the
            // next wave's frames (the even wave adds it after the exchange; the odd
            // wave's is the block's last word, added by the gatherer)
            const uint64_t m = (uint64_t)(i + 6);
            uint64_t x = 0, y = 0;
            word_contrib_s(pl.Mreg, m, stored, __shfl_down(stored, 1), lane < 63, cs_sec, x, y);
            uint64_t t8 = reduce_acc8(x, y);
            const uint32_t first_lo = (uint32_t)__shfl(stored, 0);
            const uint32_t last_hi = (uint32_t)(__shfl(stored, 63) >> 32);
            const uint32_t k = wave >> 1;
            uint64_t *xv = (uint64_t *)(smem + kXchOff + 128u * k);
            uint32_t *full = xch_flags(smem) + k, *taken = xch_flags(smem) + 2 + k;
            bool ok = true;
            if (wave & 1) {  // hand over once the even wave has taken the previous pair
                while (__hip_atomic_load(taken, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != it) {
                    __builtin_amdgcn_s_sleep(1);
                    if (rt_now() - t_start > kSpinLimitTicks) { ok = false; break; }  // bug guard
                }
                if (lane < 8) xv[lane] = t8;
                if (lane == 8) xv[8] = (uint64_t)first_lo | ((uint64_t)last_hi << 32);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (ok && lane == 0) __hip_atomic_store(full, it + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else {
                while (__hip_atomic_load(full, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != it + 1) {
                    __builtin_amdgcn_s_sleep(1);
                    if (rt_now() - t_start > kSpinLimitTicks) { ok = false; break; }
                }
                const uint64_t pt8 = xv[lane & 7];
                const uint64_t pfl = xv[8];
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (lane == 0) __hip_atomic_store(taken, it + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                // the word joining the halves: hi32 of this wave's last frame, lo32 of the odd wave's first
                uint64_t bx = 0, by = 0;
                word_contrib_s(pl.Mreg, m - lane + 63, (uint64_t)last_hi << 32, pfl, true, join_sec, bx, by);
                t8 += pt8 + (lane == 7 ? bx : 0) + (lane == 6 ? by : 0);
                if (ok) publish_block(sc, epoch, 2 * c + k, lane, t8, first_lo, (uint32_t)(pfl >> 32));
            }
        }
        ++it;
    }
    wait_vm(0);
    if (lane == 0) __hip_atomic_fetch_add(sc.exited, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------- lane-group producer
// Long frames (hashed length L > 240) under Verify. 8 lanes per frame, 8 frames
// (one "group") per wave-instruction: lane i of instruction k loads 16 B of frame
// (i >> 3), so one instruction moves one 128-B segment of each of 8 frames. The
// bytes are staged through LDS by global_load_lds_dwordx4 (the wave never waits on
// a load it just issued: an explicit constant vmcnt keeps 3 steps in flight).
//
// Lane l of a frame group loads piece (m = l>>1) of stripe (2q + (l&1)) of
// segment q: hashed words 2m, 2m+1, i.e. accumulators acc[2m], acc[2m+1] of
// that stripe (acc[j] += mul32x32(w_j ^ s), acc[j^1] += w_j stays lane-local).
// The two lanes of a pair hold partial sums of even / odd stripes; they are
// combined (DPP quad_perm) at every 1024-B block end, scrambled, and carried
// by the even lane.
//
// Work order: a sweep over 128-frame blocks. Producer WG g takes blocks g, g + NP,
// ...; at step j it takes unit (j & 3) of its block (j >> 2) (32 frames) and its
// wave w the unit's 8-frame group w, so the chip reads a window of NP blocks at a
// time and block b is done early (the batch-checksum chain starts after the first
// blocks, not after each WG's first chunk). The 4 waves deposit each unit's stored
// checksums in LDS; the WG's fifth wave sums and publishes each block.
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)x, CTRL, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(x >> 32), CTRL, 0xF, 0xF, false);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
constexpr int kDppXor1 = 0xB1;  // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;  // quad_perm [2,3,0,1]
__device__ __forceinline__ uint64_t swz_xor4(uint64_t x) {  // ds_swizzle bit mode, xor_mask 4
    const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)x, 0x101F);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)(x >> 32), 0x101F);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

// The lane-group producer's whole view of the record (a small subset of UPlan,
// so the lane-group producer loop carries no state of the other forms).
struct LgPlan {
    uint64_t S, N, L, nbF, ns, nchunks, Mreg;
    bool long_cs, nt, nopub;
    uint32_t dbg;
};
__device__ __forceinline__ LgPlan lg_plan(const UPlan &p) {
    LgPlan q;
    q.S = p.S; q.N = p.N; q.L = p.L; q.nbF = p.nbF; q.ns = p.ns; q.nchunks = p.nchunks; q.Mreg = p.Mreg;
    q.long_cs = p.long_cs; q.nt = p.nt; q.nopub = p.nopub; q.dbg = 0;
    return q;
}

struct LgBuf {
    uint4 v[8];  // 8 segments x 16 B of one block (or the partial block)
    uint4 x;     // final step: the last-stripe piece (even lanes) / the stored checksum (odd lanes)
};

struct LgLane {  // per-lane constants
    uint32_t l, m, par, fg, poff;
    uint64_t s0[8], s1[8];
    uint64_t key0, key1, init0, init1, last0, last1, mrg0, mrg1;
    uint64_t wsec[4];  // lane 0 of frame fg: secret word k + fg of the block's word t = 8k + fg, k = 4 q + wave
};

__device__ __forceinline__ int64_t lg_frame_index(uint64_t u, uint32_t w, uint32_t fg) {
    return (int64_t)(32 * u) - 6 + 8 * (int64_t)w + fg;
}

// A frame group takes nsteps = nbF + (ns > 0) steps (at least 1): one per full
// 1024-B block, plus one for the partial block when it has stripes. Every step
// issues exactly 9 loads (8 pieces, then the last-stripe piece in even lanes and
// the stored checksum in odd lanes); the ninth is real only on the group's final
// step (elsewhere it re-reads the frame start and lands in a sink). The constant
// count lets the wave wait for THIS step's loads while the next steps' stay in
// flight. C2 (L = 1064: nbF = 1, ns = 0) runs one 9-load step per group.
// uses of x cannot move above this point; forces x to be materialised here
__device__ __forceinline__ void pin_after_wait(uint64_t &x) { asm volatile("" : "+v"(x)); }

__device__ __forceinline__ uint32_t lg_nsteps(const LgPlan &pl) {
    const uint32_t n = (uint32_t)pl.nbF + (pl.ns > 0 ? 1u : 0u);
    return n ? n : 1u;
}

// Issue one step: 9 x global_load_lds_dwordx4 into the 9-KiB LDS slot `slot`; lane
// i of instruction k lands at slot + 1024k + 16i, so each lane later reads back
// exactly its own 16 B. The loads bypass VGPRs: the wave waits for them with an
// explicit vmcnt, and never blocks on the step it has just issued.
#ifndef IGGY_LG_POS_EXACT
#define IGGY_LG_POS_EXACT 0  // (build knob for a same-box A/B)
#endif
constexpr uint32_t kLgLoads = 9;
constexpr uint32_t kLgStepBytes = kLgLoads * 1024;
template <bool ONE>
__device__ __forceinline__ void lg_issue(const uint8_t *blob, const LgPlan &pl, const LgLane &c, uint64_t u,
                                         uint32_t w, uint32_t b, uint32_t nsteps, uint32_t slot) {
    const int64_t i = lg_frame_index(u, w, c.fg);
    const bool valid = i >= 0 && (uint64_t)i < pl.N;
    const uint8_t *fb = blob + (valid ? (uint64_t)i : 0) * pl.S;
    const uint8_t *hb = fb + 8 + 1024ull * b + c.poff;
    const bool full = ONE || b < pl.nbF;
    const bool fin = ONE || b + 1 == nsteps;
    if (full) {  // one base address, immediate offsets
        glds16o<0>(hb, slot);
        glds16o<128>(hb, slot + 1024u);
        glds16o<256>(hb, slot + 2048u);
        glds16o<384>(hb, slot + 3072u);
        glds16o<512>(hb, slot + 4096u);
        glds16o<640>(hb, slot + 5120u);
        glds16o<768>(hb, slot + 6144u);
        glds16o<896>(hb, slot + 7168u);
    } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) glds16((2 * q + c.par < pl.ns) ? hb + 128 * q : fb, slot + 1024u * q);
    }
    // ninth load: even lanes the last-stripe piece; lane 1 the frame's own start (its
    // stored checksum); lane 3 the NEXT frame's start (its stored checksum, for the
    // batch-checksum word that straddles the two frames, lg_words); lanes 5, 7 a sink
    const int64_t inx = i + 1;
    const bool nvalid = inx >= 0 && (uint64_t)inx < pl.N;
    const uint8_t *x9 = !c.par ? (fin ? fb + 8 + pl.L - 64 + 16 * c.m : fb)
                               : (c.m == 1 && fin && nvalid) ? blob + (uint64_t)inx * pl.S : fb;
    glds16(x9, slot + 8u * 1024u);
}
__device__ __forceinline__ void lg_read(const uint8_t *smem, uint32_t slot, int lane, LgBuf &B) {
    const uint8_t *p = smem + slot + 16u * (uint32_t)lane;
#pragma unroll
    for (int q = 0; q < 8; ++q) B.v[q] = *(const uint4 *)(p + 1024u * q);
    B.x = *(const uint4 *)(p + 8u * 1024u);
}

__device__ __forceinline__ void lg_piece(uint64_t &a0, uint64_t &a1, uint4 p, uint64_t s0, uint64_t s1) {
    const uint64_t w0 = (uint64_t)p.x | ((uint64_t)p.y << 32);
    const uint64_t w1 = (uint64_t)p.z | ((uint64_t)p.w << 32);
    a0 += mul32x32(w0 ^ s0) + w1;
    a1 += mul32x32(w1 ^ s1) + w0;
}

struct LgState {
    uint64_t a0, a1, stored, next;  // lane 0 of a frame: its stored checksum, the next frame's
    uint32_t sink;  // filler loads' values land here (keeps their loads live)
    bool sbad;
};

// One step of one frame group. Returns true on the group's final step (the
// frame's hash compared, st.stored = its stored checksum in the even lanes).
template <bool ONE>
__device__ __forceinline__ bool lg_process(const LgPlan &pl, const LgLane &c, const DecodeScratch &sc,
                                           uint64_t *frame_pos, uint64_t cap, uint64_t u, uint32_t w, uint32_t b,
                                           uint32_t nsteps, const LgBuf &B, LgState &st, int lane) {
    if (pl.nt) {  // diagnostics (dbg bit 64): staging only, no hashing
#pragma unroll
        for (int q = 0; q < 8; ++q) st.sink += B.v[q].x ^ B.v[q].w;
        st.sink += B.x.y ^ B.x.x;
        st.stored = 0;
        st.next = 0;
        return ONE || b + 1 == nsteps;
    }
    if (ONE || b == 0) {
        st.a0 = c.init0;
        st.a1 = c.init1;
        // frame header: hashed word 3 = user_headers_len | payload_len (lane 2),
        // hashed word 4 = reserved (lane 4); both in the first segment
        const int64_t i = lg_frame_index(u, w, c.fg);
        const bool valid = i >= 0 && (uint64_t)i < pl.N;
        const uint4 h0 = B.v[0];
        st.sbad = valid && ((c.l == 2 && (uint64_t)kFrameHdr + h0.z + h0.w != pl.S) ||
                            (c.l == 4 && (h0.x | h0.y) != 0));
    }
    if (ONE || b < pl.nbF) {  // a full block: accumulate, fold the pair, scramble
        // four independent partial sums per accumulator: the 16 mads overlap instead
        // of forming two dependent chains of 8 (sums commute inside a block)
        uint64_t p0[4] = {0, 0, 0, 0}, p1[4] = {0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < 8; ++q) lg_piece(p0[q & 3], p1[q & 3], B.v[q], c.s0[q], c.s1[q]);
        st.a0 += (p0[0] + p0[1]) + (p0[2] + p0[3]);
        st.a1 += (p1[0] + p1[1]) + (p1[2] + p1[3]);
        st.a0 += dpp64<kDppXor1>(st.a0);
        st.a1 += dpp64<kDppXor1>(st.a1);
        st.a0 = scramble1(st.a0, c.key0);
        st.a1 = scramble1(st.a1, c.key1);
        if (c.par) { st.a0 = 0; st.a1 = 0; }
    } else {  // the partial block's stripes (only when ns > 0)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            if (2 * q < pl.ns && 2 * q + c.par < pl.ns) lg_piece(st.a0, st.a1, B.v[q], c.s0[q], c.s1[q]);
            else st.sink += B.v[q].x ^ B.v[q].y ^ B.v[q].z ^ B.v[q].w;  // unused piece: keep its load live
        }
    }
    if (!ONE && b + 1 != nsteps) {
        st.sink += B.x.x ^ B.x.y ^ B.x.z ^ B.x.w;  // a filler load: consume the registers it writes
        return false;
    }
    // final step of the frame group: fold the pair, last stripe (even lanes), merge
    st.a0 += dpp64<kDppXor1>(st.a0);
    st.a1 += dpp64<kDppXor1>(st.a1);
    lg_piece(st.a0, st.a1, B.x, c.last0, c.last1);  // odd lanes: garbage, never used
    uint64_t t = fold64(st.a0 ^ c.mrg0, st.a1 ^ c.mrg1);
    t += dpp64<kDppXor2>(t);  // the even lanes of the four m sum among themselves
    t += swz_xor4(t);
    const uint64_t h = avalanche(pl.L * P64_1 + t);
    const int64_t i = lg_frame_index(u, w, c.fg);
    const bool valid = i >= 0 && (uint64_t)i < pl.N;
    // the stored checksum, loaded by lane 1 of the frame's lanes, for lane 0; the next
    // frame's, loaded by lane 3, lands in lane 2 and then (quad swap) in lane 0 too
    const uint64_t sraw = (uint64_t)B.x.x | ((uint64_t)B.x.y << 32);
    const uint64_t stored = dpp64<kDppXor1>(sraw);
    st.stored = stored;
    st.next = dpp64<kDppXor2>(stored);
    const bool mism = valid && c.l == 0 && h != stored;
    const uint64_t mb = __ballot(mism);
    if (mb) {  // the group's first mismatching frame (lowest lane)
        const int leader = __builtin_ctzll(mb);
        if (lane == leader) {
            atomicMax((unsigned long long *)sc.first_bad, (unsigned long long)~(uint64_t)i);
            const uint64_t grp = 4 * u + w;  // (i + 6) >> 3
            __hip_atomic_store(&sc.errslot[2 * grp], stored, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&sc.errslot[2 * grp + 1], h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    const uint64_t sb = __ballot(st.sbad);
    if (sb) {
        const int leader = __builtin_ctzll(sb);
        if (lane == leader) atomicMax((unsigned long long *)sc.spec_fail, (unsigned long long)~(uint64_t)i);
    }
    if (ONE && IGGY_LG_POS_EXACT) {
        // one store instruction per step on every path (the group's 8 lanes write the same
        // word; lanes without a frame write the sink), so the ring's vmcnt wait can count it
        if (frame_pos && !pl.nopub) {
            uint64_t *dst = (valid && (uint64_t)i < cap) ? frame_pos + i : sc.sink + lane;
            asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(dst), "v"((uint64_t)i * pl.S) : "memory");
        }
    } else if (c.l == 0 && !pl.nopub && valid && (uint64_t)i < cap && frame_pos) {
        frame_pos[i] = (uint64_t)i * pl.S;
    }
    return true;
}

// ---- per-WG block combine in LDS (after the lane-group rings)
// The batch-checksum words of a 128-frame block are formed by the producer lanes
// that hold the stored checksums: lane 0 of each frame (stored checksum from lane 1,
// the NEXT frame's from lane 3's extra load, lg_issue) forms the frame's word
// t = 8k + fg (k = 4 unit + wave: the frame group), m = 128 b + t, accumulator
// m & 7 = fg, and the 8 groups' x / y parts are combined with one DPP row rotation;
// each wave sums its 4 groups of the block in registers, then adds the 8 accumulator
// contributions into the block's LDS slot (ds_add_u64, 8 lanes) and counts itself in.
// The WG's fifth wave publishes a block once its 4 waves are in: 8 sums read back,
// the slot zeroed and released, one
// 128-B record stored. The block's last word (t = 127, straddling into the next
// block) stays the gatherer's, from the spare bytes (first_lo of frame t = 0, last_hi
// of frame t = 127, written by the two groups that hold them).
// Round 3 had the publisher form all 127 words from the 128 deposited checksums
// (two words, a 64-bit 8/16/32 shuffle reduction and the 8-way spread per block):
// ~20 us of a C2 launch. Publishing from the producer waves
// themselves (global stores) cost +81 us: a producer's constant-vmcnt wait three steps
// later must also cover its write-through stores, whose acknowledgements are slow
// under the full read stream -- the LDS adds here are not vector-memory operations.
constexpr uint32_t kLgSlots = 4;    // per wave: 1 step being hashed + 3 in flight (36 KiB)
constexpr uint32_t kBsSlots = 16;   // blocks the producers may run ahead of the publisher
constexpr uint32_t kBsOff = 4 * kLgSlots * kLgStepBytes;  // [kBsSlots] acc[8] u64, spare[2] u32, cnt[], gen[]
constexpr uint32_t kLgLds = kBsOff + 80 * kBsSlots;
__device__ __forceinline__ uint64_t *bs_acc(uint8_t *smem, uint32_t s) { return (uint64_t *)(smem + kBsOff + 64u * s); }
__device__ __forceinline__ uint32_t *bs_spare(uint8_t *smem, uint32_t s) {
    return (uint32_t *)(smem + kBsOff + 64u * kBsSlots + 8u * s);
}
__device__ __forceinline__ uint32_t *bs_cnt(uint8_t *smem) { return (uint32_t *)(smem + kBsOff + 72u * kBsSlots); }
__device__ __forceinline__ uint32_t *bs_gen(uint8_t *smem) { return bs_cnt(smem) + kBsSlots; }
constexpr int kDppRowRor8 = 0x128;  // row_ror:8: lane r of a 16-lane row <- lane r ^ 8

// Frame group (unit j of this WG, wave) adds its words to block jb = j / 4's slot.
// A wave takes the 4 units of a block on 4 consecutive steps (unit q = j & 3), so its
// contributions are summed in registers (wacc) and flushed into the block's LDS slot
// once per block, on its q = 3 step: one slot wait, one ds_add per accumulator and one
// count add per wave and block (round 4 did all three on every step: the LDS round
// trips stalled the wave, alone on its SIMD, between its ring waits). The count add is
// not ordered behind the sum adds by a wait: DS instructions of one wave execute in
// issue order, and the publisher reads the sums after it has seen the count.
#ifndef IGGY_LG_FLUSH_PER_BLOCK
#define IGGY_LG_FLUSH_PER_BLOCK 1  // (build knob for a same-box A/B: 0 = one LDS flush per step)
#endif
constexpr bool kLgFlushPerBlock = IGGY_LG_FLUSH_PER_BLOCK != 0;
__device__ __forceinline__ void lg_words(uint8_t *smem, const LgPlan &pl, const LgLane &c, uint64_t b, uint64_t j,
                                         uint32_t wave, int lane, const LgState &st, uint64_t t_start,
                                         uint64_t &wacc, uint32_t &wfirst) {
    const uint64_t jb = j >> 2;
    const uint32_t q = (uint32_t)(j & 3);
    const uint32_t k = 4 * q + wave;  // frame group of the block (frames 128 b - 6 + 8 k ..)
    const uint32_t t = 8 * k + c.fg;
    const uint64_t m = 128 * b + t;
    const bool use = c.l == 0 && t != 127 && m >= 6 && m < pl.Mreg && !pl.nopub;
    uint64_t x = 0, y = 0;
    if (use) {
        const uint64_t v = (st.stored >> 32) | (st.next << 32);
        const uint64_t sec = q == 0 ? c.wsec[0] : q == 1 ? c.wsec[1] : q == 2 ? c.wsec[2] : c.wsec[3];
        y = v;
        x = mul32x32(v ^ sec);
    }
    wacc += x + dpp64<kDppRowRor8>(y);  // lane 8 fg: acc[fg] (x of word fg, y of word fg ^ 1)
    if (q == 0) wfirst = (uint32_t)st.stored;  // (wave 0, lane 0: frame t = 0 of the block)
    if (kLgFlushPerBlock && q != 3) return;
    const uint32_t s = (uint32_t)(jb % kBsSlots), gen = (uint32_t)(jb / kBsSlots);
    while (__hip_atomic_load(&bs_gen(smem)[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != gen) {
        __builtin_amdgcn_s_sleep(1);
        if (rt_now() - t_start > kSpinLimitTicks) return;  // bug guard: the consumer times out
    }
    if (c.l == 0) {
        __hip_atomic_fetch_add(&bs_acc(smem, s)[c.fg], wacc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (wave == 0 && c.fg == 0 && (kLgFlushPerBlock || q == 0)) bs_spare(smem, s)[0] = wfirst;  // frame t = 0: lo32
        if (wave == 3 && c.fg == 7 && q == 3) bs_spare(smem, s)[1] = (uint32_t)(st.stored >> 32);  // t = 127: hi32
    }
    asm volatile("" ::: "memory");  // (compiler order only: the DS adds above issue first)
    if (lane == 0) __hip_atomic_fetch_add(&bs_cnt(smem)[s], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    wacc = 0;
}

// The publisher wave: blocks g, g + np, ... in order, each once its 4 producer waves
// are in: the 8 sums read, the slot zeroed and released, the block record stored.
__device__ __forceinline__ void lg_publisher(uint8_t *smem, const LgPlan &pl, const DecodeScratch &sc,
                                             uint32_t epoch, uint32_t g, uint32_t np, int lane, uint32_t dbg) {
    const uint64_t t_start = rt_now();
    const uint64_t blocks = 2 * pl.nchunks;
    if (g >= blocks) return;
    const uint64_t mine = (blocks - g + np - 1) / np;
    for (uint64_t jb = 0; jb < mine; ++jb) {
        const uint32_t s = (uint32_t)(jb % kBsSlots), gen = (uint32_t)(jb / kBsSlots);
        while (__hip_atomic_load(&bs_cnt(smem)[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) !=
               (kLgFlushPerBlock ? 4u : 16u)) {
            __builtin_amdgcn_s_sleep(1);
            if (rt_now() - t_start > kSpinLimitTicks) return;  // bug guard
        }
        const uint32_t t = (uint32_t)lane & 15;
        const uint64_t a = bs_acc(smem, s)[t >> 1];  // granule t = half (t & 1) of acc[t >> 1]
        const uint32_t first_lo = bs_spare(smem, s)[0], last_hi = bs_spare(smem, s)[1];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane < 8) bs_acc(smem, s)[lane] = 0;
        if (lane == 0) bs_cnt(smem)[s] = 0;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // zeroed before the slot goes back
        if (lane == 0) __hip_atomic_store(&bs_gen(smem)[s], gen + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (!pl.long_cs || pl.nopub) continue;
        const uint64_t b = g + jb * np;
        const uint32_t data = (t & 1) ? (uint32_t)(a >> 32) : (uint32_t)a;
        const uint32_t sp = t < 4 ? (first_lo >> (8 * t)) & 0xffu : t < 8 ? (last_hi >> (8 * (t - 4))) & 0xffu : 0u;
        if (lane < 16)
            __hip_atomic_store(block_rec(sc, b) + t, (uint64_t)data | ((uint64_t)sp << 32) | ((uint64_t)epoch << 40),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((dbg & 512) && b < 2 && lane == 0) ((uint64_t *)(sc.small + 256))[11 + b] = rt_now();
    }
}

// ONE: every frame group is a single full-block step (nbF == 1, ns == 0, i.e.
// 1024 < L <= 1088: the C2 shape), so the step code has no partial-block or
// filler paths. g / np: this WG among the producer WGs.
template <uint32_t SLOTS, bool ONE>
__device__ __forceinline__ void produce_lg(const uint8_t *blob, const LgPlan &pl, uint64_t *frame_pos, uint64_t cap,
                                           const DecodeScratch &sc, uint32_t epoch, uint32_t g, uint32_t np,
                                           uint32_t wave, int lane, uint8_t *smem) {
    const uint64_t t_start = rt_now();
    LgLane c;
    c.l = lane & 7; c.m = c.l >> 1; c.par = c.l & 1; c.fg = (uint32_t)lane >> 3;
    c.poff = 16 * (c.m + 4 * c.par);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        c.s0[q] = kSecretW8[2 * q + c.par + 2 * c.m];
        c.s1[q] = kSecretW8[2 * q + c.par + 2 * c.m + 1];
    }
    c.key0 = kSecretW8[16 + 2 * c.m]; c.key1 = kSecretW8[17 + 2 * c.m];
    c.init0 = c.par ? 0 : kAccInit[2 * c.m]; c.init1 = c.par ? 0 : kAccInit[2 * c.m + 1];
    c.last0 = kSecretLast[2 * c.m]; c.last1 = kSecretLast[2 * c.m + 1];
    c.mrg0 = kSecretMerge[2 * c.m]; c.mrg1 = kSecretMerge[2 * c.m + 1];
#pragma unroll
    for (int q = 0; q < 4; ++q) c.wsec[q] = kSecretW8[4 * q + wave + c.fg];
    // materialise every lane constant here: the hot loop then holds no
    // compiler-tracked load, so its only vmcnt waits are the explicit ones
#pragma unroll
    for (int q = 0; q < 8; ++q) { pin_after_wait(c.s0[q]); pin_after_wait(c.s1[q]); }
    pin_after_wait(c.key0); pin_after_wait(c.key1); pin_after_wait(c.init0); pin_after_wait(c.init1);
    pin_after_wait(c.last0); pin_after_wait(c.last1); pin_after_wait(c.mrg0); pin_after_wait(c.mrg1);
#pragma unroll
    for (int q = 0; q < 4; ++q) pin_after_wait(c.wsec[q]);
    const uint64_t blocks = 2 * pl.nchunks;                // 128-frame blocks (tail blocks hold invalid frames)
    const uint32_t nblk = ONE ? 1u : lg_nsteps(pl);       // steps per frame group
    const bool pos_st = frame_pos && !pl.nopub;            // (ONE form) a position store every step
    if (g >= blocks) return;
    const uint64_t mine = 4 * ((blocks - g + np - 1) / np);  // units of blocks g, g + np, ...
    const uint64_t total = mine * nblk;                   // steps of this wave
    auto unit_of = [&](uint64_t j) -> uint64_t { return 4 * (g + (j >> 2) * np) + (j & 3); };

    LgState st;
    st.a0 = c.init0; st.a1 = c.init1; st.stored = 0; st.next = 0; st.sbad = false; st.sink = 0;
    uint64_t wacc = 0;    // this wave's words of the current block (lg_words)
    uint32_t wfirst = 0;
    // processing cursor (pj, pb) and issue cursor (ij, ib), up to SLOTS steps ahead
    uint64_t pj = 0, ij = 0;
    uint32_t pb = 0, ib = 0;
    auto advance = [&](uint64_t &j, uint32_t &b) {
        if (ONE || ++b == nblk) { b = 0; ++j; }
    };
    const uint32_t ring = wave * (SLOTS * kLgStepBytes);
    uint32_t iss = 0;  // steps issued
    auto issue_next = [&]() {
        if (ij >= mine) return;
        lg_issue<ONE>(blob, pl, c, unit_of(ij), wave, ib, nblk, ring + (iss % SLOTS) * kLgStepBytes);
        advance(ij, ib);
        ++iss;
    };
    // Staggered start: WG group g / 16 issues its first steps (g / 16) * stagger
    // ticks after the kernel starts, so the first blocks -- the ones the serial
    // checksum chain needs first -- are not queued behind the whole chip's first
    // burst of loads.
    {
        const uint32_t stagger = (pl.dbg >> 16) & 0xff;
        const uint64_t until = t_start + (uint64_t)(g >> 4) * stagger;
        while (stagger && rt_now() < until) __builtin_amdgcn_s_sleep(1);
    }
    // every slot holds a step in flight; a slot is refilled as soon as its step has
    // been read into registers, so SLOTS steps stay in flight while one is hashed
    for (uint32_t d = 0; d < SLOTS; ++d) issue_next();
    for (uint64_t k = 0; k < total; ++k) {
        // step k landed; the later steps stay in flight (the last SLOTS-1 steps drain all)
        // steps k+1..k+3 stay in flight; with a position store per step (ONE form) the
        // stores of steps k-4..k-1 were issued after step k's loads too
        if (k + SLOTS <= total) {
            if (ONE && IGGY_LG_POS_EXACT && pos_st) wait_vm_const<kLgLoads * (SLOTS - 1) + SLOTS>();
            else wait_vm_const<kLgLoads * (SLOTS - 1)>();
        }
        else wait_vm_const<0>();
        LgBuf B;
        const uint32_t slot = ring + (k % SLOTS) * kLgStepBytes;
        lg_read(smem, slot, lane, B);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot read out before it is refilled
        if ((pl.dbg & 512) && g == 0 && wave == 0 && lane == 0 && k < 4)
            ((uint64_t *)(sc.small + 256))[13 + k] = rt_now();  // diagnostics: WG 0's first steps landed
        issue_next();  // step k + SLOTS into the slot just read
        const uint64_t u = unit_of(pj);
        if (lg_process<ONE>(pl, c, sc, frame_pos, cap, u, wave, pb, nblk, B, st, lane))
            lg_words(smem, pl, c, g + (pj >> 2) * np, pj, wave, lane, st, t_start, wacc, wfirst);
        advance(pj, pb);
    }
    wait_vm(0);
    if (st.sink == 0x5eed5eedu && pl.N == 0) sc.small[lane] = 1;  // never true (N >= 1); keeps `sink` live
}

#ifndef IGGY_LG_NPFIT
#define IGGY_LG_NPFIT 1  // (build knob for a same-box A/B: 0 = every producer WG sweeps)
#endif
__device__ __forceinline__ uint32_t lg_sweep_wgs(uint64_t blocks, uint32_t np) {
    if (!IGGY_LG_NPFIT || np < 16) return np;
    uint32_t best = np;
    uint64_t best_cost = (blocks + np - 1) / np * np;  // block slots of ceil(blocks / n) windows
    for (uint32_t n = np - 1; n >= np - np / 16; --n) {
        const uint64_t cost = (blocks + n - 1) / n * n;
        if (cost < best_cost) { best = n; best_cost = cost; }
    }
    return best;
}

constexpr uint32_t kUniformLds = kLgLds > kXchOff + kXchBytes ? kLgLds : kXchOff + kXchBytes;  // dynamic LDS
static_assert(kConsumerLds <= kLgLds && kConsumerLds <= kLdsBytes, "consumer WG fits either grid's LDS");
static_assert(kUniformLds <= 160 * 1024, "LDS budget");

// ------------------------------------------------------------- consumer
// diagnostics (dbg bit 512): s_memrealtime stamps (100 MHz) of the consumer's
// progress in sc.small[256..], read back with iggy_codec_debug_read:
// [0] consumer start, [1] batch 0 staged, [2 + bi/8] batch bi (bi % 8 == 0),
// [11], [12] blocks 0, 1 published, [13 + k] WG 0 wave 0's step k landed (k < 4),
// [20] chain done, [21] all producers exited, [22] latest producer exit,
// [23 + bi/8] batch bi fully staged by its gatherer (bi % 8 == 0).
__device__ __forceinline__ void dbg_stamp(const DecodeScratch &sc, uint32_t dbg, int idx) {
    if (dbg & 512) ((uint64_t *)(sc.small + 256))[idx] = rt_now();
}

__device__ __forceinline__ uint64_t chain_batches(const UPlan &pl) {
    return ((pl.nb >> 1) + 1 + kBatch - 1) / kBatch;  // chunks 0 .. nb/2 hold blocks 0 .. nb
}

typedef uint32_t g4 __attribute__((ext_vector_type(4)));
constexpr int kAuxSc1 = 16;  // buffer-load cache policy: sc1 (agent-coherent, as an agent-scope atomic load)

// Gatherer wave gw (0..kGatherWaves-1) of the consumer WG: batches gw, gw + kGatherWaves, ...
// Lane c of a batch loads the block records of blocks 2c and 2c + 1 (256 B) and
// stages their 16 accumulator sums, completed by the blocks' last words.
__device__ __forceinline__ void gather(const uint8_t *blob, const UPlan &pl, const DecodeScratch &sc,
                                       uint32_t epoch, uint32_t gw, uint32_t ngw, uint8_t *smem,
                                       uint64_t t_start, uint32_t dbg) {
    const int lane = threadIdx.x & 63;
    ChainCtl *ctl = (ChainCtl *)(smem + kCtlOff);
    uint64_t *ring = (uint64_t *)smem;
    const uint64_t need = (pl.nb >> 1) + 1;
    const uint64_t nbatch = chain_batches(pl);
    auto give_up = [&]() -> bool {
        return __hip_atomic_load(&ctl->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0 ||
               rt_now() - t_start > kSpinLimitTicks;
    };
    const uint32_t tag = epoch << 8;  // high dword of a granule: spare8 | tag24 << 8
    uint64_t npass = 0, npoll = 0, twait = 0;  // diagnostics (dbg 512; npoll stays 0)
    for (uint64_t bi = gw; bi < nbatch; bi += ngw) {
        const uint32_t slot = (uint32_t)(bi % kRing);
        bool abort = false;
        const uint64_t tw0 = rt_now();
        while (bi >= kRing && (uint64_t)__hip_atomic_load(&ctl->consumed, __ATOMIC_ACQUIRE,
                                                          __HIP_MEMORY_SCOPE_WORKGROUP) + kRing <= bi) {
            __builtin_amdgcn_s_sleep(1);
            if (give_up()) { abort = true; break; }
        }
        if (dbg & 512) twait += rt_now() - tw0;  // ring-full wait
        const uint64_t cbase = bi * kBatch;
        const uint64_t c = cbase + lane;
        const bool live = c < need && c < pl.nchunks;
        const bool has_next = live && c + 1 < pl.nchunks;
        // coherent 16-B loads (sc1: past this XCD's L1, as agent-scope atomic loads);
        // out-of-range lanes read zeros
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)block_rec(sc, 2 * cbase), 0,
            (int)min<uint64_t>((sc.max_chunks - cbase) * kChunkSumWords * 8, 1u << 30), 0x00020000);
        // Progressive staging: every pass loads the 32 tagged granules of each chunk
        // (and lane 63 the next batch's first block's 4 spare-carrying granules),
        // stages the chunks whose tags (and the next chunk's) all match, and publishes
        // how many LEADING chunks of the batch are staged, so the chain starts on
        // chunk 0 as soon as its 2 blocks are published.
        bool staged = !live;
        uint32_t published = 0;
        for (bool first = true; !abort; first = false) {
            if (dbg & 512) ++npass;
            if (!first) {  // the next full pass after a short sleep (a separate 2-granule poll
                           // first cost one more round trip per staged batch)
                __builtin_amdgcn_s_sleep(1);
                if (give_up()) { abort = true; break; }
            }
            g4 r[16];
#pragma unroll
            for (int q = 0; q < 16; ++q)
                r[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)lane * 256u + 16u * q, 0, kAuxSc1);
            g4 nx0 = {0, 0, 0, 0}, nx1 = {0, 0, 0, 0};
            if (lane == 63 && has_next) {  // the next batch's first chunk, block 2(c + 1)
                nx0 = __builtin_amdgcn_raw_buffer_load_b128(rs, 64u * 256u, 0, kAuxSc1);
                nx1 = __builtin_amdgcn_raw_buffer_load_b128(rs, 64u * 256u + 16u, 0, kAuxSc1);
            }
            bool own = true;
#pragma unroll
            for (int q = 0; q < 16; ++q) own &= ((r[q].y & ~0xffu) == tag) & ((r[q].w & ~0xffu) == tag);
            // spare bytes: granules 0-3 lo32(cs of the block's first frame), 4-7 hi32(cs of its last)
            auto spare = [](const g4 &p, const g4 &q2) -> uint32_t {
                return (p.y & 0xff) | (p.w & 0xff) << 8 | (q2.y & 0xff) << 16 | (q2.w & 0xff) << 24;
            };
            const uint32_t first0 = spare(r[0], r[1]), last0 = spare(r[2], r[3]);
            const uint32_t first1 = spare(r[8], r[9]), last1 = spare(r[10], r[11]);
            // the next chunk's first block's first frame: from lane c + 1 (or the loads above)
            const bool nx_ok = ((nx0.y & ~0xffu) == tag) & ((nx0.w & ~0xffu) == tag) &
                               ((nx1.y & ~0xffu) == tag) & ((nx1.w & ~0xffu) == tag);
            uint32_t next_first = (uint32_t)__shfl_down((int)first0, 1);
            bool next_ok = __shfl_down((int)own, 1) != 0;
            if (lane == 63) { next_first = spare(nx0, nx1); next_ok = nx_ok; }
            const bool ok = own && (!has_next || next_ok);
            if (!staged && ok) {
                uint64_t B[16];
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    B[t] = (uint64_t)r[t].x | ((uint64_t)r[t].z << 32);
                    B[8 + t] = (uint64_t)r[8 + t].x | ((uint64_t)r[8 + t].z << 32);
                }
                // the blocks' last words m = 256c + 127, 256c + 255: j = 7 of stripe 15
                auto last_word = [&](uint64_t m, uint32_t hi32, uint32_t lo32, uint64_t &b6, uint64_t &b7) {
                    if (m >= 6 && m < pl.Mreg) {
                        const uint64_t v = (uint64_t)hi32 | ((uint64_t)lo32 << 32);
                        b6 += v;
                        b7 += mul32x32(v ^ kSecretW8[15 + 7]);
                    }
                };
                last_word(256 * c + 127, last0, first1, B[6], B[7]);
                last_word(256 * c + 255, last1, has_next ? next_first : 0u, B[14], B[15]);
                uint64_t *dst = ring + ((uint64_t)slot * kBatch + lane) * 16;
#pragma unroll
                for (int t = 0; t < 16; ++t) dst[t] = B[t];
                staged = true;
            }
            const uint64_t notyet = __ballot(!staged);
            const uint32_t k = notyet ? (uint32_t)__builtin_ctzll(notyet) : 64u;
            if (k > published) {  // the release orders this wave's ring writes before the count
                if (lane == 0)
                    __hip_atomic_store(&ctl->staged[slot], (uint32_t)((bi + 1) << 7) | k, __ATOMIC_RELEASE,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                published = k;
            }
            if (k == 64) {
                if (lane == 0 && (bi & 7) == 0) dbg_stamp(sc, dbg, 23 + (int)(bi >> 3));
                break;
            }
            if (give_up()) abort = true;
        }
        if (abort) {
            if (lane == 0) __hip_atomic_store(&ctl->abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            return;
        }
    }
    if ((dbg & 512) && lane == 0) {
        uint64_t *d = (uint64_t *)(sc.small + 512) + 4 * gw;
        d[0] = npass; d[1] = npoll; d[2] = twait; d[3] = rt_now() - t_start;
    }
}

// The consumer WG (block 0): wave 0 runs the serial batch-checksum chain
// (batch.rs:439-459 / 474-505) and the precedence resolution of
// decode_batch_slice_with (batch.rs:395-421); waves 1..4 gather its inputs.
template <bool VERIFY>
__device__ __forceinline__ void consumer(const uint8_t *body, const HeaderInfo &hi, const UPlan &pl,
                                         iggy_decode_result *result, const DecodeScratch &sc,
                                         uint32_t epoch, uint32_t nwaves_prod, uint32_t wave,
                                         uint8_t *smem, uint32_t dbg, uint64_t pos_epilogue_cap) {
    const int lane = threadIdx.x & 63;
    const uint8_t *blob = body + kHdr;

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
                const uint64_t w[5] = {hi.h.partition_id, hi.h.base_offset, hi.h.base_timestamp,
                                       hi.h.origin_timestamp, hi.h.batch_length};
                for (int i = 0; i < 5; ++i) st64_any(s + 8 * i, w[i]);
                *(u32_ua *)(s + 40) = hi.h.message_count;
                computed = xxh3_64_lane(s, 44);
                if (computed != hi.h.batch_checksum) {
                    kind = IGGY_ERR_INVALID_BATCH_CHECKSUM; reason = 0;
                    a = hi.h.batch_checksum; b = computed; c = hi.h.base_offset;
                }
            }
        }
        if (lane == 0) write_result(result, hi, kind, reason, a, b, c, 0, computed, 1, status, 0);
        return;
    }

    const uint64_t t_start = rt_now();
    if (dbg & 4096) {  // diagnostics: give up at once, as a timed-out wait does (producers run on)
        if (wave == 0 && lane == 0) write_result(result, hi, IGGY_ERR_TIMEOUT, 0, 0, 0, 0, 0, 0, 1, kStatusDone, 0);
        return;
    }
    if (wave == 0 && lane == 0) dbg_stamp(sc, dbg, 0);
    bool timed_out = false;
    uint64_t computed = 0;
    const bool chain = VERIFY && pl.long_cs && !(dbg & 1);
    if (chain) {
        if (threadIdx.x < sizeof(ChainCtl) / 4) ((uint32_t *)(smem + kCtlOff))[threadIdx.x] = 0;
        __syncthreads();
    }
    if (wave != 0) {  // gatherer waves feed the chain wave through the LDS ring
        if (chain && wave <= kGatherWaves) gather(blob, pl, sc, epoch, wave - 1, kGatherWaves, smem, t_start, dbg);
        return;
    }
    if (chain) {
        __builtin_amdgcn_s_setprio(3);  // a gatherer shares this wave's SIMD: the chain issues first
        ChainCtl *ctl = (ChainCtl *)(smem + kCtlOff);
        const uint64_t *ring = (const uint64_t *)smem;
        const int j = lane & 7;
        uint64_t acc = kAccInit[j];
        const uint64_t key = kSecretW8[16 + j];
        const uint32_t klo = (uint32_t)key, khi = (uint32_t)(key >> 32);
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
        // the last stripe's stored checksums (frames N-8 .. N-1), loaded now: after the
        // chain they would cost one more memory round trip on the decode's critical path
        const uint64_t last_v = ld64_any(blob + (pl.N - 8 + j) * pl.S);
        // y = acc + (sum of the current block); block b >= 1: y = scramble(y) + S_b.
        // Only blocks 0 .. nb-1 are scrambled: the partial block nb just adds.
        const uint64_t nbatch = chain_batches(pl);
        uint64_t y = acc;
        for (uint64_t bi = 0; bi < nbatch && !timed_out; ++bi) {
            const uint32_t slot = (uint32_t)(bi % kRing);
            const uint64_t b0 = 2 * kBatch * bi;
            uint64_t bend = b0 + 2 * kBatch;
            if (bend > pl.nb + 1) bend = pl.nb + 1;
            // block b of this batch at src[8 * (b - b0)]
            const uint64_t *src = ring + (uint64_t)slot * (kBatch * 16) + j;
            const uint32_t kend = (uint32_t)(bend - b0);
            uint32_t k = 0;
            uint64_t va[16], vb[16];
            auto ld16 = [&](uint64_t *v, uint32_t k0) {
#pragma unroll
                for (int x = 0; x < 16; ++x) v[x] = src[8 * (k0 + x)];
            };
            auto run16 = [&](const uint64_t *v) {
#pragma unroll
                for (int x = 0; x < 16; ++x) y = chain_step(y, v[x], klo, khi);
            };
            while (k < kend) {
                // the gatherer stages the batch's chunks progressively (2 blocks each)
                uint32_t avail = 0;
                while (true) {
                    const uint32_t w = __hip_atomic_load(&ctl->staged[slot], __ATOMIC_ACQUIRE,
                                                         __HIP_MEMORY_SCOPE_WORKGROUP);
                    avail = (w >> 7) == (uint32_t)(bi + 1) ? 2 * (w & 127u) : 0u;
                    if (avail > kend) avail = kend;
                    if (avail > k) break;
                    __builtin_amdgcn_s_sleep(1);
                    if (__hip_atomic_load(&ctl->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) ||
                        rt_now() - t_start > kSpinLimitTicks) {
                        timed_out = true;
                        break;
                    }
                }
                if (timed_out) break;
                if (k == 0 && (dbg & 512) && lane == 0 && (bi & 7) == 0)
                    dbg_stamp(sc, dbg, bi == 0 ? 1 : 2 + (int)(bi >> 3));
                if (bi == 0 && k == 0) { y += src[0]; k = 1; }
                if (IGGY_CHAIN_ASM && k + 16 <= avail) {  // 16-step groups in asm (chain_span)
                    typedef __attribute__((address_space(3))) const uint64_t lds_u64;
                    const uint32_t n16 = (avail - k) >> 4;
                    y = chain_span(y, (uint32_t)(uintptr_t)(lds_u64 *)(src + 8 * k), n16, klo, khi);
                    k += 16 * n16;
                }
                // groups of 16 blocks, the next group's LDS reads in flight during this group
                if (k + 16 <= avail) {
                    ld16(va, k);
                    while (true) {
                        const bool more = k + 32 <= avail;
                        if (more) ld16(vb, k + 16);
                        run16(va);
                        k += 16;
                        if (!more) break;
                        const bool more2 = k + 32 <= avail;
                        if (more2) ld16(va, k + 16);
                        run16(vb);
                        k += 16;
                        if (!more2) break;
                    }
                }
                for (; k < avail; ++k) y = chain_step(y, src[8 * k], klo, khi);
            }
            if (timed_out) break;
            __hip_atomic_store(&ctl->consumed, (uint32_t)(bi + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (timed_out) {
            __hip_atomic_store(&ctl->abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
            acc = y;
            // last stripe = stored checksums of frames N-8 .. N-1 (secret offset 121)
            const uint64_t v = last_v;
            acc += __shfl_xor(v, 1);
            acc += mul32x32(v ^ kSecretLast[j]);
            uint64_t a[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) a[i] = __shfl(acc, i);
            uint64_t r = pl.n * P64_1;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                r += fold64(a[2 * i] ^ Secret::w(11 + 16 * i), a[2 * i + 1] ^ Secret::w(19 + 16 * i));
            computed = avalanche(r);
            if (lane == 0) dbg_stamp(sc, dbg, 20);
        }
    } else if (VERIFY && !pl.long_cs) {
        // short checksum input (N <= 24): hash it directly
        if (lane == 0) {
            uint8_t *s = sc.small;
            const uint64_t w[5] = {hi.h.partition_id, hi.h.base_offset, hi.h.base_timestamp,
                                   hi.h.origin_timestamp, hi.h.batch_length};
            for (int i = 0; i < 5; ++i) st64_any(s + 8 * i, w[i]);
            *(u32_ua *)(s + 40) = hi.h.message_count;
            for (uint64_t i = 0; i < pl.N; ++i) st64_any(s + 44 + 8 * i, ld64_any(blob + i * pl.S));
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
    // every producer wave done => their stores / atomics are visible
    while (!timed_out &&
           __hip_atomic_load(sc.exited, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != nwaves_prod) {
        __builtin_amdgcn_s_sleep(4);
        if (rt_now() - t_start > kSpinLimitTicks) timed_out = true;
    }
    if (lane != 0) return;
    dbg_stamp(sc, dbg, 21);
    if (timed_out) {
        write_result(result, hi, IGGY_ERR_TIMEOUT, 0, 0, 0, 0, 0, 0, 1, kStatusDone, 0);
        return;  // the sync words are re-armed by this decode's general kernel (k_decode_general)
    }
    uint64_t fb_enc = __hip_atomic_load(sc.first_bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tail_bad && fb_enc == 0) fb_enc = ~(pl.N - 1);  // producers only report smaller indices
    const uint64_t sf_enc = __hip_atomic_load(sc.spec_fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool has_fb = fb_enc != 0, has_sf = sf_enc != 0;
    const uint64_t fb = ~fb_enc, sf = ~sf_enc;
    uint32_t kind = IGGY_OK, reason = 0, status = kStatusDone;
    uint64_t a = 0, b = 0, c = 0, nframes = pl.N;
    auto msg_err = [&](uint64_t idx) {
        const uint64_t slot = (idx + 6) >> 3;  // the frame's 8-frame group
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
    // frame positions the producers left to k_decode_general (kPosEpilogue): the walked
    // frames' (entries past frame_count are unspecified, include/iggy_codec.h)
    const uint64_t npos = nframes < pos_epilogue_cap ? nframes : pos_epilogue_cap;
    if (status == kStatusDone && npos) {
        __hip_atomic_store(&sc.gmisc[kPosStrideWord], pl.S, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&sc.gmisc[kPosCountWord], npos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // re-arm the scratch for the next call on this stream
    __hip_atomic_store(sc.exited, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(sc.first_bad, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(sc.spec_fail, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------- kernel
// Frame positions of a lane-group decode (i * S). Stored from the producer waves inside
// their step loop (8 B per frame, 8 lanes per step) they cost ~17 us of a C2 decode's
// producer phase: a store behind a step's ring loads lengthens the constant-vmcnt wait
// of the steps after it (same box, chain off: 0.211 -> 0.194 ms without them,
// scripts/diag_decode.py DIAG_NOPOS). Mode 2 (default): each producer wave stores a
// contiguous share of them after its loop (coalesced 512-B wave stores, no ring wait
// left to lengthen), beside the chain's tail. Mode 1: the next kernel of the decode
// (k_decode_general, which otherwise returns at once) writes them with the whole chip.
// Mode 0: the round-4 per-step stores.
#ifndef IGGY_POS_MODE
#define IGGY_POS_MODE 2  // (build knob for a same-box A/B)
#endif
constexpr bool kPosEpilogue = IGGY_POS_MODE == 1;
constexpr bool kPosTail = IGGY_POS_MODE == 2;
template <bool VERIFY>
__device__ __forceinline__ bool uniform_uses_lg(const UPlan &pl, uint32_t dbg) {
    return VERIFY && pl.state == 0 && pl.long_frames && !(dbg & 32);  // dbg bit 32: force the LDS form
}

// One persistent grid of one WG per CU (256 threads, up to 160 KiB LDS): block 0
// is the consumer WG (chain wave + gatherers), blocks 1.. the producers, either
// lane-group (long frames under Verify) or LDS-staged (short frames, LayoutOnly).
// Producers never wait for the consumer, so a grid that is only partly resident
// (or kernels serialised by a profiler) still completes.
template <bool VERIFY>
__global__ __launch_bounds__(kUniformThreads, 1) void k_decode_uniform(const uint8_t *__restrict__ body, uint64_t len,
                                                           uint64_t *frame_pos, uint64_t cap,
                                                           iggy_decode_result *result, DecodeScratch sc,
                                                           uint32_t epoch, uint32_t allow_unaligned,
                                                           uint32_t dbg) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    dbg &= kDiagMask;  // product build: no ablation bit survives
    const int lane = threadIdx.x & 63;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // the previous decode's general kernel has completed (stream order): re-arm its
        // barrier, registration and first-bad words for this decode's general kernel
        __hip_atomic_store(&sc.gbar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&sc.gbar[2], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&sc.gbar[3], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&sc.gmisc[2], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&sc.gmisc[kPosCountWord], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (blockIdx.x == 0 && threadIdx.x < kBar2Words)
        __hip_atomic_store(&sc.gbar2[32 * threadIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    HeaderInfo hi;
    parse_header(body, len, hi);
    UPlan pl;
    make_plan(hi, body + kHdr, len, VERIFY, sc.max_chunks, allow_unaligned != 0, pl);
    const bool lg = uniform_uses_lg<VERIFY>(pl, dbg);
    if (lg) pl.tail_unsafe = false;  // every lane-group load stays inside its frame
    const uint32_t nprod = gridDim.x - 1;
    // lane-group decodes leave the frame positions to k_decode_general (kPosEpilogue)
    const uint64_t pos_epi = (kPosEpilogue && lg && frame_pos) ? cap : 0;
    if (blockIdx.x == 0) {
        consumer<VERIFY>(body, hi, pl, result, sc, epoch, 4 * nprod, wave, smem, dbg, pos_epi);
        return;
    }
    if (pl.state != 0) return;
    const uint8_t *blob = body + kHdr;
    const uint32_t g = blockIdx.x - 1;
    if (VERIFY && lg) {
        pl.nt = (dbg & 64) != 0;
        pl.nopub = (dbg & 128) != 0;
        LgPlan lp = lg_plan(pl);
        lp.dbg = dbg;
        if (threadIdx.x < 8 * kBsSlots) bs_acc(smem, 0)[threadIdx.x] = 0;  // block sums, counters, generations
        if (threadIdx.x < 2 * kBsSlots) bs_cnt(smem)[threadIdx.x] = 0;
        __syncthreads();
        // producer WGs that sweep the blocks: the count in [nprod - nprod/16, nprod] whose
        // block windows waste the least (a last, partly filled window of blocks takes a
        // whole block time while most WGs idle: C2's 8 194 blocks on 254 WGs leave 66 in
        // it, on 249 WGs 226); the others only store their share of the positions
        const uint32_t npe = lg_sweep_wgs(2 * lp.nchunks, nprod);
        if (g < npe) {
            if (wave == 4) {  // the WG's publisher
                lg_publisher(smem, lp, sc, epoch, g, npe, lane, dbg);
                return;
            }
            uint64_t *fp = IGGY_POS_MODE ? nullptr : frame_pos;
            if (lp.nbF == 1 && lp.ns == 0)
                produce_lg<kLgSlots, true>(blob, lp, fp, cap, sc, epoch, g, npe, wave, lane, smem);
            else
                produce_lg<kLgSlots, false>(blob, lp, fp, cap, sc, epoch, g, npe, wave, lane, smem);
        } else if (wave == 4) {
            return;
        }
        if (kPosTail && frame_pos) {  // this wave's contiguous share of the positions
            const uint64_t n = pl.N < cap ? pl.N : cap;
            const uint64_t nw = 4ull * nprod, per = ((n + nw - 1) / nw + 63) & ~63ull;
            const uint64_t i0 = (4ull * g + wave) * per, i1 = i0 + per < n ? i0 + per : n;
            for (uint64_t i = i0 + (uint64_t)lane; i < i1; i += 64) frame_pos[i] = i * pl.S;
        }
        // Exit count: relaxed after this wave's own vmcnt drain. Everything the
        // consumer reads after it (first_bad, spec_fail, errslot, unit sums) was
        // written by device atomics or sc1 stores and is read with sc1 loads, so no
        // release is needed -- and a release here (buffer_wbl2 per wave, 1020 of
        // them at the kernel tail) measured +40 us per C2 decode (scripts/lg_micro.hip).
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if ((dbg & 512) && lane == 0)
            atomicMax((unsigned long long *)(sc.small + 256 + 8 * 22), (unsigned long long)rt_now());
        if (lane == 0) __hip_atomic_fetch_add(sc.exited, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    if (threadIdx.x < 4) xch_flags(smem)[threadIdx.x] = 0;  // the wave pairs' exchange flags
    __syncthreads();
    if (wave >= 4) return;  // the LDS-staged producers are waves 0-3
    pl.nt = (dbg & 16) != 0;
    if (VERIFY && pl.long_frames)
        produce<8, 4, 3, VERIFY>(blob, pl, frame_pos, cap, sc, epoch, g, nprod, wave, lane, smem, dbg);
    else
        produce<16, 2, 1, VERIFY>(blob, pl, frame_pos, cap, sc, epoch, g, nprod, wave, lane, smem, dbg);
}

template __global__ void k_decode_uniform<true>(const uint8_t *__restrict__, uint64_t, uint64_t *, uint64_t,
                                                iggy_decode_result *, DecodeScratch, uint32_t, uint32_t, uint32_t);
template __global__ void k_decode_uniform<false>(const uint8_t *__restrict__, uint64_t, uint64_t *, uint64_t,
                                                 iggy_decode_result *, DecodeScratch, uint32_t, uint32_t, uint32_t);

}  // namespace iggy

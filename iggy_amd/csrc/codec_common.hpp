// codec_common.hpp — shared device-side definitions of the batch codec.
//
// Wire layout (core/binary_protocol/src/batch.rs:18-30, 36-73, 228-275):
//   batch  = [256 B header][frame_0 .. frame_{n-1}]
//   header = partition_id u64 | base_offset u64 | base_timestamp u64 |
//            origin_timestamp u64 | batch_length u64 | batch_checksum u64 |
//            message_count u32 | 204 reserved zero bytes
//   frame  = checksum u64 | id u128 | offset_delta u32 | timestamp_delta u32 |
//            user_headers_length u32 | payload_length u32 | reserved u64 |
//            payload | user_headers
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/iggy_codec.h"
#include "xxh3_device.hpp"

namespace iggy {

constexpr uint32_t kHdr = 256;
constexpr uint32_t kFrameHdr = 48;
constexpr uint64_t kNone = 0;  // "no index" in the max-encoded slots below

// Ablation / diagnostic bits (loads only, no chain, forced kernel forms, progress
// stamps) exist only in the separate diagnostic build (`make diag` ->
// libiggy_codec_diag.so, -DIGGY_CODEC_DIAG). In the product library the mask is
// zero, so every such branch is compiled out and nothing can switch verification off.
#ifdef IGGY_CODEC_DIAG
constexpr uint32_t kDiagMask = 0xFFFFFFFFu;
#else
constexpr uint32_t kDiagMask = 0u;
#endif

// Device-side status values in iggy_decode_result::status
constexpr uint32_t kStatusDone = 0;
constexpr uint32_t kStatusNeedGeneral = 1;
constexpr uint32_t kStatusPending = 2;
// words of the decode's misc scratch (DecodeScratch::gmisc == GeneralScratch::misc): the
// stride and count of the frame positions a lane-group uniform decode leaves to
// k_decode_general (decode_uniform.hip kPosEpilogue); the count is re-armed (zeroed) by
// every uniform launch
constexpr uint32_t kPosStrideWord = 8, kPosCountWord = 9;

// Wave-uniform header parse shared by every role of every decode kernel.
struct HeaderInfo {
    iggy_batch_header h;
    uint32_t err_kind, err_reason;
    uint64_t ea, eb, ec;
    uint64_t blob_len;
};

__device__ inline void set_err(HeaderInfo &hi, uint32_t k, uint32_t r, uint64_t a, uint64_t b,
                               uint64_t c) {
    hi.err_kind = k; hi.err_reason = r; hi.ea = a; hi.eb = b; hi.ec = c;
}

// BatchHeader::decode (batch.rs:98-134) + the EOF check of
// decode_batch_slice_with (batch.rs:397-403). Every lane of the calling wave
// must call it (the reserved-byte scan is wave-parallel).
__device__ inline void parse_header(const uint8_t *body, uint64_t len, HeaderInfo &hi) {
    hi.err_kind = IGGY_OK; hi.err_reason = 0; hi.ea = hi.eb = hi.ec = 0; hi.blob_len = 0;
    hi.h = iggy_batch_header{};
    if (len < kHdr) {
        set_err(hi, IGGY_ERR_UNEXPECTED_EOF, 0, 0, kHdr, len);
        return;
    }
    uint64_t batch_length = ld64_any(body + 32);
    if (batch_length < kHdr) {
        set_err(hi, IGGY_ERR_VALIDATION, IGGY_V_BATCH_LENGTH_SHORT, 0, 0, 0);
        return;
    }
    // bytes 52..255 must be zero: 51 dwords, one per lane
    const int lane = threadIdx.x & 63;
    uint32_t w = (lane < 51) ? ld32_any(body + 52 + 4 * lane) : 0u;
    if (__ballot(w != 0) != 0ull) {
        set_err(hi, IGGY_ERR_VALIDATION, IGGY_V_BATCH_RESERVED, 0, 0, 0);
        return;
    }
    hi.h.partition_id = ld64_any(body + 0);
    hi.h.base_offset = ld64_any(body + 8);
    hi.h.base_timestamp = ld64_any(body + 16);
    hi.h.origin_timestamp = ld64_any(body + 24);
    hi.h.batch_length = batch_length;
    hi.h.batch_checksum = ld64_any(body + 40);
    hi.h.message_count = ld32_any(body + 48);
    if (len < batch_length) {
        set_err(hi, IGGY_ERR_UNEXPECTED_EOF, 0, 0, batch_length, len);
        return;
    }
    hi.blob_len = batch_length - kHdr;
}

__device__ inline void write_result(iggy_decode_result *r, const HeaderInfo &hi, uint32_t kind,
                                    uint32_t reason, uint64_t a, uint64_t b, uint64_t c,
                                    uint64_t nframes, uint64_t computed, uint32_t path,
                                    uint32_t status, uint64_t covered) {
    r->header = hi.h;
    r->error.kind = kind;
    r->error.reason = reason;
    r->error.a = a;
    r->error.b = b;
    r->error.c = c;
    r->frame_count = nframes;
    r->computed_checksum = computed;
    r->path = path;
    r->status = status;
    r->covered = covered;
}

__device__ __forceinline__ uint64_t sat_add(uint64_t a, uint64_t b) {
    uint64_t s = a + b;
    return s < a ? ~0ull : s;
}

// bounded spin support: s_memrealtime ticks at 100 MHz on gfx950
__device__ __forceinline__ uint64_t rt_now() { return __builtin_amdgcn_s_memrealtime(); }
constexpr uint64_t kSpinLimitTicks = 100000000ull * 4;  // 4 s: a bug guard, never a timing knob

// LDS-DMA (global_load_lds_dwordx4) issue and the constant vmcnt wait that goes with it
// M0 carries the LDS destination; it is declared clobbered (the compiler
// re-materialises M0 itself wherever it needs it) instead of saved/restored.
__device__ __forceinline__ void glds16(const void *gsrc, uint32_t lds_addr, bool nt = false) {
    if (nt) {
        asm volatile(
            "s_mov_b32 m0, %1\n\t"
            "s_nop 0\n\t"
            "global_load_lds_dwordx4 %0, off nt"
            :
            : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_addr))
            : "memory", "m0");
        return;
    }
    asm volatile(
        "s_mov_b32 m0, %1\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %0, off"
        :
        : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_addr))
        : "memory", "m0");
}
// gsrc + OFF -> lds_addr. The instruction offset is added to the LDS address too
// (LDS_ADDR = M0 + inst_offset + 16 * lane), so M0 gets lds_addr - OFF.
// (IGGY_LG_NT: the non-temporal policy on these loads, a build knob for a same-box A/B)
#ifndef IGGY_LG_NT
#define IGGY_LG_NT 0
#endif
#if IGGY_LG_NT
#define IGGY_LG_NT_SUFFIX " nt"
#else
#define IGGY_LG_NT_SUFFIX ""
#endif
template <int OFF>
__device__ __forceinline__ void glds16o(const void *gsrc, uint32_t lds_addr) {
    asm volatile(
        "s_mov_b32 m0, %1\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %0, off offset:%2" IGGY_LG_NT_SUFFIX
        :
        : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_addr - OFF)), "i"(OFF)
        : "memory", "m0");
}
template <int N>
__device__ __forceinline__ void wait_vm_const() {
    static_assert(N >= 0 && N <= 63, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// lane-group XXH3 helpers (decode_uniform / decode_general / encode): DPP quad_perm
// and ds_swizzle moves of a 64-bit value, and one 16-B stripe-pair piece
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

}  // namespace iggy

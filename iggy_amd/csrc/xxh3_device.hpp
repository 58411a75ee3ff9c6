// xxh3_device.hpp — XXH3-64 (seed 0, default secret) building blocks for gfx950.
//
// The reference hashes with twox-hash 2.1.3 `XxHash3_64` (Cargo.lock:13579-13586,
// call sites core/binary_protocol/src/batch.rs:440-485,
// requests/messages/send_messages.rs:162). Everything here is integer work:
// 32x32->64 multiplies (v_mad_u64_u32), 64x64->128 folds, xors and shifts.
// The long-input form is split into its two parallel-friendly halves:
//   * per 64-B stripe accumulation (sums commute inside a 1024-B block), and
//   * the per-block scramble chain (serial),
// so kernels can accumulate stripes from any lane/wave mapping and run the
// scramble chain where the data is complete.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace iggy {

constexpr uint32_t P32_1 = 0x9E3779B1u;
constexpr uint32_t P32_2 = 0x85EBCA77u;
constexpr uint32_t P32_3 = 0xC2B2AE3Du;
constexpr uint64_t P64_1 = 0x9E3779B185EBCA87ull;
constexpr uint64_t P64_2 = 0xC2B2AE3D27D4EB4Full;
constexpr uint64_t P64_3 = 0x165667B19E3779F9ull;
constexpr uint64_t P64_4 = 0x85EBCA77C2B2AE63ull;
constexpr uint64_t P64_5 = 0x27D4EB2F165667C5ull;
constexpr uint64_t PMX1 = 0x165667919E3779F9ull;
constexpr uint64_t PMX2 = 0x9FB21C651E98DF25ull;

// Default 192-byte secret as little-endian u64 words read at ANY byte offset.
// Evaluated at compile time whenever the offset is a constant (unrolled code).
struct Secret {
    static constexpr uint8_t b[192 + 8] = {
        0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c, 0xf7, 0x21, 0xad, 0x1c,
        0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb, 0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3, 0x67, 0x1f,
        0xcb, 0x79, 0xe6, 0x4e, 0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc, 0xff, 0x72, 0x21,
        0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6, 0x81, 0x3a, 0x26, 0x4c,
        0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb, 0x88, 0xd0, 0x65, 0x8b, 0x1b, 0x53, 0x2e, 0xa3,
        0x71, 0x64, 0x48, 0x97, 0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19, 0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8,
        0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9, 0xdc, 0xbb, 0xc7, 0xc7, 0x0b, 0x4f, 0x1d,
        0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31, 0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64,
        0xea, 0xc5, 0xac, 0x83, 0x34, 0xd3, 0xeb, 0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb,
        0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0, 0xda, 0x49, 0xd3, 0x16, 0x55, 0x26, 0x29, 0xd4, 0x68, 0x9e,
        0x2b, 0x16, 0xbe, 0x58, 0x7d, 0x47, 0xa1, 0xfc, 0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce,
        0x45, 0xcb, 0x3a, 0x8f, 0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e,
        0, 0, 0, 0, 0, 0, 0, 0};
    static constexpr __host__ __device__ uint64_t w(int off) {
        uint64_t v = 0;
        for (int i = 7; i >= 0; --i) v = (v << 8) | b[off + i];
        return v;
    }
};

// Aligned secret words (offset = 8*i, i in 0..23) for runtime-indexed lookups
// (per-lane stripe/word positions). Lives in the constant segment.
__constant__ static const uint64_t kSecretW8[24] = {
    Secret::w(0),   Secret::w(8),   Secret::w(16),  Secret::w(24),  Secret::w(32),
    Secret::w(40),  Secret::w(48),  Secret::w(56),  Secret::w(64),  Secret::w(72),
    Secret::w(80),  Secret::w(88),  Secret::w(96),  Secret::w(104), Secret::w(112),
    Secret::w(120), Secret::w(128), Secret::w(136), Secret::w(144), Secret::w(152),
    Secret::w(160), Secret::w(168), Secret::w(176), Secret::w(184)};

// Secret words of the XXH3 "last stripe" (byte offset 121 + 8j, unaligned).
__constant__ static const uint64_t kSecretLast[8] = {
    Secret::w(121), Secret::w(129), Secret::w(137), Secret::w(145),
    Secret::w(153), Secret::w(161), Secret::w(169), Secret::w(177)};
// Secret words of the XXH3 long-path merge: acc[2i] ^ w(11 + 16i), acc[2i+1] ^ w(19 + 16i).
__constant__ static const uint64_t kSecretMerge[8] = {
    Secret::w(11), Secret::w(19), Secret::w(27), Secret::w(35),
    Secret::w(43), Secret::w(51), Secret::w(59), Secret::w(67)};
// Initial accumulators of the XXH3 long path.
__constant__ static const uint64_t kAccInit[8] = {P32_3, P64_1, P64_2, P64_3,
                                                  P64_4, P32_2, P64_5, P32_1};

// Secret word of word m = 128 b + 64 half + lane of a 1024-B block (any b): it depends
// on (half, lane) only -- (m >> 3) & 15 = 8 half + (lane >> 3), m & 7 = lane & 7 -- so
// block loops load it once instead of a runtime-indexed table read per block.
__device__ __forceinline__ uint64_t block_word_secret(int half, int lane) {
    return kSecretW8[8 * half + (lane >> 3) + (lane & 7)];
}

__device__ __forceinline__ uint64_t mul32x32(uint64_t k) {
    return (uint64_t)(uint32_t)k * (uint64_t)(uint32_t)(k >> 32);
}
__device__ __forceinline__ uint64_t fold64(uint64_t a, uint64_t b) {
    return (a * b) ^ __umul64hi(a, b);
}
__device__ __forceinline__ uint64_t avalanche(uint64_t h) {
    h ^= h >> 37;
    h *= PMX1;
    h ^= h >> 32;
    return h;
}
__device__ __forceinline__ uint64_t xxh64_avalanche(uint64_t h) {
    h ^= h >> 33; h *= P64_2; h ^= h >> 29; h *= P64_3; h ^= h >> 32;
    return h;
}
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t rrmxmx(uint64_t h, uint64_t len) {
    h ^= rotl64(h, 49) ^ rotl64(h, 24);
    h *= PMX2;
    h ^= (h >> 35) + len;
    h *= PMX2;
    return h ^ (h >> 28);
}

struct Acc8 {
    uint64_t a[8];
    __device__ __forceinline__ void init() {
        a[0] = P32_3; a[1] = P64_1; a[2] = P64_2; a[3] = P64_3;
        a[4] = P64_4; a[5] = P32_2; a[6] = P64_5; a[7] = P32_1;
    }
    // one 8-byte word of a stripe: word j of the stripe, secret word `sec`.
    template <int J>
    __device__ __forceinline__ void word(uint64_t v, uint64_t sec) {
        uint64_t k = v ^ sec;
        a[J ^ 1] += v;
        a[J] += mul32x32(k);
    }
    __device__ __forceinline__ void scramble() {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            uint64_t x = a[i];
            x ^= x >> 47;
            x ^= Secret::w(128 + 8 * i);
            x *= P32_1;
            a[i] = x;
        }
    }
    __device__ __forceinline__ uint64_t merge(uint64_t len) const {
        uint64_t r = len * P64_1;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            r += fold64(a[2 * i] ^ Secret::w(11 + 16 * i), a[2 * i + 1] ^ Secret::w(11 + 16 * i + 8));
        return avalanche(r);
    }
};

// One scramble of a single accumulator lane j (used by the serial batch
// checksum chain, where lane j of a wave carries acc[j]).
__device__ __forceinline__ uint64_t scramble1(uint64_t x, uint64_t key) {
    x ^= x >> 47;
    x ^= key;
    return x * P32_1;
}

// ---------------------------------------------------------------- readers
// Little-endian loads at any byte address. gfx950 has unaligned global
// access in hardware (LLVM feature unaligned-buffer-access); hipcc lowers these
// to single global_load_dword{,x2,x4} instructions.
typedef uint64_t __attribute__((aligned(1))) u64_ua;
typedef uint32_t __attribute__((aligned(1))) u32_ua;
typedef uint16_t __attribute__((aligned(1))) u16_ua;
typedef uint4 __attribute__((aligned(1))) u128_ua;
__device__ __forceinline__ uint64_t ld64_any(const uint8_t *p) { return *(const u64_ua *)p; }
__device__ __forceinline__ uint32_t ld32_any(const uint8_t *p) { return *(const u32_ua *)p; }
__device__ __forceinline__ uint4 ld128_any(const uint8_t *p) { return *(const u128_ua *)p; }
__device__ __forceinline__ void st64_any(uint8_t *p, uint64_t v) { *(u64_ua *)p = v; }
__device__ __forceinline__ void st128_any(uint8_t *p, uint4 v) { *(u128_ua *)p = v; }

// Generic one-lane XXH3-64 over [p, p+len) in global memory (any alignment).
// Used by the general walk, the ranges API, the encoder and error paths.
__device__ inline uint64_t xxh3_64_lane(const uint8_t *p, uint64_t len) {
    if (len <= 16) {
        if (len > 8) {
            uint64_t lo = ld64_any(p) ^ (Secret::w(24) ^ Secret::w(32));
            uint64_t hi = ld64_any(p + len - 8) ^ (Secret::w(40) ^ Secret::w(48));
            uint64_t acc = len + __builtin_bswap64(lo) + hi + fold64(lo, hi);
            return avalanche(acc);
        }
        if (len >= 4) {
            uint32_t in1 = ld32_any(p), in2 = ld32_any(p + len - 4);
            uint64_t bitflip = Secret::w(8) ^ Secret::w(16);
            uint64_t in64 = (uint64_t)in2 + ((uint64_t)in1 << 32);
            return rrmxmx(in64 ^ bitflip, len);
        }
        if (len > 0) {
            uint32_t c1 = p[0], c2 = p[len >> 1], c3 = p[len - 1];
            uint32_t combined = (c1 << 16) | (c2 << 24) | c3 | ((uint32_t)len << 8);
            uint64_t bitflip = (uint64_t)((uint32_t)Secret::w(0) ^ (uint32_t)Secret::w(4));
            return xxh64_avalanche((uint64_t)combined ^ bitflip);
        }
        return xxh64_avalanche(Secret::w(56) ^ Secret::w(64));
    }
    auto mix16 = [&](uint64_t off, uint64_t s0, uint64_t s1) {
        return fold64(ld64_any(p + off) ^ s0, ld64_any(p + off + 8) ^ s1);
    };
    if (len <= 128) {
        uint64_t acc = len * P64_1;
        if (len > 32) {
            if (len > 64) {
                if (len > 96) {
                    acc += mix16(48, Secret::w(96), Secret::w(104));
                    acc += mix16(len - 64, Secret::w(112), Secret::w(120));
                }
                acc += mix16(32, Secret::w(64), Secret::w(72));
                acc += mix16(len - 48, Secret::w(80), Secret::w(88));
            }
            acc += mix16(16, Secret::w(32), Secret::w(40));
            acc += mix16(len - 32, Secret::w(48), Secret::w(56));
        }
        acc += mix16(0, Secret::w(0), Secret::w(8));
        acc += mix16(len - 16, Secret::w(16), Secret::w(24));
        return avalanche(acc);
    }
    if (len <= 240) {
        uint64_t acc = len * P64_1;
#pragma unroll
        for (int i = 0; i < 8; ++i) acc += mix16(16 * i, Secret::w(16 * i), Secret::w(16 * i + 8));
        acc = avalanche(acc);
        uint32_t rounds = (uint32_t)(len / 16);
        // offsets 16*(i-8)+3 for i = 8..14 (rounds <= 15)
#pragma unroll
        for (int i = 8; i < 15; ++i)
            if ((uint32_t)i < rounds)
                acc += mix16(16 * i, Secret::w(16 * (i - 8) + 3), Secret::w(16 * (i - 8) + 11));
        acc += mix16(len - 16, Secret::w(119), Secret::w(127));
        return avalanche(acc);
    }
    Acc8 acc;
    acc.init();
    uint64_t nb = (len - 1) / 1024;
    for (uint64_t b = 0; b < nb; ++b) {
        const uint8_t *blk = p + b * 1024;
#pragma unroll 4
        for (int s = 0; s < 16; ++s) {
            const uint8_t *st = blk + 64 * s;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                uint64_t v = ld64_any(st + 8 * j);
                uint64_t k = v ^ kSecretW8[s + j];
                acc.a[j ^ 1] += v;
                acc.a[j] += mul32x32(k);
            }
        }
        acc.scramble();
    }
    uint32_t ns = (uint32_t)(((len - 1) - 1024 * nb) / 64);
    const uint8_t *blk = p + nb * 1024;
    for (uint32_t s = 0; s < ns; ++s) {
        const uint8_t *st = blk + 64 * s;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint64_t v = ld64_any(st + 8 * j);
            uint64_t k = v ^ kSecretW8[s + j];
            acc.a[j ^ 1] += v;
            acc.a[j] += mul32x32(k);
        }
    }
    const uint8_t *last = p + len - 64;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        uint64_t v = ld64_any(last + 8 * j);
        uint64_t k = v ^ Secret::w(121 + 8 * j);
        acc.a[j ^ 1] += v;
        acc.a[j] += mul32x32(k);
    }
    return acc.merge(len);
}

}  // namespace iggy

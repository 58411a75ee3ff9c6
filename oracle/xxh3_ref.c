/*
 * xxh3_ref.c — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Scalar XXH3-64, seed 0, default 192-byte secret, restated from the public
 * XXH3 specification (xxHash v0.8.x; output frozen since v0.8.0). The
 * reference gets this from twox-hash 2.1.3 `XxHash3_64::oneshot`
 * (call sites: core/binary_protocol/src/batch.rs:485,
 * requests/messages/send_messages.rs:162, common/src/utils/checksum.rs:21).
 * Pinned by tests/test_oracle.py against libxxhash 0.8.2 for every length
 * 0..1200 and spot lengths to 1 MiB, and by the Rust golden vectors.
 *
 * oracle_xxh3_64_fast is the same function with the long-input accumulate in
 * AVX2 (as twox-hash's own AVX2 backend); it is the timed CPU baseline and is
 * cross-checked against the scalar form.
 */
#include "oracle.h"
#include <string.h>

#define P32_1 0x9E3779B1u
#define P32_2 0x85EBCA77u
#define P32_3 0xC2B2AE3Du
#define P64_1 0x9E3779B185EBCA87ull
#define P64_2 0xC2B2AE3D27D4EB4Full
#define P64_3 0x165667B19E3779F9ull
#define P64_4 0x85EBCA77C2B2AE63ull
#define P64_5 0x27D4EB2F165667C5ull
#define PMX1 0x165667919E3779F9ull
#define PMX2 0x9FB21C651E98DF25ull

static const uint8_t kSecret[192] = {
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
};

static inline uint64_t rd64(const uint8_t *p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v; /* little-endian host */
}
static inline uint32_t rd32(const uint8_t *p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}
static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }
static inline uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

static inline uint64_t fold64(uint64_t a, uint64_t b) {
    unsigned __int128 p = (unsigned __int128)a * b;
    return (uint64_t)p ^ (uint64_t)(p >> 64);
}
static inline uint64_t xxh64_avalanche(uint64_t h) {
    h ^= h >> 33; h *= P64_2; h ^= h >> 29; h *= P64_3; h ^= h >> 32;
    return h;
}
static inline uint64_t xxh3_avalanche(uint64_t h) {
    h ^= h >> 37; h *= PMX1; h ^= h >> 32;
    return h;
}
static inline uint64_t rrmxmx(uint64_t h, uint64_t len) {
    h ^= rotl64(h, 49) ^ rotl64(h, 24);
    h *= PMX2;
    h ^= (h >> 35) + len;
    h *= PMX2;
    return h ^ (h >> 28);
}
static inline uint64_t mix16(const uint8_t *in, const uint8_t *sec) {
    return fold64(rd64(in) ^ rd64(sec), rd64(in + 8) ^ rd64(sec + 8));
}

static uint64_t len_0to16(const uint8_t *p, size_t len) {
    const uint8_t *s = kSecret;
    if (len > 8) {
        uint64_t lo = rd64(p) ^ (rd64(s + 24) ^ rd64(s + 32));
        uint64_t hi = rd64(p + len - 8) ^ (rd64(s + 40) ^ rd64(s + 48));
        uint64_t acc = (uint64_t)len + bswap64(lo) + hi + fold64(lo, hi);
        return xxh3_avalanche(acc);
    }
    if (len >= 4) {
        uint64_t seed = 0;
        seed ^= (uint64_t)bswap32((uint32_t)seed) << 32;
        uint32_t in1 = rd32(p), in2 = rd32(p + len - 4);
        uint64_t bitflip = (rd64(s + 8) ^ rd64(s + 16)) - seed;
        uint64_t in64 = in2 + ((uint64_t)in1 << 32);
        return rrmxmx(in64 ^ bitflip, len);
    }
    if (len > 0) {
        uint8_t c1 = p[0], c2 = p[len >> 1], c3 = p[len - 1];
        uint32_t combined = ((uint32_t)c1 << 16) | ((uint32_t)c2 << 24) | ((uint32_t)c3 << 0) |
                            ((uint32_t)len << 8);
        uint64_t bitflip = (uint64_t)(rd32(s) ^ rd32(s + 4));
        return xxh64_avalanche((uint64_t)combined ^ bitflip);
    }
    return xxh64_avalanche(rd64(s + 56) ^ rd64(s + 64));
}

static uint64_t len_17to128(const uint8_t *p, size_t len) {
    const uint8_t *s = kSecret;
    uint64_t acc = (uint64_t)len * P64_1;
    if (len > 32) {
        if (len > 64) {
            if (len > 96) {
                acc += mix16(p + 48, s + 96);
                acc += mix16(p + len - 64, s + 112);
            }
            acc += mix16(p + 32, s + 64);
            acc += mix16(p + len - 48, s + 80);
        }
        acc += mix16(p + 16, s + 32);
        acc += mix16(p + len - 32, s + 48);
    }
    acc += mix16(p, s);
    acc += mix16(p + len - 16, s + 16);
    return xxh3_avalanche(acc);
}

static uint64_t len_129to240(const uint8_t *p, size_t len) {
    const uint8_t *s = kSecret;
    uint64_t acc = (uint64_t)len * P64_1;
    size_t rounds = len / 16;
    for (size_t i = 0; i < 8; i++) acc += mix16(p + 16 * i, s + 16 * i);
    acc = xxh3_avalanche(acc);
    for (size_t i = 8; i < rounds; i++) acc += mix16(p + 16 * i, s + 16 * (i - 8) + 3);
    acc += mix16(p + len - 16, s + 136 - 17);
    return xxh3_avalanche(acc);
}

static void accumulate_512(uint64_t acc[8], const uint8_t *in, const uint8_t *sec) {
    for (int i = 0; i < 8; i++) {
        uint64_t v = rd64(in + 8 * i);
        uint64_t k = v ^ rd64(sec + 8 * i);
        acc[i ^ 1] += v;
        acc[i] += (uint64_t)(uint32_t)k * (k >> 32);
    }
}
static void scramble(uint64_t acc[8], const uint8_t *sec) {
    for (int i = 0; i < 8; i++) {
        uint64_t a = acc[i];
        a ^= a >> 47;
        a ^= rd64(sec + 8 * i);
        a *= P32_1;
        acc[i] = a;
    }
}
static uint64_t merge_accs(const uint64_t acc[8], uint64_t start) {
    const uint8_t *s = kSecret + 11;
    uint64_t r = start;
    for (int i = 0; i < 4; i++)
        r += fold64(acc[2 * i] ^ rd64(s + 16 * i), acc[2 * i + 1] ^ rd64(s + 16 * i + 8));
    return xxh3_avalanche(r);
}

typedef void (*acc512_fn)(uint64_t acc[8], const uint8_t *in, const uint8_t *sec);

static uint64_t hash_long(const uint8_t *p, size_t len, acc512_fn acc512) {
    uint64_t acc[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
    const size_t block = 1024, stripes_per_block = 16;
    size_t nb = (len - 1) / block;
    for (size_t b = 0; b < nb; b++) {
        for (size_t s = 0; s < stripes_per_block; s++)
            acc512(acc, p + b * block + 64 * s, kSecret + 8 * s);
        scramble(acc, kSecret + 192 - 64);
    }
    size_t ns = ((len - 1) - block * nb) / 64;
    for (size_t s = 0; s < ns; s++) acc512(acc, p + nb * block + 64 * s, kSecret + 8 * s);
    acc512(acc, p + len - 64, kSecret + 192 - 64 - 7);
    return merge_accs(acc, (uint64_t)len * P64_1);
}

uint64_t oracle_xxh3_64(const void *data, size_t len) {
    const uint8_t *p = (const uint8_t *)data;
    if (len <= 16) return len_0to16(p, len);
    if (len <= 128) return len_17to128(p, len);
    if (len <= 240) return len_129to240(p, len);
    return hash_long(p, len, accumulate_512);
}

/* ---- AVX2 accumulate (CPU baseline speed; identical arithmetic) ---- */
#if defined(__x86_64__)
#include <immintrin.h>
__attribute__((target("avx2"))) static void accumulate_512_avx2(uint64_t acc[8],
                                                                 const uint8_t *in,
                                                                 const uint8_t *sec) {
    for (int h = 0; h < 2; h++) {
        __m256i a = _mm256_loadu_si256((const __m256i *)(acc + 4 * h));
        __m256i v = _mm256_loadu_si256((const __m256i *)(in + 32 * h));
        __m256i k = _mm256_xor_si256(v, _mm256_loadu_si256((const __m256i *)(sec + 32 * h)));
        __m256i khi = _mm256_srli_epi64(k, 32);
        __m256i prod = _mm256_mul_epu32(k, khi);
        __m256i vsw = _mm256_shuffle_epi32(v, _MM_SHUFFLE(1, 0, 3, 2)); /* swap u64 pairs */
        a = _mm256_add_epi64(a, _mm256_add_epi64(prod, vsw));
        _mm256_storeu_si256((__m256i *)(acc + 4 * h), a);
    }
}
__attribute__((target("avx2"))) static int cpu_avx2(void) { return __builtin_cpu_supports("avx2"); }
int oracle_has_avx2(void) { return cpu_avx2(); }
#else
int oracle_has_avx2(void) { return 0; }
#endif

uint64_t oracle_xxh3_64_fast(const void *data, size_t len) {
    const uint8_t *p = (const uint8_t *)data;
    if (len <= 240) return oracle_xxh3_64(data, len);
#if defined(__x86_64__)
    if (oracle_has_avx2()) return hash_long(p, len, accumulate_512_avx2);
#endif
    return hash_long(p, len, accumulate_512);
}

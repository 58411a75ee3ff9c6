// crypt.hip — at-rest encryption re-encode of a batch record:
// encrypt_batch_request / decrypt_batch_record
// (core/server_common/src/send_messages.rs:293-355, :357-415) with
// Aes256GcmEncryptor (core/common/src/utils/crypto.rs:47-90).
//
// A section (a message's payload, or its user headers when non-empty) becomes
// nonce(12) || AES-256-GCM(ct) || tag(16), empty associated data; decrypt reverses
// it. Pipeline (one stream order, see iggy_codec_{en,de}crypt_batch_device):
//   decode walk  -> frame positions (Verify for encrypt, LayoutOnly for decrypt)
//   k_crypt_sizes / k_crypt_scan -> output frame positions (tile-local scan + tile prefix)
//   k_crypt_frames: one wave per frame, one 16-B block per lane per pass:
//       AES-256 CTR keystream (T-table rounds, table in LDS), 16-B unaligned loads and
//       stores, GHASH as sum_j X_j * H^(r - j) with 4-bit tables of H^1..H^64 in LDS
//       (lane 0 folds the running hash in), then the length block and E_K(J0)
//   k_crypt_checksums: per-frame XXH3 over frame[8..]
//   block sums + scramble chain (batch_checksum.hip) -> the batch checksum
//   k_crypt_finish: header, precedence, result.
// Integer / byte work, no MFMA: the bound is VALU + LDS (AES and GHASH tables).
#include "codec_common.hpp"
#include "xxh3_device.hpp"

namespace iggy {

struct CryptKey {
    uint32_t rk[60];  // AES-256 round keys, FIPS-197 words w[0..59] (big-endian byte order)
};

struct CryptScratch {
    const iggy_decode_result *dres;  // the input walk (frame_count, error)
    const uint64_t *pos;             // input frame starts (blob-relative)
    uint64_t *osize;                 // [n] output frame size -> exclusive prefix inside its tile
    uint64_t *tsum;                  // [ntiles] tile sums -> exclusive tile prefix
    uint64_t *opos;                  // [n] output frame starts (blob-relative)
    uint64_t *misc;                  // [8]: 0 ~(2 i + section) of the first bad section, 1 ~i u32 overflow, 2 blob bytes
    const uint64_t *gtab;            // [64][16][2]: 4-bit GHASH tables {HL, HH} of H^1 .. H^64
    iggy_batch_header *dh;           // header of the output for the checksum kernels
    uint64_t *dn;                    // frame count for the checksum kernels
    uint64_t *dsum;                  // batch checksum of the output
};

constexpr uint32_t kCryptTile = 1024;   // frames per scan tile
constexpr uint32_t kGhPowers = 64;      // H^1 .. H^64 (one pass of 64 blocks)
constexpr uint32_t kCryptLds = 1024 + 256 + 64 + kGhPowers * 16 * 16;  // Te0, S-box, last4, tables

__constant__ static const uint8_t kAesSbox[256] = {
    0x63, 0x7c, 0x77, 0x7b, 0xf2, 0x6b, 0x6f, 0xc5, 0x30, 0x01, 0x67, 0x2b, 0xfe, 0xd7, 0xab, 0x76,
    0xca, 0x82, 0xc9, 0x7d, 0xfa, 0x59, 0x47, 0xf0, 0xad, 0xd4, 0xa2, 0xaf, 0x9c, 0xa4, 0x72, 0xc0,
    0xb7, 0xfd, 0x93, 0x26, 0x36, 0x3f, 0xf7, 0xcc, 0x34, 0xa5, 0xe5, 0xf1, 0x71, 0xd8, 0x31, 0x15,
    0x04, 0xc7, 0x23, 0xc3, 0x18, 0x96, 0x05, 0x9a, 0x07, 0x12, 0x80, 0xe2, 0xeb, 0x27, 0xb2, 0x75,
    0x09, 0x83, 0x2c, 0x1a, 0x1b, 0x6e, 0x5a, 0xa0, 0x52, 0x3b, 0xd6, 0xb3, 0x29, 0xe3, 0x2f, 0x84,
    0x53, 0xd1, 0x00, 0xed, 0x20, 0xfc, 0xb1, 0x5b, 0x6a, 0xcb, 0xbe, 0x39, 0x4a, 0x4c, 0x58, 0xcf,
    0xd0, 0xef, 0xaa, 0xfb, 0x43, 0x4d, 0x33, 0x85, 0x45, 0xf9, 0x02, 0x7f, 0x50, 0x3c, 0x9f, 0xa8,
    0x51, 0xa3, 0x40, 0x8f, 0x92, 0x9d, 0x38, 0xf5, 0xbc, 0xb6, 0xda, 0x21, 0x10, 0xff, 0xf3, 0xd2,
    0xcd, 0x0c, 0x13, 0xec, 0x5f, 0x97, 0x44, 0x17, 0xc4, 0xa7, 0x7e, 0x3d, 0x64, 0x5d, 0x19, 0x73,
    0x60, 0x81, 0x4f, 0xdc, 0x22, 0x2a, 0x90, 0x88, 0x46, 0xee, 0xb8, 0x14, 0xde, 0x5e, 0x0b, 0xdb,
    0xe0, 0x32, 0x3a, 0x0a, 0x49, 0x06, 0x24, 0x5c, 0xc2, 0xd3, 0xac, 0x62, 0x91, 0x95, 0xe4, 0x79,
    0xe7, 0xc8, 0x37, 0x6d, 0x8d, 0xd5, 0x4e, 0xa9, 0x6c, 0x56, 0xf4, 0xea, 0x65, 0x7a, 0xae, 0x08,
    0xba, 0x78, 0x25, 0x2e, 0x1c, 0xa6, 0xb4, 0xc6, 0xe8, 0xdd, 0x74, 0x1f, 0x4b, 0xbd, 0x8b, 0x8a,
    0x70, 0x3e, 0xb5, 0x66, 0x48, 0x03, 0xf6, 0x0e, 0x61, 0x35, 0x57, 0xb9, 0x86, 0xc1, 0x1d, 0x9e,
    0xe1, 0xf8, 0x98, 0x11, 0x69, 0xd9, 0x8e, 0x94, 0x9b, 0x1e, 0x87, 0xe9, 0xce, 0x55, 0x28, 0xdf,
    0x8c, 0xa1, 0x89, 0x0d, 0xbf, 0xe6, 0x42, 0x68, 0x41, 0x99, 0x2d, 0x0f, 0xb0, 0x54, 0xbb, 0x16};

__device__ __forceinline__ uint32_t ror32(uint32_t x, int r) { return __builtin_amdgcn_alignbit(x, x, r); }

// AES-256 of one block (big-endian words in s0..s3): T-table rounds, Te1..Te3 as
// rotations of Te0 (LDS), the last round from the S-box (LDS)
__device__ __forceinline__ void aes256_enc(const CryptKey &k, const uint32_t *te, const uint8_t *sb, uint32_t &s0,
                                           uint32_t &s1, uint32_t &s2, uint32_t &s3) {
    s0 ^= k.rk[0]; s1 ^= k.rk[1]; s2 ^= k.rk[2]; s3 ^= k.rk[3];
#pragma unroll
    for (int r = 1; r < 14; ++r) {
        const uint32_t t0 = te[s0 >> 24] ^ ror32(te[(s1 >> 16) & 0xff], 8) ^ ror32(te[(s2 >> 8) & 0xff], 16) ^
                            ror32(te[s3 & 0xff], 24) ^ k.rk[4 * r];
        const uint32_t t1 = te[s1 >> 24] ^ ror32(te[(s2 >> 16) & 0xff], 8) ^ ror32(te[(s3 >> 8) & 0xff], 16) ^
                            ror32(te[s0 & 0xff], 24) ^ k.rk[4 * r + 1];
        const uint32_t t2 = te[s2 >> 24] ^ ror32(te[(s3 >> 16) & 0xff], 8) ^ ror32(te[(s0 >> 8) & 0xff], 16) ^
                            ror32(te[s1 & 0xff], 24) ^ k.rk[4 * r + 2];
        const uint32_t t3 = te[s3 >> 24] ^ ror32(te[(s0 >> 16) & 0xff], 8) ^ ror32(te[(s1 >> 8) & 0xff], 16) ^
                            ror32(te[s2 & 0xff], 24) ^ k.rk[4 * r + 3];
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    auto last = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t rk) {
        return ((uint32_t)sb[a >> 24] << 24) ^ ((uint32_t)sb[(b >> 16) & 0xff] << 16) ^
               ((uint32_t)sb[(c >> 8) & 0xff] << 8) ^ (uint32_t)sb[d & 0xff] ^ rk;
    };
    const uint32_t o0 = last(s0, s1, s2, s3, k.rk[56]), o1 = last(s1, s2, s3, s0, k.rk[57]);
    const uint32_t o2 = last(s2, s3, s0, s1, k.rk[58]), o3 = last(s3, s0, s1, s2, k.rk[59]);
    s0 = o0; s1 = o1; s2 = o2; s3 = o3;
}

// X * H^e in GF(2^128) (GCM bit order; X = xh || xl big-endian halves) with the
// power's 4-bit table t[16] = {HL[i], HH[i]} (Shoup's method, 32 nibble steps)
__device__ __forceinline__ void gmul(uint64_t &xh, uint64_t &xl, const uint64_t *t, const uint32_t *last4) {
    uint32_t n = (uint32_t)xl & 0xf;
    uint64_t zl = t[2 * n], zh = t[2 * n + 1];
    auto step = [&](uint32_t nib) {
        const uint32_t rem = (uint32_t)zl & 0xf;
        zl = (zh << 60) | (zl >> 4);
        zh = (zh >> 4) ^ ((uint64_t)last4[rem] << 48);
        zh ^= t[2 * nib + 1];
        zl ^= t[2 * nib];
    };
    step(((uint32_t)xl >> 4) & 0xf);  // byte 15, high nibble
#pragma unroll
    for (int i = 14; i >= 0; --i) {
        const uint32_t byte = (uint32_t)((i >= 8 ? xl >> (8 * (15 - i)) : xh >> (8 * (7 - i))) & 0xff);
        step(byte & 0xf);
        step(byte >> 4);
    }
    xh = zh;
    xl = zl;
}

__device__ __forceinline__ uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }

// The group's first bad section (encrypt: never; decrypt: too short, or the tag)
__device__ __forceinline__ void mark_bad(const CryptScratch &cs, uint64_t i, uint32_t section) {
    atomicMax((unsigned long long *)&cs.misc[0], (unsigned long long)~(2 * i + section));
}

// 1) output frame sizes, exclusive prefix inside each 1024-frame tile
template <bool ENC>
__global__ __launch_bounds__(256) void k_crypt_sizes(const uint8_t *record, CryptScratch cs) {
    __shared__ uint64_t part[256];
    if (cs.dres->error.kind != IGGY_OK) return;
    const uint64_t n = cs.dres->frame_count;
    const uint8_t *blob = record + kHdr;
    const uint64_t ntiles = (n + kCryptTile - 1) / kCryptTile;
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        uint64_t sz[4], sum = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint64_t i = t * kCryptTile + 4 * threadIdx.x + k;
            sz[k] = 0;
            if (i < n) {
                const uint8_t *f = blob + cs.pos[i];
                const uint64_t uh = ld32_any(f + 32), pl = ld32_any(f + 36);
                if (ENC) {
                    if (pl + 28 > 0xffffffffull || (uh && uh + 28 > 0xffffffffull))  // u32::try_from
                        atomicMax((unsigned long long *)&cs.misc[1], (unsigned long long)~i);
                    sz[k] = kFrameHdr + pl + 28 + (uh ? uh + 28 : 0);
                } else {
                    if (pl < 28) mark_bad(cs, i, 0);
                    else if (uh && uh < 28) mark_bad(cs, i, 1);
                    sz[k] = kFrameHdr + (pl >= 28 ? pl - 28 : 0) + (uh >= 28 ? uh - 28 : 0);
                }
            }
            sum += sz[k];
        }
        part[threadIdx.x] = sum;
        __syncthreads();
        for (uint32_t d = 1; d < 256; d <<= 1) {  // inclusive scan of the 256 partial sums
            const uint64_t v = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
            __syncthreads();
            part[threadIdx.x] += v;
            __syncthreads();
        }
        uint64_t run = part[threadIdx.x] - sum;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint64_t i = t * kCryptTile + 4 * threadIdx.x + k;
            if (i < n) cs.osize[i] = run;
            run += sz[k];
        }
        if (threadIdx.x == 255) cs.tsum[t] = part[255];
        __syncthreads();
    }
}

// 2) exclusive prefix of the tile sums (one WG), total blob bytes -> misc[2]
__global__ __launch_bounds__(1024) void k_crypt_scan(CryptScratch cs) {
    __shared__ uint64_t part[1024];
    if (cs.dres->error.kind != IGGY_OK) return;
    const uint64_t n = cs.dres->frame_count;
    const uint64_t ntiles = (n + kCryptTile - 1) / kCryptTile;
    uint64_t carry = 0;
    for (uint64_t base = 0; base < ntiles; base += 1024) {
        const uint64_t t = base + threadIdx.x;
        const uint64_t v = t < ntiles ? cs.tsum[t] : 0;
        part[threadIdx.x] = v;
        __syncthreads();
        for (uint32_t d = 1; d < 1024; d <<= 1) {
            const uint64_t w = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
            __syncthreads();
            part[threadIdx.x] += w;
            __syncthreads();
        }
        if (t < ntiles) cs.tsum[t] = carry + part[threadIdx.x] - v;
        carry += part[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) cs.misc[2] = carry;
}

// One section: ENC in = plaintext (n B), nonce from `nonce`, out = nonce || ct || tag;
// DEC in = nonce || ct || tag (n B), out = plaintext (n - 28 B), tag checked.
template <bool ENC>
__device__ __forceinline__ bool crypt_section(const CryptKey &key, const uint32_t *te, const uint8_t *sb,
                                              const uint64_t *tabs, const uint32_t *last4, const uint8_t *in,
                                              uint64_t n, const uint8_t *nonce, uint8_t *out, int lane) {
    const uint8_t *np = ENC ? nonce : in;
    const uint32_t nw0 = __builtin_bswap32(ld32_any(np)), nw1 = __builtin_bswap32(ld32_any(np + 4));
    const uint32_t nw2 = __builtin_bswap32(ld32_any(np + 8));
    const uint64_t clen = ENC ? n : n - 28;          // ciphertext bytes
    const uint8_t *src = ENC ? in : in + 12;         // bytes XORed with the keystream
    uint8_t *dst = ENC ? out + 12 : out;
    const uint64_t m = (clen + 15) / 16;             // data blocks
    uint64_t yh = 0, yl = 0;                         // the running GHASH (lane-uniform)
    for (uint64_t p0 = 0; p0 < m; p0 += 64) {
        const uint64_t b = p0 + lane;
        const uint32_t r = (uint32_t)min<uint64_t>(64, m - p0);  // blocks in this pass
        uint64_t xh = 0, xl = 0;
        if (b < m) {
            uint32_t s0 = nw0, s1 = nw1, s2 = nw2, s3 = (uint32_t)(b + 2);
            aes256_enc(key, te, sb, s0, s1, s2, s3);
            const uint64_t kl = (uint64_t)__builtin_bswap32(s0) | ((uint64_t)__builtin_bswap32(s1) << 32);
            const uint64_t kh = (uint64_t)__builtin_bswap32(s2) | ((uint64_t)__builtin_bswap32(s3) << 32);
            const uint64_t kb = clen - 16 * b;  // bytes of this block (>= 1)
            uint64_t d0 = 0, d1 = 0;            // little-endian halves of the 16 bytes
            if (kb >= 16) {
                const uint4 v = ld128_any(src + 16 * b);
                d0 = (uint64_t)v.x | ((uint64_t)v.y << 32);
                d1 = (uint64_t)v.z | ((uint64_t)v.w << 32);
            } else {
                for (uint32_t q = 0; q < (uint32_t)kb; ++q) {
                    const uint64_t byte = src[16 * b + q];
                    if (q < 8) d0 |= byte << (8 * q);
                    else d1 |= byte << (8 * (q - 8));
                }
            }
            uint64_t e0 = d0 ^ kl, e1 = d1 ^ kh;
            if (kb < 16) {  // the partial block: bytes past the end are zero (GHASH padding)
                const uint64_t mk0 = kb >= 8 ? ~0ull : ((1ull << (8 * kb)) - 1);
                const uint64_t mk1 = kb >= 16 ? ~0ull : kb <= 8 ? 0 : ((1ull << (8 * (kb - 8))) - 1);
                e0 &= mk0; e1 &= mk1;
            }
            if (kb >= 16) {
                st128_any(dst + 16 * b, make_uint4((uint32_t)e0, (uint32_t)(e0 >> 32), (uint32_t)e1,
                                                   (uint32_t)(e1 >> 32)));
            } else {
                for (uint32_t q = 0; q < (uint32_t)kb; ++q)
                    dst[16 * b + q] = (uint8_t)((q < 8 ? e0 >> (8 * q) : e1 >> (8 * (q - 8))) & 0xff);
            }
            // GHASH input: the ciphertext block (ENC: e, DEC: d masked)
            const uint64_t c0 = ENC ? e0 : (kb >= 16 ? d0 : d0 & (kb >= 8 ? ~0ull : ((1ull << (8 * kb)) - 1)));
            const uint64_t c1 = ENC ? e1 : (kb >= 16 ? d1 : (kb <= 8 ? 0 : d1 & ((1ull << (8 * (kb - 8))) - 1)));
            xh = bswap64(c0);
            xl = bswap64(c1);
            if (lane == 0) { xh ^= yh; xl ^= yl; }
            gmul(xh, xl, tabs + 32 * (r - lane - 1), last4);  // * H^(r - lane)
        }
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            xh ^= __shfl_xor(xh, d);
            xl ^= __shfl_xor(xl, d);
        }
        yh = xh;
        yl = xl;
    }
    // the length block (empty AAD), then * H; E_K(J0) for the tag
    yl ^= clen * 8;
    gmul(yh, yl, tabs, last4);
    uint32_t j0 = nw0, j1 = nw1, j2 = nw2, j3 = 1;
    aes256_enc(key, te, sb, j0, j1, j2, j3);
    const uint64_t th = yh ^ (((uint64_t)j0 << 32) | j1), tl = yl ^ (((uint64_t)j2 << 32) | j3);
    // tag bytes big-endian: th then tl
    const uint64_t tag0 = bswap64(th), tag1 = bswap64(tl);
    if (ENC) {
        if (lane == 0) {
            *(u32_ua *)(out + 0) = ld32_any(nonce);
            *(u32_ua *)(out + 4) = ld32_any(nonce + 4);
            *(u32_ua *)(out + 8) = ld32_any(nonce + 8);
            st128_any(out + 12 + clen,
                      make_uint4((uint32_t)tag0, (uint32_t)(tag0 >> 32), (uint32_t)tag1, (uint32_t)(tag1 >> 32)));
        }
        return true;
    }
    const uint4 st = ld128_any(in + 12 + clen);
    return st.x == (uint32_t)tag0 && st.y == (uint32_t)(tag0 >> 32) && st.z == (uint32_t)tag1 &&
           st.w == (uint32_t)(tag1 >> 32);
}

// 3) frames: one wave per frame (both sections, then the 40 header bytes after the checksum)
template <bool ENC>
__global__ __launch_bounds__(256) void k_crypt_frames(const uint8_t *record, uint8_t *out, uint64_t cap,
                                                      const uint8_t *nonces, CryptKey key, CryptScratch cs) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t *te = (uint32_t *)smem;
    uint8_t *sb = smem + 1024;
    uint32_t *last4 = (uint32_t *)(smem + 1280);
    uint64_t *tabs = (uint64_t *)(smem + 1344);
    if (cs.dres->error.kind != IGGY_OK) return;
    const uint64_t n = cs.dres->frame_count;
    if (kHdr + cs.misc[2] > cap || cs.misc[1] != 0) return;  // capacity / overflow: nothing is written
    for (uint32_t x = threadIdx.x; x < 256; x += blockDim.x) {
        const uint32_t s = kAesSbox[x];
        const uint32_t s2 = ((s << 1) ^ ((s & 0x80) ? 0x1b : 0)) & 0xff, s3 = s2 ^ s;
        te[x] = (s2 << 24) | (s << 16) | (s << 8) | s3;
        sb[x] = (uint8_t)s;
    }
    if (threadIdx.x < 16) {  // x * 0x1c20 carry-less: the 4-bit reduction table
        const uint32_t r = threadIdx.x;
        last4[r] = ((r & 1) ? 0x1c20u : 0) ^ ((r & 2) ? 0x3840u : 0) ^ ((r & 4) ? 0x7080u : 0) ^ ((r & 8) ? 0xe100u : 0);
    }
    for (uint32_t x = threadIdx.x; x < kGhPowers * 32; x += blockDim.x) tabs[x] = cs.gtab[x];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint64_t wid = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint8_t *blob = record + kHdr;
    uint8_t *oblob = out + kHdr;
    for (uint64_t i = wid; i < n; i += nwaves) {
        const uint8_t *f = blob + cs.pos[i];
        const uint64_t uh = ld32_any(f + 32), pl = ld32_any(f + 36);
        const uint64_t op = cs.tsum[i / kCryptTile] + cs.osize[i];
        uint8_t *of = oblob + op;
        if (lane == 0) cs.opos[i] = op;
        uint64_t opl, ouh;
        if (ENC) {
            opl = pl + 28;
            ouh = uh ? uh + 28 : 0;
            crypt_section<true>(key, te, sb, tabs, last4, f + kFrameHdr, pl, nonces + 24 * i, of + kFrameHdr, lane);
            if (uh)
                crypt_section<true>(key, te, sb, tabs, last4, f + kFrameHdr + pl, uh, nonces + 24 * i + 12,
                                    of + kFrameHdr + opl, lane);
        } else {
            if (pl < 28 || (uh && uh < 28)) continue;  // marked by k_crypt_sizes
            opl = pl - 28;
            ouh = uh ? uh - 28 : 0;
            if (!crypt_section<false>(key, te, sb, tabs, last4, f + kFrameHdr, pl, nullptr, of + kFrameHdr, lane)) {
                if (lane == 0) mark_bad(cs, i, 0);
            } else if (uh && !crypt_section<false>(key, te, sb, tabs, last4, f + kFrameHdr + pl, uh, nullptr,
                                                   of + kFrameHdr + opl, lane)) {
                if (lane == 0) mark_bad(cs, i, 1);
            }
        }
        // header bytes 8..48: id, offset_delta, timestamp_delta kept; lengths; reserved 0
        if (lane < 10) {
            uint32_t w = 0;
            if (lane < 6) w = ld32_any(f + 8 + 4 * lane);
            else if (lane == 6) w = (uint32_t)ouh;
            else if (lane == 7) w = (uint32_t)opl;
            *(u32_ua *)(of + 8 + 4 * lane) = w;
        }
    }
}

// 4) per-frame XXH3 over frame[8..] into frame[0..8)
__global__ __launch_bounds__(256) void k_crypt_checksums(uint8_t *out, uint64_t cap, CryptScratch cs) {
    if (cs.dres->error.kind != IGGY_OK) return;
    if (kHdr + cs.misc[2] > cap || cs.misc[1] != 0 || cs.misc[0] != 0) return;
    const uint64_t n = cs.dres->frame_count;
    uint8_t *oblob = out + kHdr;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t op = cs.opos[i];
        const uint64_t end = (i + 1 < n) ? cs.opos[i + 1] : cs.misc[2];
        st64_any(oblob + op, xxh3_64_lane(oblob + op + 8, end - op - 8));
    }
}

// 5) the output header for the checksum kernels (input header, new batch_length)
// (no frames when anything failed: the checksum kernels then read no output position)
__global__ void k_crypt_header(uint64_t cap, CryptScratch cs) {
    if (threadIdx.x != 0) return;
    iggy_batch_header h = cs.dres->header;
    h.batch_length = kHdr + cs.misc[2];
    *cs.dh = h;
    const bool ok = cs.dres->error.kind == IGGY_OK && kHdr + cs.misc[2] <= cap && cs.misc[0] == 0 && cs.misc[1] == 0;
    *cs.dn = ok ? cs.dres->frame_count : 0;
}

// 6) precedence, header, result (one wave: the header is copied 4 B per lane; the
// input's reserved bytes 52..255 are zero, validated by the decode)
template <bool ENC>
__global__ void k_crypt_finish(const uint8_t *record, uint64_t len, uint8_t *out, uint64_t cap, CryptScratch cs,
                               iggy_crypt_result *res) {
    const int lane = threadIdx.x & 63;
    iggy_crypt_result r;
    memset(&r, 0, sizeof(r));
    r.error = cs.dres->error;
    bool ok = false;
    if (r.error.kind == IGGY_OK) {
        const uint64_t total = kHdr + cs.misc[2];
        const uint64_t bl = cs.dres->header.batch_length;
        r.frame_count = cs.dres->frame_count;
        if (!ENC && len != bl) {  // decrypt_batch_record: record.len() != total_size()
            r.error.kind = IGGY_ERR_INVALID_COMMAND;
            r.error.a = len;
            r.error.b = bl;
        } else if (cs.misc[1] != 0) {  // encrypt: a section length past u32
            r.error.kind = IGGY_ERR_INVALID_COMMAND;
            r.error.a = ~cs.misc[1];
        } else if (total > cap) {
            r.error.kind = IGGY_ERR_CAPACITY;
            r.error.a = total;
            r.error.b = cap;
        } else if (cs.misc[0] != 0) {
            const uint64_t enc = ~cs.misc[0];
            r.error.kind = IGGY_ERR_CANNOT_DECRYPT_DATA;
            r.error.a = enc >> 1;
            r.error.b = enc & 1;
        } else {
            ok = true;
            r.out_len = total;
            r.batch_checksum = *cs.dsum;
        }
    }
    if (ok) {
        uint32_t w = ld32_any(record + 4 * lane);
        if (lane == 8) w = (uint32_t)r.out_len;
        if (lane == 9) w = (uint32_t)(r.out_len >> 32);
        if (lane == 10) w = (uint32_t)r.batch_checksum;
        if (lane == 11) w = (uint32_t)(r.batch_checksum >> 32);
        *(u32_ua *)(out + 4 * lane) = w;
    }
    if (lane == 0) *res = r;
}

}  // namespace iggy

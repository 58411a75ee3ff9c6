// host_crypt.hpp -- at-rest encryption host setup: AES-256 key schedule, GHASH tables and the
// encrypt / decrypt entries (kernels in crypt.hip)
//
// Part of the unity build of libiggy_codec.so: included by codec_api.hip, after the
// kernel translation units and the units before it (see codec_api.hip for the order).
#pragma once

extern "C" {

// ------------------------------------------------- at-rest encryption (crypt.hip)
namespace {
const uint8_t kAesSboxHost[256] = {
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

uint32_t sub_word(uint32_t w) {
    return ((uint32_t)kAesSboxHost[w >> 24] << 24) | ((uint32_t)kAesSboxHost[(w >> 16) & 0xff] << 16) |
           ((uint32_t)kAesSboxHost[(w >> 8) & 0xff] << 8) | kAesSboxHost[w & 0xff];
}
// FIPS-197 5.2, Nk = 8: words w[0..59], big-endian byte order
void aes256_key_schedule(const uint8_t key[32], uint32_t w[60]) {
    for (int i = 0; i < 8; ++i)
        w[i] = ((uint32_t)key[4 * i] << 24) | ((uint32_t)key[4 * i + 1] << 16) | ((uint32_t)key[4 * i + 2] << 8) |
               key[4 * i + 3];
    uint32_t rcon = 0x01000000u;
    for (int i = 8; i < 60; ++i) {
        uint32_t t = w[i - 1];
        if (i % 8 == 0) {
            t = sub_word((t << 8) | (t >> 24)) ^ rcon;
            rcon = ((rcon << 1) ^ ((rcon & 0x80000000u) ? 0x1b000000u : 0)) & 0xff000000u;
        } else if (i % 8 == 4) {
            t = sub_word(t);
        }
        w[i] = w[i - 8] ^ t;
    }
}
uint8_t gf_xtime(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }
// one block, byte-oriented rounds (only H = E_K(0) is computed on the host)
void aes256_block_host(const uint32_t w[60], const uint8_t in[16], uint8_t out[16]) {
    uint8_t s[16];
    auto add_key = [&](int r) {
        for (int c = 0; c < 4; ++c)
            for (int k = 0; k < 4; ++k) s[4 * c + k] ^= (uint8_t)(w[4 * r + c] >> (24 - 8 * k));
    };
    memcpy(s, in, 16);
    add_key(0);
    for (int r = 1; r <= 14; ++r) {
        uint8_t t[16];
        for (int i = 0; i < 16; ++i) t[i] = kAesSboxHost[s[i]];
        for (int c = 0; c < 4; ++c)
            for (int k = 0; k < 4; ++k) s[4 * c + k] = t[4 * ((c + k) % 4) + k];
        if (r != 14)
            for (int c = 0; c < 4; ++c) {
                uint8_t *a = s + 4 * c;
                const uint8_t a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3], x = (uint8_t)(a0 ^ a1 ^ a2 ^ a3);
                a[0] ^= (uint8_t)(x ^ gf_xtime((uint8_t)(a0 ^ a1)));
                a[1] ^= (uint8_t)(x ^ gf_xtime((uint8_t)(a1 ^ a2)));
                a[2] ^= (uint8_t)(x ^ gf_xtime((uint8_t)(a2 ^ a3)));
                a[3] ^= (uint8_t)(x ^ gf_xtime((uint8_t)(a3 ^ a0)));
            }
        add_key(r);
    }
    memcpy(out, s, 16);
}
// GF(2^128) product, GCM bit order, (hi, lo) big-endian halves
void gf128_mul(uint64_t xh, uint64_t xl, uint64_t yh, uint64_t yl, uint64_t &zh, uint64_t &zl) {
    zh = zl = 0;
    for (int i = 0; i < 128; ++i) {
        const uint64_t bit = i < 64 ? (xh >> (63 - i)) & 1 : (xl >> (127 - i)) & 1;
        if (bit) { zh ^= yh; zl ^= yl; }
        const uint64_t lsb = yl & 1;
        yl = (yl >> 1) | (yh << 63);
        yh >>= 1;
        if (lsb) yh ^= 0xe100000000000000ull;
    }
}
// Shoup 4-bit table of P: t[2 i] = HL[i], t[2 i + 1] = HH[i] (entry 8 = P itself)
void ghash_table(uint64_t ph, uint64_t pl, uint64_t *t) {
    uint64_t HL[16] = {}, HH[16] = {};
    uint64_t vh = ph, vl = pl;
    HL[8] = vl; HH[8] = vh;
    for (int i = 4; i > 0; i >>= 1) {
        const uint64_t T = (vl & 1) ? 0xe1000000ull : 0;
        vl = (vh << 63) | (vl >> 1);
        vh = (vh >> 1) ^ (T << 32);
        HL[i] = vl; HH[i] = vh;
    }
    for (int i = 2; i <= 8; i *= 2)
        for (int j = 1; j < i; ++j) {
            HH[i + j] = HH[i] ^ HH[j];
            HL[i + j] = HL[i] ^ HL[j];
        }
    for (int i = 0; i < 16; ++i) { t[2 * i] = HL[i]; t[2 * i + 1] = HH[i]; }
}
constexpr size_t kCrMisc = 0, kCrHdr = 64, kCrN = 192, kCrSum = 200, kCrRes = 256, kCrTab = 1024,
                 kCrTabBytes = (size_t)kGhPowers * 32 * 8, kCrArrays = kCrTab + kCrTabBytes;

// every scratch buffer a crypt enqueue of a record of up to len bytes uses, sized
// before the first enqueue of a sequence (a buffer grown between two enqueues of one
// stream order would be freed under the earlier one's kernels)
int crypt_reserve(iggy_codec_ctx *c, uint64_t len) {
    const uint64_t nmax = (len > kHdr ? (len - kHdr) / kFrameHdr : 0) + 1;
    const uint64_t ntiles = (nmax + kCryptTile - 1) / kCryptTile;
    const void *cr_before = c->cr.p;
    int r = c->cr.ensure(kCrArrays + (2 * nmax + ntiles + 2) * 8);
    if (c->cr.p != cr_before) c->cr_key_set = false;  // a grown buffer lost the tables
    r |= c->dpos.ensure((nmax + 1) * 8);
    r |= c->gbsums.ensure(((44 + 8 * nmax) / 1024 + 2) * 64);
    if (r) return IGGY_ERR_DEVICE;
    return ensure_decode_scratch(c, len);
}

int enqueue_crypt(iggy_codec_ctx *c, bool enc, const uint8_t *key, const uint8_t *d_record, uint64_t len,
                  const uint8_t *d_nonces, uint8_t *d_out, uint64_t cap, iggy_crypt_result *d_result, void *stream) {
    if (!c || !key || !d_record || !d_out || !d_result || (enc && !d_nonces)) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    hipStream_t s = bind(c, stream);
    const uint64_t nmax = (len > kHdr ? (len - kHdr) / kFrameHdr : 0) + 1;
    const uint64_t ntiles = (nmax + kCryptTile - 1) / kCryptTile;
    int r = crypt_reserve(c, len);
    if (r) return r;
    if (!c->cr_pinned && hipHostMalloc(&c->cr_pinned, kCrTabBytes, hipHostMallocDefault) != hipSuccess) {
        c->cr_pinned = nullptr;
        return IGGY_ERR_DEVICE;
    }
    CryptKey ck;
    aes256_key_schedule(key, ck.rk);
    uint8_t fp[32] = {};
    fp[16 + 15] = 1;
    aes256_block_host(ck.rk, fp, fp);            // E_K(0)
    aes256_block_host(ck.rk, fp + 16, fp + 16);  // E_K(1)
    if (!c->cr_key_set || memcmp(c->cr_fp, fp, 32) != 0) {
        // new key: H = E_K(0), tables of H^1 .. H^64 (the staging buffer is rewritten
        // only after every earlier upload on this stream order has run)
        HIP_OK(hipStreamSynchronize(s));
        uint8_t zero[16] = {}, hb[16];
        aes256_block_host(ck.rk, zero, hb);
        uint64_t hh = 0, hl = 0;
        for (int k = 0; k < 8; ++k) { hh = (hh << 8) | hb[k]; hl = (hl << 8) | hb[8 + k]; }
        uint64_t ph = hh, pl = hl;
        uint64_t *tab = (uint64_t *)c->cr_pinned;
        for (uint32_t e = 1; e <= kGhPowers; ++e) {
            ghash_table(ph, pl, tab + 32 * (e - 1));
            uint64_t nh, nl;
            gf128_mul(ph, pl, hh, hl, nh, nl);
            ph = nh; pl = nl;
        }
        HIP_OK(hipMemcpyAsync(c->cr.as<uint8_t>(kCrTab), c->cr_pinned, kCrTabBytes, hipMemcpyHostToDevice, s));
        memcpy(c->cr_fp, fp, 32);
        c->cr_key_set = true;
    }
    CryptScratch cs;
    iggy_decode_result *dres = c->cr.as<iggy_decode_result>(kCrRes);
    cs.dres = dres;
    cs.pos = c->dpos.as<uint64_t>();
    cs.osize = c->cr.as<uint64_t>(kCrArrays);
    cs.opos = cs.osize + nmax;
    cs.tsum = cs.opos + nmax;
    cs.misc = c->cr.as<uint64_t>(kCrMisc);
    cs.gtab = c->cr.as<uint64_t>(kCrTab);
    cs.dh = c->cr.as<iggy_batch_header>(kCrHdr);
    cs.dn = c->cr.as<uint64_t>(kCrN);
    cs.dsum = c->cr.as<uint64_t>(kCrSum);
    HIP_OK(hipMemsetAsync(cs.misc, 0, 64, s));
    r = enqueue_decode(c, d_record, len, enc ? IGGY_INTEGRITY_VERIFY : IGGY_INTEGRITY_LAYOUT_ONLY,
                       c->dpos.as<uint64_t>(), nmax, dres, s);
    if (r) return r;
    const uint32_t sg = (uint32_t)std::min<uint64_t>(ntiles, (uint64_t)c->ncu * 4);
    if (enc) {
        hipLaunchKernelGGL(k_crypt_sizes<true>, dim3(sg), dim3(256), 0, s, d_record, cs);
    } else {
        hipLaunchKernelGGL(k_crypt_sizes<false>, dim3(sg), dim3(256), 0, s, d_record, cs);
    }
    hipLaunchKernelGGL(k_crypt_scan, dim3(1), dim3(1024), 0, s, cs);
    if (enc) {
        hipLaunchKernelGGL(k_crypt_frames<true>, dim3(c->ncu * 8), dim3(256), kCryptLds, s, d_record, d_out, cap,
                           d_nonces, ck, cs);
    } else {
        hipLaunchKernelGGL(k_crypt_frames<false>, dim3(c->ncu * 8), dim3(256), kCryptLds, s, d_record, d_out, cap,
                           (const uint8_t *)nullptr, ck, cs);
    }
    hipLaunchKernelGGL(k_crypt_checksums, dim3(c->ncu * 16), dim3(256), 0, s, d_out, cap, cs);
    hipLaunchKernelGGL(k_crypt_header, dim3(1), dim3(64), 0, s, cap, cs);
    CsSource src{nullptr, d_out + kHdr, cs.opos};
    hipLaunchKernelGGL(k_bsum_blocks, dim3(bsum_grid(c, cap / 48 + 1)), dim3(256), 0, s, cs.dh, cs.dn, src,
                       c->gbsums.as<uint64_t>(), nullptr);
    hipLaunchKernelGGL(k_bsum_chain, dim3(1), dim3(128), 0, s, cs.dh, cs.dn, src,
                       (const uint64_t *)c->gbsums.as<uint64_t>(), c->dsync.as<uint8_t>(kSyncSmall), cs.dsum,
                       nullptr);
    if (enc) {
        hipLaunchKernelGGL(k_crypt_finish<true>, dim3(1), dim3(64), 0, s, d_record, len, d_out, cap, cs, d_result);
    } else {
        hipLaunchKernelGGL(k_crypt_finish<false>, dim3(1), dim3(64), 0, s, d_record, len, d_out, cap, cs, d_result);
    }
    HIP_OK(hipGetLastError());
    return 0;
}
}  // namespace

int iggy_codec_encrypt_batch_device(iggy_codec_ctx *c, const uint8_t *key, const uint8_t *d_record, uint64_t len,
                                    const uint8_t *d_nonces, uint8_t *d_out, uint64_t cap,
                                    iggy_crypt_result *d_result, void *stream) {
    return enqueue_crypt(c, true, key, d_record, len, d_nonces, d_out, cap, d_result, stream);
}

int iggy_codec_decrypt_batch_device(iggy_codec_ctx *c, const uint8_t *key, const uint8_t *d_record, uint64_t len,
                                    uint8_t *d_out, uint64_t cap, iggy_crypt_result *d_result, void *stream) {
    return enqueue_crypt(c, false, key, d_record, len, nullptr, d_out, cap, d_result, stream);
}

}  // extern "C"

/*
 * crypt_ref.c — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CPU restatement of Iggy's at-rest encryption re-encode:
 *   encrypt_batch_request / decrypt_batch_record
 *     (core/server_common/src/send_messages.rs:293-355, :357-415)
 *   Aes256GcmEncryptor::{encrypt, decrypt}
 *     (core/common/src/utils/crypto.rs:70-90): a section becomes
 *     nonce(12) || AES-256-GCM ciphertext || tag(16), empty associated data.
 * AES-256-GCM itself comes from the third-party crate `aes-gcm` (RustCrypto),
 * absent from /root/reference; it is restated here from FIPS-197 (AES, plain
 * byte-oriented rounds) and NIST SP 800-38D (GCM, 96-bit IV, bitwise GHASH
 * "Algorithm 1"), deliberately unlike the device's T-table / 4-bit-table
 * kernels. Pinned in tests/test_crypt_oracle.py against the system OpenSSL
 * (libcrypto EVP_aes_256_gcm, spec-identical) and the GCM spec's AES-256 test
 * cases 13-16. The reference draws nonces from the OS RNG; the oracle (like the
 * device API) takes them as input, 24 B per message: payload nonce, then the
 * user-headers nonce (used only when the message has user headers).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

/* ------------------------------------------------------------------ AES-256 */
static const uint8_t kSbox[256] = {
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

static uint8_t xtime(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }

/* FIPS-197 5.2 KeyExpansion, Nk = 8, Nr = 14: 240 bytes of round keys */
static void aes256_expand(const uint8_t key[32], uint8_t rk[240]) {
    memcpy(rk, key, 32);
    uint8_t rcon = 1;
    for (int i = 8; i < 60; ++i) {
        uint8_t t[4];
        memcpy(t, rk + 4 * (i - 1), 4);
        if (i % 8 == 0) {
            const uint8_t u = t[0];
            t[0] = (uint8_t)(kSbox[t[1]] ^ rcon);
            t[1] = kSbox[t[2]];
            t[2] = kSbox[t[3]];
            t[3] = kSbox[u];
            rcon = xtime(rcon);
        } else if (i % 8 == 4) {
            for (int k = 0; k < 4; ++k) t[k] = kSbox[t[k]];
        }
        for (int k = 0; k < 4; ++k) rk[4 * i + k] = (uint8_t)(rk[4 * (i - 8) + k] ^ t[k]);
    }
}

/* FIPS-197 5.1 Cipher: SubBytes, ShiftRows, MixColumns, AddRoundKey on a
 * column-major 4x4 byte state */
static void aes256_block(const uint8_t rk[240], const uint8_t in[16], uint8_t out[16]) {
    uint8_t s[16];
    for (int i = 0; i < 16; ++i) s[i] = (uint8_t)(in[i] ^ rk[i]);
    for (int r = 1; r <= 14; ++r) {
        uint8_t t[16];
        for (int i = 0; i < 16; ++i) t[i] = kSbox[s[i]];
        /* ShiftRows: row k of column c comes from column (c + k) mod 4 */
        for (int c = 0; c < 4; ++c)
            for (int k = 0; k < 4; ++k) s[4 * c + k] = t[4 * ((c + k) % 4) + k];
        if (r != 14) {
            for (int c = 0; c < 4; ++c) {
                uint8_t *a = s + 4 * c;
                const uint8_t a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3];
                const uint8_t all = (uint8_t)(a0 ^ a1 ^ a2 ^ a3);
                a[0] = (uint8_t)(a0 ^ all ^ xtime((uint8_t)(a0 ^ a1)));
                a[1] = (uint8_t)(a1 ^ all ^ xtime((uint8_t)(a1 ^ a2)));
                a[2] = (uint8_t)(a2 ^ all ^ xtime((uint8_t)(a2 ^ a3)));
                a[3] = (uint8_t)(a3 ^ all ^ xtime((uint8_t)(a3 ^ a0)));
            }
        }
        for (int i = 0; i < 16; ++i) s[i] ^= rk[16 * r + i];
    }
    memcpy(out, s, 16);
}

/* ------------------------------------------------------------------ GCM */
/* SP 800-38D 6.3 Algorithm 1: X * Y in GF(2^128), bit 0 = MSB of byte 0 */
static void gf_mult(const uint8_t x[16], const uint8_t y[16], uint8_t z[16]) {
    uint8_t v[16], r[16];
    memcpy(v, y, 16);
    memset(r, 0, 16);
    for (int i = 0; i < 128; ++i) {
        if ((x[i >> 3] >> (7 - (i & 7))) & 1)
            for (int k = 0; k < 16; ++k) r[k] ^= v[k];
        const int lsb = v[15] & 1;
        for (int k = 15; k > 0; --k) v[k] = (uint8_t)((v[k] >> 1) | (v[k - 1] << 7));
        v[0] >>= 1;
        if (lsb) v[0] ^= 0xe1;
    }
    memcpy(z, r, 16);
}

/* GHASH_H over the ciphertext (empty AAD) and the length block, XOR E_K(J0) */
static void gcm_tag(const uint8_t rk[240], const uint8_t iv[12], const uint8_t *ct, uint64_t n, uint8_t tag[16]) {
    uint8_t h[16] = {0}, y[16] = {0}, blk[16];
    aes256_block(rk, h, h);
    for (uint64_t off = 0; off < n; off += 16) {
        memset(blk, 0, 16);
        memcpy(blk, ct + off, n - off < 16 ? n - off : 16);
        for (int k = 0; k < 16; ++k) y[k] ^= blk[k];
        gf_mult(y, h, y);
    }
    memset(blk, 0, 16);
    const uint64_t bits = n * 8;
    for (int k = 0; k < 8; ++k) blk[15 - k] = (uint8_t)(bits >> (8 * k));
    for (int k = 0; k < 16; ++k) y[k] ^= blk[k];
    gf_mult(y, h, y);
    uint8_t j0[16], ek[16];
    memcpy(j0, iv, 12);
    j0[12] = 0; j0[13] = 0; j0[14] = 0; j0[15] = 1;
    aes256_block(rk, j0, ek);
    for (int k = 0; k < 16; ++k) tag[k] = (uint8_t)(y[k] ^ ek[k]);
}

/* GCTR from inc32(J0) (counter 2) */
static void gcm_ctr(const uint8_t rk[240], const uint8_t iv[12], const uint8_t *in, uint64_t n, uint8_t *out) {
    uint8_t cb[16], ks[16];
    memcpy(cb, iv, 12);
    uint32_t ctr = 2;
    for (uint64_t off = 0; off < n; off += 16, ++ctr) {
        cb[12] = (uint8_t)(ctr >> 24); cb[13] = (uint8_t)(ctr >> 16);
        cb[14] = (uint8_t)(ctr >> 8);  cb[15] = (uint8_t)ctr;
        aes256_block(rk, cb, ks);
        const uint64_t k = n - off < 16 ? n - off : 16;
        for (uint64_t i = 0; i < k; ++i) out[off + i] = (uint8_t)(in[off + i] ^ ks[i]);
    }
}

void oracle_aes256_block(const uint8_t key[32], const uint8_t in[16], uint8_t out[16]) {
    uint8_t rk[240];
    aes256_expand(key, rk);
    aes256_block(rk, in, out);
}

/* Aes256GcmEncryptor::encrypt with a given nonce: out = nonce || ct || tag (n + 28 B) */
void oracle_gcm_seal(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *pt, uint64_t n, uint8_t *out) {
    uint8_t rk[240];
    aes256_expand(key, rk);
    memcpy(out, nonce, 12);
    gcm_ctr(rk, nonce, pt, n, out + 12);
    gcm_tag(rk, nonce, out + 12, n, out + 12 + n);
}

/* Aes256GcmEncryptor::decrypt: data = nonce || ct || tag; 0 and n - 28 plaintext
 * bytes on success, -1 when the data is too short or the tag does not match */
int oracle_gcm_open(const uint8_t key[32], const uint8_t *data, uint64_t n, uint8_t *pt) {
    if (n < 12 + 16) return -1;  /* try_into of the nonce (< 12), or the AEAD (< 16 B after it) */
    uint8_t rk[240], tag[16];
    aes256_expand(key, rk);
    const uint64_t cn = n - 28;
    gcm_tag(rk, data, data + 12, cn, tag);
    if (memcmp(tag, data + 12 + cn, 16) != 0) return -1;
    gcm_ctr(rk, data, data + 12, cn, pt);
    return 0;
}

/* ------------------------------------------------------- batch re-encode */
static uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static void wr32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }
static void wr64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }

static void set_err(iggy_wire_error *e, uint32_t kind, uint64_t a, uint64_t b) {
    memset(e, 0, sizeof(*e));
    e->kind = kind;
    e->a = a;
    e->b = b;
}

/* One frame of the re-encoded blob (send_messages.rs:318-336 / :383-401): the 48-B
 * header with id, offset_delta and timestamp_delta kept, new lengths, reserved 0,
 * then the sections, then the checksum over frame[8..]. */
static uint64_t put_frame(uint8_t *dst, const uint8_t *src_hdr, const uint8_t *pl, uint64_t pl_len,
                          const uint8_t *uh, uint64_t uh_len) {
    memset(dst, 0, 48);
    memcpy(dst + 8, src_hdr + 8, 24); /* id (16), offset_delta (4), timestamp_delta (4) */
    wr32(dst + 32, (uint32_t)uh_len);
    wr32(dst + 36, (uint32_t)pl_len);
    if (pl_len && pl != dst + 48) memcpy(dst + 48, pl, pl_len);
    if (uh_len && uh != dst + 48 + pl_len) memcpy(dst + 48 + pl_len, uh, uh_len);
    const uint64_t size = 48 + pl_len + uh_len;
    wr64(dst, oracle_xxh3_64(dst + 8, size - 8));
    return size;
}

/* encrypt_batch_request's batch transform (send_messages.rs:307-355): Verify decode,
 * every payload (and non-empty user headers) sealed with its nonce, restamped.
 * out: [256 B header][blob]; *out_len its size. Returns 0 or an error (e). */
int oracle_encrypt_batch(const uint8_t key[32], const uint8_t *record, uint64_t len, const uint8_t *nonces,
                         uint8_t *out, uint64_t cap, uint64_t *out_len, iggy_wire_error *e) {
    iggy_batch_header h;
    uint64_t nframes = 0;
    const uint64_t fcap = len / 48 + 1;
    uint64_t *pos = (uint64_t *)malloc(fcap * 8);
    if (!pos) return IGGY_ERR_DEVICE;
    int r = oracle_decode_batch_slice_with(record, len, IGGY_INTEGRITY_VERIFY, &h, pos, fcap, &nframes, e);
    if (r) { free(pos); return r; }
    const uint8_t *blob = record + 256;
    uint64_t need = 256;
    for (uint64_t i = 0; i < nframes; ++i) {
        const uint8_t *f = blob + pos[i];
        const uint64_t uh = rd32(f + 32), pl = rd32(f + 36);
        if (pl + 28 > 0xffffffffull || (uh && uh + 28 > 0xffffffffull)) {  /* u32::try_from -> InvalidCommand */
            set_err(e, IGGY_ERR_INVALID_COMMAND, i, 0);
            free(pos);
            return IGGY_ERR_INVALID_COMMAND;
        }
        need += 48 + pl + 28 + (uh ? uh + 28 : 0);
    }
    if (need > cap) {
        set_err(e, IGGY_ERR_CAPACITY, need, cap);
        free(pos);
        return IGGY_ERR_CAPACITY;
    }
    uint8_t *ob = out + 256, *sec = NULL;
    uint64_t at = 0, seccap = 0;
    for (uint64_t i = 0; i < nframes; ++i) {
        const uint8_t *f = blob + pos[i];
        const uint64_t uh = rd32(f + 32), pl = rd32(f + 36);
        const uint64_t epl = pl + 28, euh = uh ? uh + 28 : 0;
        if (epl + euh > seccap) {
            seccap = 2 * (epl + euh);
            uint8_t *n2 = (uint8_t *)realloc(sec, seccap);
            if (!n2) { free(sec); free(pos); return IGGY_ERR_DEVICE; }
            sec = n2;
        }
        oracle_gcm_seal(key, nonces + 24 * i, f + 48, pl, sec);
        if (uh) oracle_gcm_seal(key, nonces + 24 * i + 12, f + 48 + pl, uh, sec + epl);
        at += put_frame(ob + at, f, sec, epl, sec + epl, euh);
    }
    free(sec);
    free(pos);
    h.batch_length = 256 + at;
    h.batch_checksum = oracle_calculate_batch_checksum(&h, ob, at);
    oracle_batch_header_encode(&h, out);
    *out_len = 256 + at;
    memset(e, 0, sizeof(*e));
    return 0;
}

/* decrypt_batch_record (send_messages.rs:369-415): LayoutOnly decode, the record
 * must be exactly batch_length bytes, every section opened in frame order. */
int oracle_decrypt_batch(const uint8_t key[32], const uint8_t *record, uint64_t len, uint8_t *out, uint64_t cap,
                         uint64_t *out_len, iggy_wire_error *e) {
    iggy_batch_header h;
    uint64_t nframes = 0;
    const uint64_t fcap = len / 48 + 1;
    uint64_t *pos = (uint64_t *)malloc(fcap * 8);
    if (!pos) return IGGY_ERR_DEVICE;
    int r = oracle_decode_batch_slice_with(record, len, IGGY_INTEGRITY_LAYOUT_ONLY, &h, pos, fcap, &nframes, e);
    if (r) { free(pos); return r; }
    if (len != h.batch_length) {
        set_err(e, IGGY_ERR_INVALID_COMMAND, len, h.batch_length);
        free(pos);
        return IGGY_ERR_INVALID_COMMAND;
    }
    const uint8_t *blob = record + 256;
    uint8_t *ob = out + 256;
    uint64_t at = 0;
    /* the output never exceeds the input: check capacity up front */
    if (cap < len) {
        set_err(e, IGGY_ERR_CAPACITY, len, cap);
        free(pos);
        return IGGY_ERR_CAPACITY;
    }
    for (uint64_t i = 0; i < nframes; ++i) {
        const uint8_t *f = blob + pos[i];
        const uint64_t uh = rd32(f + 32), pl = rd32(f + 36);
        uint8_t *dst = ob + at;
        /* plaintexts go straight to their places in the output frame */
        if (oracle_gcm_open(key, f + 48, pl, dst + 48) != 0) {
            set_err(e, IGGY_ERR_CANNOT_DECRYPT_DATA, i, 0);
            free(pos);
            return IGGY_ERR_CANNOT_DECRYPT_DATA;
        }
        const uint64_t dpl = pl - 28;
        uint64_t duh = 0;
        if (uh) {
            if (oracle_gcm_open(key, f + 48 + pl, uh, dst + 48 + dpl) != 0) {
                set_err(e, IGGY_ERR_CANNOT_DECRYPT_DATA, i, 1);
                free(pos);
                return IGGY_ERR_CANNOT_DECRYPT_DATA;
            }
            duh = uh - 28;
        }
        at += put_frame(dst, f, dst + 48, dpl, dst + 48 + dpl, duh);
    }
    free(pos);
    h.batch_length = 256 + at;
    h.batch_checksum = oracle_calculate_batch_checksum(&h, ob, at);
    oracle_batch_header_encode(&h, out);
    *out_len = 256 + at;
    memset(e, 0, sizeof(*e));
    return 0;
}

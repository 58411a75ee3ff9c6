// sdk.cpp — the SDK side of the path above the codec ABI (host code, no kernels of
// its own): the SendMessages request body around the GPU-encoded batch, the
// PollMessages response prefix, and the producer's buffering in front of the
// encoder. Everything device-side goes through the public entry points of
// codec_api.hip (iggy_codec_encode_batch / _submit, iggy_codec_poll_decode).
//
// Reference (apache/iggy):
//   core/binary_protocol/src/primitives/identifier.rs:97-231   WireIdentifier
//   core/binary_protocol/src/primitives/partitioning.rs:24-140 WirePartitioning
//   core/binary_protocol/src/requests/messages/send_messages.rs:65-241
//   core/common/src/types/message/polled_messages.rs:53-90
//   core/sdk/src/clients/producer_sharding.rs:91-293, producer.rs:406-470
//   core/message_bus/src/framing.rs:107-171 (socket framing)
//   core/server_common/src/send_messages.rs:459-540 (convert_request_message)
//   core/binary_protocol/src/batch.rs:98-150 (BatchHeader decode / encode_into)
//
// -DIGGY_HOST_ONLY builds the host-pure half alone (no HIP, no codec entry points:
// the functions that call the device are left out, staging memory is plain malloc)
// for the host sanitizer run of tests/test_sdk_fuzz_cpu.py (-fsanitize=address,undefined).
#ifndef IGGY_HOST_ONLY
#include <hip/hip_runtime.h>
#endif

#include <errno.h>
#include <stdlib.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/iggy_codec.h"

namespace {

void seterr(iggy_wire_error *e, uint32_t kind, uint32_t reason = 0, uint64_t a = 0, uint64_t b = 0,
            uint64_t c = 0) {
    if (e) *e = iggy_wire_error{kind, reason, a, b, c};
}

uint64_t have_from(uint64_t len, uint64_t off) { return len > off ? len - off : 0; }

// std::str::from_utf8 acceptance (RFC 3629: no overlongs, no surrogates, <= U+10FFFF)
bool utf8_ok(const uint8_t *s, uint64_t n) {
    uint64_t i = 0;
    while (i < n) {
        const uint8_t c = s[i];
        if (c < 0x80) { ++i; continue; }
        int k;
        uint8_t lo = 0x80, hi = 0xBF;
        if (c >= 0xC2 && c <= 0xDF) k = 1;
        else if (c == 0xE0) { k = 2; lo = 0xA0; }
        else if (c >= 0xE1 && c <= 0xEC) k = 2;
        else if (c == 0xED) { k = 2; hi = 0x9F; }
        else if (c >= 0xEE && c <= 0xEF) k = 2;
        else if (c == 0xF0) { k = 3; lo = 0x90; }
        else if (c >= 0xF1 && c <= 0xF3) k = 3;
        else if (c == 0xF4) { k = 3; hi = 0x8F; }
        else return false;
        if (n - i <= (uint64_t)k) return false;
        if (s[i + 1] < lo || s[i + 1] > hi) return false;
        for (int j = 2; j <= k; ++j)
            if (s[i + j] < 0x80 || s[i + j] > 0xBF) return false;
        i += k + 1;
    }
    return true;
}

// what the Rust constructors guarantee (WireIdentifier::numeric / named, WireName::new
// identifier.rs:18-28, WirePartitioning::messages_key partitioning.rs:26-40)
bool id_valid(const iggy_identifier &id) {
    if (id.kind == IGGY_ID_NUMERIC) return id.length == 4;
    if (id.kind == IGGY_ID_STRING) return id.length >= 1 && id.length <= 255 && utf8_ok(id.value, id.length);
    return false;
}
bool part_valid(const iggy_partitioning &p) {
    if (p.kind == IGGY_PART_BALANCED) return p.length == 0;
    if (p.kind == IGGY_PART_PARTITION_ID) return p.length == 4;
    if (p.kind == IGGY_PART_MESSAGES_KEY) return p.length >= 1 && p.length <= 255;
    return false;
}
// WireEncode::encoded_size (identifier.rs:158-160, partitioning.rs:44-50): kind, length, value
uint64_t field_size(uint32_t length) { return 2 + (uint64_t)length; }

uint8_t *put_field(uint8_t *o, uint32_t kind, uint32_t length, const uint8_t *value) {
    *o++ = (uint8_t)kind;
    *o++ = (uint8_t)length;
    memcpy(o, value, length);
    return o + length;
}

void put_u32(uint8_t *o, uint32_t v) { memcpy(o, &v, 4); }

uint64_t metadata_length(const iggy_send_messages_header &h) {  // send_messages.rs:201-206
    return field_size(h.stream_id.length) + field_size(h.topic_id.length) + field_size(h.partitioning.length) + 4;
}

// WireIdentifier::decode (identifier.rs:194-231) on buf[0..len) (a sub-slice: offsets are relative)
int decode_identifier(const uint8_t *buf, uint64_t len, iggy_identifier *out, uint64_t *consumed,
                      iggy_wire_error *err) {
    if (len < 1) { seterr(err, IGGY_ERR_UNEXPECTED_EOF, 0, 0, 1, 0); return IGGY_ERR_UNEXPECTED_EOF; }
    const uint32_t kind = buf[0];
    if (len < 2) { seterr(err, IGGY_ERR_UNEXPECTED_EOF, 0, 1, 1, 0); return IGGY_ERR_UNEXPECTED_EOF; }
    const uint32_t length = buf[1];
    if (len - 2 < length) {
        seterr(err, IGGY_ERR_UNEXPECTED_EOF, 0, 2, length, len - 2);
        return IGGY_ERR_UNEXPECTED_EOF;
    }
    const uint8_t *value = buf + 2;
    if (kind == IGGY_ID_NUMERIC) {
        if (length != 4) {
            seterr(err, IGGY_ERR_VALIDATION, IGGY_V_NUMERIC_ID_LENGTH, length);
            return IGGY_ERR_VALIDATION;
        }
    } else if (kind == IGGY_ID_STRING) {
        if (length == 0) {
            seterr(err, IGGY_ERR_VALIDATION, IGGY_V_STRING_ID_EMPTY);
            return IGGY_ERR_VALIDATION;
        }
        if (!utf8_ok(value, length)) {
            seterr(err, IGGY_ERR_INVALID_UTF8, 0, 2);
            return IGGY_ERR_INVALID_UTF8;
        }
    } else {
        seterr(err, IGGY_ERR_UNKNOWN_DISCRIMINANT, 0, IGGY_TYPE_WIRE_IDENTIFIER, kind, 0);
        return IGGY_ERR_UNKNOWN_DISCRIMINANT;
    }
    memset(out, 0, sizeof(*out));
    out->kind = kind;
    out->length = length;
    memcpy(out->value, value, length);
    *consumed = 2 + (uint64_t)length;
    return 0;
}

// WirePartitioning::decode (partitioning.rs:106-140): the kind decides before any value read
int decode_partitioning(const uint8_t *buf, uint64_t len, iggy_partitioning *out, uint64_t *consumed,
                        iggy_wire_error *err) {
    if (len < 1) { seterr(err, IGGY_ERR_UNEXPECTED_EOF, 0, 0, 1, 0); return IGGY_ERR_UNEXPECTED_EOF; }
    const uint32_t kind = buf[0];
    if (len < 2) { seterr(err, IGGY_ERR_UNEXPECTED_EOF, 0, 1, 1, 0); return IGGY_ERR_UNEXPECTED_EOF; }
    const uint32_t length = buf[1];
    memset(out, 0, sizeof(*out));
    out->kind = kind;
    if (kind == IGGY_PART_BALANCED) {
        if (length != 0) {
            seterr(err, IGGY_ERR_VALIDATION, IGGY_V_BALANCED_LENGTH, length);
            return IGGY_ERR_VALIDATION;
        }
        *consumed = 2;
        return 0;
    }
    if (kind == IGGY_PART_PARTITION_ID) {
        if (length != 4) {
            seterr(err, IGGY_ERR_VALIDATION, IGGY_V_PARTITION_ID_LENGTH, length);
            return IGGY_ERR_VALIDATION;
        }
        if (len - 2 < 4) {
            seterr(err, IGGY_ERR_UNEXPECTED_EOF, 0, 2, 4, len - 2);
            return IGGY_ERR_UNEXPECTED_EOF;
        }
        out->length = 4;
        memcpy(out->value, buf + 2, 4);
        *consumed = 6;
        return 0;
    }
    if (kind == IGGY_PART_MESSAGES_KEY) {
        if (length == 0) {
            seterr(err, IGGY_ERR_VALIDATION, IGGY_V_MESSAGES_KEY_EMPTY);
            return IGGY_ERR_VALIDATION;
        }
        if (len - 2 < length) {
            seterr(err, IGGY_ERR_UNEXPECTED_EOF, 0, 2, length, len - 2);
            return IGGY_ERR_UNEXPECTED_EOF;
        }
        out->length = length;
        memcpy(out->value, buf + 2, length);
        *consumed = 2 + (uint64_t)length;
        return 0;
    }
    seterr(err, IGGY_ERR_UNKNOWN_DISCRIMINANT, 0, IGGY_TYPE_WIRE_PARTITIONING, kind, 0);
    return IGGY_ERR_UNKNOWN_DISCRIMINANT;
}

bool same_field(uint32_t k1, uint32_t l1, const uint8_t *v1, uint32_t k2, uint32_t l2, const uint8_t *v2) {
    return k1 == k2 && l1 == l2 && memcmp(v1, v2, l1) == 0;
}

// page-locked host array that grows by doubling (the flush's H2D copies are DMA)
template <class T>
struct Pinned {
    T *p = nullptr;
    uint64_t n = 0, cap = 0;
    ~Pinned() { release(p); }
    static void release(void *q) {
#ifdef IGGY_HOST_ONLY
        free(q);
#else
        if (q) (void)hipHostFree(q);
#endif
    }
    bool reserve(uint64_t want) {
        if (want <= cap) return true;
        uint64_t nc = cap ? cap : 4096 / sizeof(T) + 1;
        while (nc < want) nc *= 2;
        void *q = nullptr;
#ifdef IGGY_HOST_ONLY
        if (!(q = malloc(nc * sizeof(T)))) return false;
#else
        if (hipHostMalloc(&q, nc * sizeof(T), hipHostMallocDefault) != hipSuccess) return false;
#endif
        if (n) memcpy(q, p, n * sizeof(T));
        release(p);
        p = (T *)q;
        cap = nc;
        return true;
    }
    bool append(const T *src, uint64_t k) {
        if (!reserve(n + k)) return false;
        if (k) memcpy(p + n, src, k * sizeof(T));
        n += k;
        return true;
    }
    bool append_zero(uint64_t k) {
        if (!reserve(n + k)) return false;
        memset(p + n, 0, k * sizeof(T));
        n += k;
        return true;
    }
};

}  // namespace

// one ShardMessage of the buffer: its destination and its messages in the staging
struct ProducerEntry {
    iggy_identifier stream, topic;
    iggy_partitioning part;
    uint64_t m0, m1;        // message index range
    uint64_t pay0, uh0;     // byte offsets of its first payload / user-header byte
};

struct iggy_producer {
    iggy_codec_ctx *ctx;
    iggy_producer_config cfg;
    std::vector<ProducerEntry> entries;
    uint64_t bytes = 0;  // ShardMessage::get_size_bytes summed (producer_sharding.rs:155)
    Pinned<uint64_t> ids, ots;
    Pinned<uint32_t> plen, uhl;
    Pinned<uint8_t> pay, uh;
    bool any_uh = false;
};

namespace {

// Remove messages [0, upto) (whole flushed requests) from the staging: the arrays
// keep their tails, the entries are rebased, fully flushed entries disappear.
void drop_flushed(iggy_producer *p, uint64_t upto) {
    const uint64_t N = p->ids.n / 2;
    if (upto >= N) {
        p->entries.clear();
        p->bytes = 0;
        p->ids.n = p->ots.n = p->plen.n = p->uhl.n = p->pay.n = p->uh.n = 0;
        p->any_uh = false;
        return;
    }
    uint64_t pay_cut = 0, uh_cut = 0;
    for (uint64_t i = 0; i < upto; ++i) {
        pay_cut += p->plen.p[i];
        uh_cut += p->uhl.p[i];
    }
    auto shift = [](auto &a, uint64_t cut) {
        memmove(a.p, a.p + cut, (a.n - cut) * sizeof(*a.p));
        a.n -= cut;
    };
    shift(p->ids, 2 * upto);
    shift(p->ots, upto);
    shift(p->plen, upto);
    shift(p->uhl, upto);
    shift(p->pay, pay_cut);
    shift(p->uh, uh_cut);
    std::vector<ProducerEntry> keep;
    uint64_t bytes = 0;
    for (ProducerEntry e : p->entries) {
        if (e.m1 <= upto) continue;
        const uint64_t m0 = std::max(e.m0, upto);
        e.m0 = m0 - upto;
        e.m1 -= upto;
        uint64_t spl = 0, suh = 0;
        for (uint64_t i = e.m0; i < e.m1; ++i) {
            spl += p->plen.p[i];
            suh += p->uhl.p[i];
        }
        bytes += (2 + (uint64_t)e.stream.length) + (2 + (uint64_t)e.topic.length) + 64 * (e.m1 - e.m0) + spl + suh;
        keep.push_back(e);
    }
    uint64_t pay0 = 0, uh0 = 0, i = 0;
    for (ProducerEntry &e : keep) {  // byte offsets of the kept entries
        for (; i < e.m0; ++i) { pay0 += p->plen.p[i]; uh0 += p->uhl.p[i]; }
        e.pay0 = pay0;
        e.uh0 = uh0;
    }
    p->entries.swap(keep);
    p->bytes = bytes;
}

}  // namespace

extern "C" {

// ------------------------------------------------------------ batch header (host pure)
// BatchHeader::decode (batch.rs:98-134): EOF below 256 B, batch_length < 256 before
// the reserved bytes 52..256 (which must be zero)
int iggy_batch_header_decode(const uint8_t *b, uint64_t len, iggy_batch_header *h, iggy_wire_error *err) {
    seterr(err, IGGY_OK);
    if (!b && len) return IGGY_ERR_INVALID_ARGUMENT;
    if (len < 256) {
        seterr(err, IGGY_ERR_UNEXPECTED_EOF, 0, 0, 256, len);
        return IGGY_ERR_UNEXPECTED_EOF;
    }
    uint64_t bl;
    memcpy(&bl, b + 32, 8);
    if (bl < 256) {
        seterr(err, IGGY_ERR_VALIDATION, IGGY_V_BATCH_LENGTH_SHORT);
        return IGGY_ERR_VALIDATION;
    }
    for (int i = 52; i < 256; ++i)
        if (b[i]) {
            seterr(err, IGGY_ERR_VALIDATION, IGGY_V_BATCH_RESERVED);
            return IGGY_ERR_VALIDATION;
        }
    if (h) {
        memset(h, 0, sizeof(*h));
        memcpy(&h->partition_id, b + 0, 8);
        memcpy(&h->base_offset, b + 8, 8);
        memcpy(&h->base_timestamp, b + 16, 8);
        memcpy(&h->origin_timestamp, b + 24, 8);
        h->batch_length = bl;
        memcpy(&h->batch_checksum, b + 40, 8);
        memcpy(&h->message_count, b + 48, 4);
    }
    return 0;
}

// BatchHeader::encode_into (batch.rs:138-150)
void iggy_batch_header_encode(const iggy_batch_header *h, uint8_t out[256]) {
    memset(out, 0, 256);
    memcpy(out + 0, &h->partition_id, 8);
    memcpy(out + 8, &h->base_offset, 8);
    memcpy(out + 16, &h->base_timestamp, 8);
    memcpy(out + 24, &h->origin_timestamp, 8);
    memcpy(out + 32, &h->batch_length, 8);
    memcpy(out + 40, &h->batch_checksum, 8);
    memcpy(out + 48, &h->message_count, 4);
}

uint64_t iggy_encoded_batch_size(const iggy_raw_messages *m) {
    if (!m) return 0;
    uint64_t t = 256;
    for (uint64_t i = 0; i < m->count; ++i)
        t += 48 + (uint64_t)m->payload_lengths[i] + (m->user_headers_lengths ? m->user_headers_lengths[i] : 0);
    return t;
}

int iggy_send_messages_header_encode(const iggy_send_messages_header *h, uint8_t *out, uint64_t cap,
                                     uint64_t *out_len) {
    if (!h || !id_valid(h->stream_id) || !id_valid(h->topic_id) || !part_valid(h->partitioning))
        return IGGY_ERR_INVALID_ARGUMENT;
    const uint64_t need = metadata_length(*h);
    if (out_len) *out_len = need;
    if (!out || cap < need) return IGGY_ERR_CAPACITY;
    uint8_t *o = put_field(out, h->stream_id.kind, h->stream_id.length, h->stream_id.value);
    o = put_field(o, h->topic_id.kind, h->topic_id.length, h->topic_id.value);
    o = put_field(o, h->partitioning.kind, h->partitioning.length, h->partitioning.value);
    put_u32(o, h->messages_count);
    return 0;
}

int iggy_send_messages_header_decode(const uint8_t *buf, uint64_t len, iggy_send_messages_header *out,
                                     uint64_t *consumed, iggy_wire_error *err) {
    if (!out || (!buf && len)) return IGGY_ERR_INVALID_ARGUMENT;
    seterr(err, IGGY_OK);
    iggy_send_messages_header h;
    memset(&h, 0, sizeof(h));
    uint64_t pos = 0, used = 0;
    int r = decode_identifier(buf, len, &h.stream_id, &used, err);
    if (r) return r;
    pos += used;
    r = decode_identifier(buf + pos, len - pos, &h.topic_id, &used, err);
    if (r) return r;
    pos += used;
    r = decode_partitioning(buf + pos, len - pos, &h.partitioning, &used, err);
    if (r) return r;
    pos += used;
    if (len - pos < 4) {  // read_u32_le(buf, pos): offset relative to the whole metadata
        seterr(err, IGGY_ERR_UNEXPECTED_EOF, 0, pos, 4, have_from(len, pos));
        return IGGY_ERR_UNEXPECTED_EOF;
    }
    memcpy(&h.messages_count, buf + pos, 4);
    pos += 4;
    *out = h;
    if (consumed) *consumed = pos;
    return 0;
}

uint64_t iggy_send_messages_encoded_size(const iggy_send_messages_header *h, const iggy_raw_messages *m) {
    if (!h || !m) return 0;
    return 4 + metadata_length(*h) + iggy_encoded_batch_size(m);
}

#ifndef IGGY_HOST_ONLY
int iggy_codec_send_messages_encode(iggy_codec_ctx *ctx, const iggy_send_messages_header *h,
                                    const iggy_raw_messages *m, uint8_t *out, uint64_t cap, uint64_t *out_len,
                                    iggy_wire_error *err) {
    if (!ctx || !h || !m) return IGGY_ERR_INVALID_ARGUMENT;
    seterr(err, IGGY_OK);
    if (m->count == 0) {  // send_messages.rs:96-100, before any byte is written
        seterr(err, IGGY_ERR_VALIDATION, IGGY_V_EMPTY_BATCH);
        return IGGY_ERR_VALIDATION;
    }
    if (m->count > 0xFFFFFFFFull) {  // :112-116
        seterr(err, IGGY_ERR_PAYLOAD_TOO_LARGE, 0, m->count, 0xFFFFFFFFull);
        return IGGY_ERR_PAYLOAD_TOO_LARGE;
    }
    iggy_send_messages_header hh = *h;
    hh.messages_count = (uint32_t)m->count;
    const uint64_t meta = metadata_length(hh);
    const uint64_t need = 4 + meta + iggy_encoded_batch_size(m);
    if (!out || cap < need) {
        seterr(err, IGGY_ERR_CAPACITY, 0, need, cap);
        return IGGY_ERR_CAPACITY;
    }
    put_u32(out, (uint32_t)meta);
    int r = iggy_send_messages_header_encode(&hh, out + 4, meta, nullptr);
    if (r) return r;
    uint64_t blen = 0;
    r = iggy_codec_encode_batch(ctx, m, 0, out + 4 + meta, cap - 4 - meta, &blen, err);
    if (r) return r;
    if (out_len) *out_len = 4 + meta + blen;
    return 0;
}

int iggy_codec_polled_messages_from_bytes(iggy_codec_ctx *ctx, const uint8_t *bytes, uint64_t len,
                                          iggy_polled_prefix *prefix, iggy_polled_message *out, uint64_t cap,
                                          uint64_t *n, iggy_wire_error *err) {
    if (!ctx || (!bytes && len)) return IGGY_ERR_INVALID_ARGUMENT;
    seterr(err, IGGY_OK);
    if (n) *n = 0;
    if (len < 16) {  // polled_messages.rs:62-64
        seterr(err, IGGY_ERR_INVALID_NUMBER_ENCODING);
        return IGGY_ERR_INVALID_NUMBER_ENCODING;
    }
    iggy_polled_prefix pf;
    memcpy(&pf.partition_id, bytes, 4);
    memcpy(&pf.current_offset, bytes + 4, 8);
    memcpy(&pf.count, bytes + 12, 4);
    if (prefix) *prefix = pf;
    uint64_t k = 0;
    const int r = iggy_codec_poll_decode(ctx, bytes + 16, len - 16, IGGY_POLL_MODE_SDK, out, cap, &k, err);
    for (uint64_t i = 0; i < k; ++i) {  // views into the response buffer (Bytes::slice, :133-138)
        out[i].payload_pos += 16;
        out[i].user_headers_pos += 16;
    }
    if (n) *n = k;
    return r;
}

#endif  // IGGY_HOST_ONLY

// ------------------------------------------------------------------- producer
int iggy_producer_create(iggy_codec_ctx *ctx, const iggy_producer_config *cfg, iggy_producer **out) {
    if (!ctx || !cfg || !out) return IGGY_ERR_INVALID_ARGUMENT;
    iggy_producer *p = new (std::nothrow) iggy_producer();
    if (!p) return IGGY_ERR_DEVICE;
    p->ctx = ctx;
    p->cfg = *cfg;
    *out = p;
    return 0;
}

void iggy_producer_destroy(iggy_producer *p) { delete p; }

int iggy_producer_pending(const iggy_producer *p, uint64_t *entries, uint64_t *bytes, uint64_t *messages) {
    if (!p) return IGGY_ERR_INVALID_ARGUMENT;
    if (entries) *entries = p->entries.size();
    if (bytes) *bytes = p->bytes;
    if (messages) *messages = p->ids.n / 2;
    return 0;
}

int iggy_producer_append(iggy_producer *p, const iggy_identifier *stream_id, const iggy_identifier *topic_id,
                         const iggy_partitioning *part, const iggy_raw_messages *m, int *flush_due) {
    if (!p || !stream_id || !topic_id || !part || !m) return IGGY_ERR_INVALID_ARGUMENT;
    if (!id_valid(*stream_id) || !id_valid(*topic_id) || !part_valid(*part)) return IGGY_ERR_INVALID_ARGUMENT;
    if (m->count && (!m->ids || !m->origin_timestamps || !m->payload_lengths)) return IGGY_ERR_INVALID_ARGUMENT;
    const uint64_t n = m->count;
    uint64_t spl = 0, suh = 0;
    for (uint64_t i = 0; i < n; ++i) {
        spl += m->payload_lengths[i];
        suh += m->user_headers_lengths ? m->user_headers_lengths[i] : 0;
    }
    if ((spl && !m->payloads) || (suh && !m->user_headers)) return IGGY_ERR_INVALID_ARGUMENT;
    ProducerEntry e;
    e.stream = *stream_id;
    e.topic = *topic_id;
    e.part = *part;
    e.m0 = p->ids.n / 2;
    e.m1 = e.m0 + n;
    e.pay0 = p->pay.n;
    e.uh0 = p->uh.n;
    // every staging array is grown first; the entry is appended only once all six
    // reservations succeeded, so a failed allocation leaves the buffer as it was
    const bool has_uh = m->user_headers_lengths != nullptr;
    if (!p->ids.reserve(p->ids.n + 2 * n) || !p->ots.reserve(p->ots.n + n) || !p->plen.reserve(p->plen.n + n) ||
        !p->pay.reserve(p->pay.n + spl) || !p->uhl.reserve(p->uhl.n + n) || !p->uh.reserve(p->uh.n + suh))
        return IGGY_ERR_DEVICE;
    p->ids.append(m->ids, 2 * n);
    p->ots.append(m->origin_timestamps, n);
    p->plen.append(m->payload_lengths, n);
    p->pay.append(m->payloads, spl);
    if (has_uh) {
        p->uhl.append(m->user_headers_lengths, n);
        p->uh.append(m->user_headers, suh);
        p->any_uh = p->any_uh || suh > 0;
    } else {
        p->uhl.append_zero(n);
    }
    p->entries.push_back(e);
    // ShardMessage::get_size_bytes (producer_sharding.rs:99-109; Identifier: length + 2,
    // common/src/types/identifier/mod.rs:206-210; IggyMessage: 64 + payload + user headers,
    // iggy_message.rs:471-491 with IGGY_MESSAGE_HEADER_SIZE = 64, message_header.rs:23)
    p->bytes += (2 + (uint64_t)stream_id->length) + (2 + (uint64_t)topic_id->length) + 64 * n + spl + suh;
    if (flush_due) {
        if (p->cfg.direct) {
            *flush_due = 1;
        } else {
            const bool by_len = p->cfg.batch_length != 0 && p->entries.size() >= p->cfg.batch_length;
            const bool by_size = p->cfg.batch_size != 0 && p->bytes >= p->cfg.batch_size;
            *flush_due = (by_len || by_size) ? 1 : 0;
        }
    }
    return 0;
}

#ifndef IGGY_HOST_ONLY
int iggy_producer_flush(iggy_producer *p, uint8_t *out, uint64_t cap, iggy_producer_request *reqs,
                        uint64_t max_reqs, uint64_t *nreqs, iggy_wire_error *err) {
    if (!p || (!out && cap) || (!reqs && max_reqs)) return IGGY_ERR_INVALID_ARGUMENT;
    seterr(err, IGGY_OK);
    if (nreqs) *nreqs = 0;
    // 1. the requests: background = runs of same-destination entries merged
    //    (flush_buffer, producer_sharding.rs:226-235); direct = each entry split into
    //    chunks of batch_length (or MAX_BATCH_LENGTH) messages (producer.rs:433-455)
    struct Plan {
        uint32_t entry;
        uint64_t m0, m1;
    };
    std::vector<Plan> plan;
    const size_t E = p->entries.size();
    if (p->cfg.direct) {
        const uint64_t mx = p->cfg.batch_length ? p->cfg.batch_length : IGGY_MAX_BATCH_LENGTH;
        for (size_t k = 0; k < E; ++k) {
            const ProducerEntry &e = p->entries[k];
            for (uint64_t a = e.m0; a < e.m1; a += mx) plan.push_back({(uint32_t)k, a, std::min(a + mx, e.m1)});
        }
    } else {
        for (size_t k = 0; k < E; ++k) {
            const ProducerEntry &e = p->entries[k];
            if (!plan.empty()) {
                const ProducerEntry &l = p->entries[plan.back().entry];
                if (same_field(l.stream.kind, l.stream.length, l.stream.value, e.stream.kind, e.stream.length,
                               e.stream.value) &&
                    same_field(l.topic.kind, l.topic.length, l.topic.value, e.topic.kind, e.topic.length,
                               e.topic.value) &&
                    same_field(l.part.kind, l.part.length, l.part.value, e.part.kind, e.part.length, e.part.value)) {
                    plan.back().m1 = e.m1;  // consecutive entries: contiguous in the staging
                    continue;
                }
            }
            plan.push_back({(uint32_t)k, e.m0, e.m1});
        }
    }
    // send_internal returns at once for an empty message list (producer.rs:413-415)
    std::vector<Plan> sendable;
    for (const Plan &q : plan)
        if (q.m1 > q.m0) sendable.push_back(q);
    // 2. sizes: prefix sums of payload / user-header bytes per message
    const uint64_t N = p->ids.n / 2;
    std::vector<uint64_t> pfx_pay(N + 1, 0), pfx_uh(N + 1, 0);
    for (uint64_t i = 0; i < N; ++i) {
        pfx_pay[i + 1] = pfx_pay[i] + p->plen.p[i];
        pfx_uh[i + 1] = pfx_uh[i] + p->uhl.p[i];
    }
    std::vector<uint64_t> off(sendable.size() + 1, 0), meta(sendable.size());
    for (size_t r = 0; r < sendable.size(); ++r) {
        const Plan &q = sendable[r];
        const ProducerEntry &e = p->entries[q.entry];
        meta[r] = field_size(e.stream.length) + field_size(e.topic.length) + field_size(e.part.length) + 4;
        const uint64_t n = q.m1 - q.m0;
        off[r + 1] = off[r] + 4 + meta[r] + 256 + 48 * n + (pfx_pay[q.m1] - pfx_pay[q.m0]) +
                     (pfx_uh[q.m1] - pfx_uh[q.m0]);
    }
    if (sendable.size() > max_reqs) {
        seterr(err, IGGY_ERR_CAPACITY, 0, sendable.size(), max_reqs);
        return IGGY_ERR_CAPACITY;
    }
    if (off.back() > cap) {
        seterr(err, IGGY_ERR_CAPACITY, 0, off.back(), cap);
        return IGGY_ERR_CAPACITY;
    }
    // 3. metadata on the host, batch sections on the GPU (up to the context's slots in
    //    flight; a full set retires its oldest request)
    std::vector<iggy_ticket> tick(sendable.size(), 0);
    std::vector<uint8_t> live(sendable.size(), 0);
    // every request slot this flush may report is cleared first: a caller reusing its
    // array from an earlier flush must not see a stale `sent` past a failure
    if (!sendable.empty()) memset(reqs, 0, sendable.size() * sizeof(iggy_producer_request));
    size_t oldest = 0;
    int rc = 0;
    auto retire = [&](size_t r) -> int {
        iggy_completion c;
        const int w = iggy_codec_wait(p->ctx, tick[r], &c);
        live[r] = 0;
        if (w) {
            reqs[r].sent = 0;  // no verdict: the request is not complete and is not reported
            return w;
        }
        reqs[r].error = c.error;
        return 0;
    };
    for (size_t r = 0; r < sendable.size() && !rc; ++r) {
        const Plan &q = sendable[r];
        const ProducerEntry &e = p->entries[q.entry];
        iggy_producer_request &rq = reqs[r];
        memset(&rq, 0, sizeof(rq));
        rq.offset = off[r];
        rq.length = off[r + 1] - off[r];
        rq.first_message = q.m0;
        rq.messages = q.m1 - q.m0;
        rq.entry = q.entry;
        uint8_t *o = out + off[r];
        put_u32(o, (uint32_t)meta[r]);
        o = put_field(o + 4, e.stream.kind, e.stream.length, e.stream.value);
        o = put_field(o, e.topic.kind, e.topic.length, e.topic.value);
        o = put_field(o, e.part.kind, e.part.length, e.part.value);
        put_u32(o, (uint32_t)rq.messages);
        o += 4;
        iggy_raw_messages m;
        m.count = rq.messages;
        m.ids = p->ids.p + 2 * q.m0;
        m.origin_timestamps = p->ots.p + q.m0;
        m.payloads = p->pay.p + pfx_pay[q.m0];
        m.payload_lengths = p->plen.p + q.m0;
        m.user_headers = p->any_uh ? p->uh.p + pfx_uh[q.m0] : nullptr;
        m.user_headers_lengths = p->any_uh ? p->uhl.p + q.m0 : nullptr;
        while (true) {
            const int s = iggy_codec_encode_submit(p->ctx, &m, 0, o, off[r + 1] - (uint64_t)(o - out), &tick[r]);
            if (s == IGGY_ERR_BUSY) {
                while (oldest < r && !live[oldest]) ++oldest;
                // every slot is held by other operations of the context: the caller's
                // own submits must drain first (not a device failure)
                if (oldest >= r) { rc = IGGY_ERR_BUSY; break; }
                rc = retire(oldest++);
                if (rc) break;
                continue;
            }
            if (s) rc = s;
            break;
        }
        if (rc) break;
        live[r] = 1;
        rq.sent = 1;
    }
    for (size_t r = 0; r < sendable.size(); ++r) {
        if (live[r]) {
            const int w = retire(r);
            if (!rc) rc = w;
        }
    }
    // requests encoded AND retired with a verdict: the prefix up to the first that is
    // not (submission stops at the first failure; a failed wait clears its request)
    size_t nsent = 0;
    while (nsent < sendable.size() && reqs[nsent].sent) ++nsent;
    // direct sends: the chunks after a failed one were never sent (producer.rs:446-452)
    if (!rc && p->cfg.direct)
        for (size_t r = 1; r < sendable.size(); ++r) {
            const iggy_producer_request &pr = reqs[r - 1];
            if (sendable[r].entry == sendable[r - 1].entry && (pr.error.kind != IGGY_OK || !pr.sent)) {
                reqs[r].sent = 0;
                reqs[r].error = iggy_wire_error{};
            }
        }
    if (rc) {
        // A submit or wait failed part-way: reqs[0..nsent) are written (each with its
        // own verdict) and must be sent by the caller; they leave the buffer, which keeps
        // only the messages of the requests after them, so a retry never re-sends one.
        for (size_t r = nsent; r < sendable.size(); ++r) reqs[r].sent = 0;  // staged again, not reported
        if (nreqs) *nreqs = nsent;
        if (nsent) drop_flushed(p, sendable[nsent - 1].m1);
        return rc;
    }
    if (nreqs) *nreqs = sendable.size();
    drop_flushed(p, N);
    return 0;
}

#endif  // IGGY_HOST_ONLY


// ---------------------------------------------------------- server socket side
// read_exact on a blocking stream socket (compio's read_exact: EOF before the
// requested bytes -> UnexpectedEof)
static int read_exact_fd(int fd, uint8_t *p, uint64_t n) {
    uint64_t got = 0;
    while (got < n) {
        const ssize_t r = read(fd, p + got, n - got);
        if (r > 0) {
            got += (uint64_t)r;
            continue;
        }
        if (r == 0) return IGGY_ERR_CONNECTION_CLOSED;  // framing.rs:165-171 to_read_error
        if (errno == EINTR) continue;
        return IGGY_ERR_TCP_ERROR;
    }
    return 0;
}

int iggy_frame_read(int fd, uint8_t *buf, uint64_t cap, uint64_t max_message_size, uint64_t *total_size,
                    iggy_wire_error *err) {
    if (fd < 0 || !buf || !total_size) return IGGY_ERR_INVALID_ARGUMENT;
    seterr(err, IGGY_OK);
    *total_size = 0;
    if (cap < IGGY_FRAME_HEADER_BYTES) {
        seterr(err, IGGY_ERR_CAPACITY, 0, IGGY_FRAME_HEADER_BYTES);
        return IGGY_ERR_CAPACITY;
    }
    // stage 1: the fixed header (framing.rs:114-116)
    int r = read_exact_fd(fd, buf, IGGY_FRAME_HEADER_BYTES);
    if (r) {
        seterr(err, (uint32_t)r);
        return r;
    }
    uint32_t size;  // read_size_field (consensus/header.rs:73-78)
    memcpy(&size, buf + IGGY_FRAME_SIZE_OFFSET, 4);
    if (size < IGGY_FRAME_HEADER_BYTES || size > max_message_size) {  // framing.rs:120-122
        seterr(err, IGGY_ERR_INVALID_COMMAND);
        return IGGY_ERR_INVALID_COMMAND;
    }
    if (size > cap) {  // the reference grows its Owned buffer in place; ours is the caller's
        *total_size = size;  // the caller resumes with iggy_frame_read_rest
        seterr(err, IGGY_ERR_CAPACITY, 0, size, cap);
        return IGGY_ERR_CAPACITY;
    }
    r = iggy_frame_read_rest(fd, buf, size, err);
    if (r == IGGY_ERR_INVALID_COMMAND) *total_size = size;  // consumed whole: the stream stays in sync
    if (r) return r;
    *total_size = size;
    return 0;
}

int iggy_frame_read_rest(int fd, uint8_t *buf, uint64_t size, iggy_wire_error *err) {
    if (fd < 0 || !buf || size < IGGY_FRAME_HEADER_BYTES) return IGGY_ERR_INVALID_ARGUMENT;
    seterr(err, IGGY_OK);
    // stage 2: the body into the tail of the same buffer (framing.rs:128-160)
    if (size > IGGY_FRAME_HEADER_BYTES) {
        const int r = read_exact_fd(fd, buf + IGGY_FRAME_HEADER_BYTES, size - IGGY_FRAME_HEADER_BYTES);
        if (r) {
            seterr(err, (uint32_t)r);
            return r;
        }
    }
    // Message::<GenericHeader>::try_from (consensus_message.rs:468-500): the checked bit
    // pattern of the header (only `command` has invalid patterns, command.rs:90-95),
    // validate() (always Ok for GenericHeader), size >= 256 and <= the bytes read
    // (both hold by construction here)
    if (buf[IGGY_FRAME_COMMAND_OFFSET] > IGGY_FRAME_COMMAND_MAX) {
        seterr(err, IGGY_ERR_INVALID_COMMAND);
        return IGGY_ERR_INVALID_COMMAND;
    }
    return 0;
}

#ifndef IGGY_HOST_ONLY
int iggy_codec_convert_request(iggy_codec_ctx *ctx, const uint8_t *frame, uint64_t len, uint64_t partition_id,
                               int checksum_mode, uint8_t *out, uint64_t cap, uint64_t *out_len,
                               iggy_batch_header *hdr_out, iggy_wire_error *err) {
    if (!ctx || !frame || !out || !out_len) return IGGY_ERR_INVALID_ARGUMENT;
    seterr(err, IGGY_OK);
    *out_len = 0;
    const uint64_t hs = IGGY_FRAME_HEADER_BYTES;
    auto invalid = [&]() {
        seterr(err, IGGY_ERR_INVALID_COMMAND);
        return IGGY_ERR_INVALID_COMMAND;
    };
    if (len < hs) return invalid();
    uint32_t total;
    memcpy(&total, frame + IGGY_FRAME_SIZE_OFFSET, 4);
    if (total < hs || total > len) return invalid();  // a Message's size never exceeds its buffer
    const uint8_t *body = frame + hs;
    const uint64_t blen = total - hs;
    // 1. a body that already IS one canonical batch (send_messages.rs:466-476): the
    //    checksum-verified decode decides; any failure falls through to the wire form
    iggy_batch_header h;
    iggy_wire_error e;
    if (iggy_batch_header_decode(body, blen, &h, &e) == 0 && h.batch_length <= blen &&
        iggy_codec_decode_batch(ctx, body, blen, IGGY_INTEGRITY_VERIFY, &h, nullptr, 0, nullptr, &e) == 0) {
        if (h.message_count == 0 || blen != h.batch_length || h.partition_id != partition_id) return invalid();
        if (cap < total) {
            seterr(err, IGGY_ERR_CAPACITY, 0, total, cap);
            return IGGY_ERR_CAPACITY;
        }
        if (out != frame) memcpy(out, frame, total);
        *out_len = total;
        if (hdr_out) *hdr_out = h;
        return 0;
    }
    // 2. admit_wire_request (send_messages.rs:480-540)
    if (blen < 4) return invalid();
    uint32_t mlen;
    memcpy(&mlen, body, 4);
    const uint64_t batch_start = 4 + (uint64_t)mlen;
    if (blen < batch_start) return invalid();
    iggy_send_messages_header meta;
    uint64_t consumed = 0;
    if (iggy_send_messages_header_decode(body + 4, mlen, &meta, &consumed, &e) != 0 || consumed != mlen)
        return invalid();
    const uint8_t *batch = body + batch_start;
    const uint64_t batch_len = blen - batch_start;
    if (cap < hs) {
        seterr(err, IGGY_ERR_CAPACITY, 0, hs + batch_len, cap);
        return IGGY_ERR_CAPACITY;
    }
    iggy_batch_header ah;
    const int r = iggy_codec_admit_batch(ctx, batch, batch_len, meta.messages_count, partition_id, checksum_mode,
                                         out + hs, cap - hs, &ah, err);
    if (r) return r;
    // the request header with the pipeline form's size (:523-528)
    if (out != frame) memcpy(out, frame, hs);
    const uint64_t new_total = hs + ah.batch_length;
    if (new_total > 0xFFFFFFFFull) return invalid();
    const uint32_t nt = (uint32_t)new_total;
    memcpy(out + IGGY_FRAME_SIZE_OFFSET, &nt, 4);
    *out_len = new_total;
    if (hdr_out) *hdr_out = ah;
    return 0;
}

#endif  // IGGY_HOST_ONLY

}  // extern "C"

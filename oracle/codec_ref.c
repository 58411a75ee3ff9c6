/*
 * codec_ref.c — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Plain-C restatement of the reference message-batch walks, one function per
 * reference item, each citing the file:line it follows (paths relative to the
 * apache/iggy tree). Serial, byte-at-a-time semantics exactly as the Rust
 * code: this is the checker the HIP path is compared against.
 */
#include "oracle.h"
#include <stdlib.h>
#include <string.h>

#define HDR 256u
#define FHDR 48u

static inline uint64_t rd64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline void wr64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }
static inline void wr32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }

static void set_err(iggy_wire_error *e, uint32_t kind, uint32_t reason, uint64_t a, uint64_t b,
                    uint64_t c) {
    if (!e) return;
    e->kind = kind; e->reason = reason; e->a = a; e->b = b; e->c = c;
}

/* BatchHeader::decode — batch.rs:98-134 */
int oracle_batch_header_decode(const uint8_t *b, uint64_t len, iggy_batch_header *h,
                               iggy_wire_error *e) {
    set_err(e, IGGY_OK, 0, 0, 0, 0);
    if (len < HDR) {
        set_err(e, IGGY_ERR_UNEXPECTED_EOF, 0, 0, HDR, len);
        return IGGY_ERR_UNEXPECTED_EOF;
    }
    uint64_t batch_length = rd64(b + 32);
    if (batch_length < HDR) { /* checked before the reserved bytes (batch.rs:108) */
        set_err(e, IGGY_ERR_VALIDATION, IGGY_V_BATCH_LENGTH_SHORT, 0, 0, 0);
        return IGGY_ERR_VALIDATION;
    }
    for (uint32_t i = IGGY_BATCH_RESERVED_OFFSET; i < HDR; i++) {
        if (b[i] != 0) {
            set_err(e, IGGY_ERR_VALIDATION, IGGY_V_BATCH_RESERVED, 0, 0, 0);
            return IGGY_ERR_VALIDATION;
        }
    }
    memset(h, 0, sizeof(*h));
    h->partition_id = rd64(b + 0);
    h->base_offset = rd64(b + 8);
    h->base_timestamp = rd64(b + 16);
    h->origin_timestamp = rd64(b + 24);
    h->batch_length = batch_length;
    h->batch_checksum = rd64(b + 40);
    h->message_count = rd32(b + 48);
    return 0;
}

/* BatchHeader::encode_into — batch.rs:138-150 */
void oracle_batch_header_encode(const iggy_batch_header *h, uint8_t *out) {
    memset(out, 0, HDR);
    wr64(out + 0, h->partition_id);
    wr64(out + 8, h->base_offset);
    wr64(out + 16, h->base_timestamp);
    wr64(out + 24, h->origin_timestamp);
    wr64(out + 32, h->batch_length);
    wr64(out + 40, h->batch_checksum);
    wr32(out + 48, h->message_count);
}

/* One step of BatchIteratorWithOffsets::next — batch.rs:332-354.
 * Returns 1 and the frame extent on success, 0 when the walk stops. */
static int walk_next(const uint8_t *blob, uint64_t blob_len, uint64_t pos, uint64_t *end,
                     uint32_t *pl, uint32_t *uh) {
    if (pos >= blob_len) return 0;
    if (blob_len - pos < FHDR) return 0;                  /* BatchMessageHeader::decode EOF */
    if (rd64(blob + pos + 40) != 0) return 0;             /* reserved, batch.rs:254 */
    uint32_t p = rd32(blob + pos + 36), u = rd32(blob + pos + 32);
    uint64_t payload_end = pos + FHDR + p;                 /* batch.rs:340 */
    uint64_t headers_end = payload_end + u;                /* batch.rs:341 */
    if (payload_end > blob_len) return 0;                  /* blob.get(..)? */
    if (headers_end > blob_len) return 0;
    *end = headers_end;
    *pl = p; *uh = u;
    return 1;
}

/* Batch checksum input = header fields (44 B) || stored checksum of every
 * walked frame; streaming XXH3 == one-shot over the concatenation
 * (batch.rs:439-459; pinned by server_common/src/send_messages.rs:833-871). */
static uint64_t hash_checksum_stream(const iggy_batch_header *h, const uint8_t *blob,
                                     const uint64_t *starts, uint64_t n) {
    uint64_t total = 44 + 8 * n;
    uint8_t *buf = (uint8_t *)malloc(total ? total : 1);
    wr64(buf + 0, h->partition_id);
    wr64(buf + 8, h->base_offset);
    wr64(buf + 16, h->base_timestamp);
    wr64(buf + 24, h->origin_timestamp);
    wr64(buf + 32, h->batch_length);
    wr32(buf + 40, h->message_count);
    for (uint64_t i = 0; i < n; i++) memcpy(buf + 44 + 8 * i, blob + starts[i], 8);
    uint64_t r = oracle_xxh3_64(buf, total);
    free(buf);
    return r;
}

/* calculate_batch_checksum — batch.rs:439-450 (infallible walk) */
uint64_t oracle_calculate_batch_checksum(const iggy_batch_header *h, const uint8_t *blob,
                                         uint64_t blob_len) {
    uint64_t cap = blob_len / FHDR + 1, n = 0, pos = 0, end;
    uint32_t pl, uh;
    uint64_t *starts = (uint64_t *)malloc(cap * sizeof(uint64_t));
    while (walk_next(blob, blob_len, pos, &end, &pl, &uh)) {
        starts[n++] = pos;
        pos = end;
    }
    uint64_t r = hash_checksum_stream(h, blob, starts, n);
    free(starts);
    return r;
}

/* verify_and_recompute_batch_checksum — batch.rs:474-506 */
int oracle_verify_and_recompute(const iggy_batch_header *h, const uint8_t *blob,
                                uint64_t blob_len, uint64_t *out, uint64_t *frame_pos,
                                uint64_t cap, uint64_t *nframes, iggy_wire_error *e) {
    set_err(e, IGGY_OK, 0, 0, 0, 0);
    uint64_t scap = blob_len / FHDR + 1, n = 0, pos = 0, end, covered = 0;
    uint32_t pl, uh;
    uint64_t *starts = (uint64_t *)malloc(scap * sizeof(uint64_t));
    while (walk_next(blob, blob_len, pos, &end, &pl, &uh)) {
        uint64_t stored = rd64(blob + pos);
        uint64_t expected = oracle_xxh3_64(blob + pos + 8, end - pos - 8);  /* :485 */
        if (expected != stored) {
            uint32_t od = rd32(blob + pos + 24);
            uint64_t off = h->base_offset + od;
            if (off < h->base_offset) off = UINT64_MAX;  /* saturating_add, :490-493 */
            set_err(e, IGGY_ERR_INVALID_MESSAGE_CHECKSUM, 0, stored, expected, off);
            free(starts);
            return IGGY_ERR_INVALID_MESSAGE_CHECKSUM;
        }
        starts[n++] = pos;
        covered = end;
        pos = end;
    }
    /* verified is a u32 in the reference (:478); n <= blob_len/48 < 2^32 here */
    if (n != (uint64_t)h->message_count || covered != blob_len) {
        set_err(e, IGGY_ERR_VALIDATION, IGGY_V_FRAMES_DO_NOT_TILE, 0, 0, 0);
        free(starts);
        return IGGY_ERR_VALIDATION;
    }
    if (out) *out = hash_checksum_stream(h, blob, starts, n);
    if (frame_pos) {
        for (uint64_t i = 0; i < n && i < cap; i++) frame_pos[i] = starts[i];
    }
    if (nframes) *nframes = n;
    free(starts);
    return 0;
}

/* validate_batch_layout — batch.rs:513-527 */
static int validate_layout(const iggy_batch_header *h, const uint8_t *blob, uint64_t blob_len,
                           uint64_t *frame_pos, uint64_t cap, uint64_t *nframes,
                           iggy_wire_error *e) {
    uint64_t n = 0, pos = 0, end, covered = 0;
    uint32_t pl, uh;
    while (walk_next(blob, blob_len, pos, &end, &pl, &uh)) {
        if (frame_pos && n < cap) frame_pos[n] = pos;
        n++;
        covered = end;
        pos = end;
    }
    if (n != (uint64_t)h->message_count || covered != blob_len) {
        set_err(e, IGGY_ERR_VALIDATION, IGGY_V_FRAMES_DO_NOT_TILE, 0, 0, 0);
        return IGGY_ERR_VALIDATION;
    }
    if (nframes) *nframes = n;
    return 0;
}

/* decode_batch_slice_with — batch.rs:391-422 */
int oracle_decode_batch_slice_with(const uint8_t *body, uint64_t len, int integrity,
                                   iggy_batch_header *h, uint64_t *frame_pos, uint64_t cap,
                                   uint64_t *nframes, iggy_wire_error *e) {
    int rc = oracle_batch_header_decode(body, len, h, e);
    if (rc) return rc;
    /* blob_len() cannot fail after decode (batch_length >= 256). */
    if (len < h->batch_length) {
        set_err(e, IGGY_ERR_UNEXPECTED_EOF, 0, 0, h->batch_length, len);
        return IGGY_ERR_UNEXPECTED_EOF;
    }
    const uint8_t *blob = body + HDR;
    uint64_t blob_len = h->batch_length - HDR;
    if (integrity == IGGY_INTEGRITY_VERIFY) {
        uint64_t computed = 0;
        rc = oracle_verify_and_recompute(h, blob, blob_len, &computed, frame_pos, cap, nframes, e);
        if (rc) return rc;
        if (h->batch_checksum != computed) {
            set_err(e, IGGY_ERR_INVALID_BATCH_CHECKSUM, 0, h->batch_checksum, computed,
                    h->base_offset);
            return IGGY_ERR_INVALID_BATCH_CHECKSUM;
        }
        return 0;
    }
    return validate_layout(h, blob, blob_len, frame_pos, cap, nframes, e);
}

/* SendMessagesEncoder::encoded_size batch part — send_messages.rs:69-79 */
uint64_t oracle_encoded_batch_size(const iggy_raw_messages *m) {
    uint64_t total = HDR;
    for (uint64_t i = 0; i < m->count; i++)
        total += FHDR + m->payload_lengths[i] +
                 (m->user_headers_lengths ? m->user_headers_lengths[i] : 0);
    return total;
}

/* SendMessagesEncoder::encode, batch section — send_messages.rs:89-181
 * (partition_id != 0: SendMessagesOwned::from_messages,
 *  server_common/src/send_messages.rs:104-168). */
int oracle_encode_batch(const iggy_raw_messages *m, uint64_t partition_id, uint8_t *out,
                        uint64_t cap, uint64_t *out_len, iggy_wire_error *e) {
    set_err(e, IGGY_OK, 0, 0, 0, 0);
    if (m->count == 0) {
        set_err(e, IGGY_ERR_VALIDATION, IGGY_V_EMPTY_BATCH, 0, 0, 0);
        return IGGY_ERR_VALIDATION;
    }
    if (m->count > 0xFFFFFFFFull) {
        set_err(e, IGGY_ERR_PAYLOAD_TOO_LARGE, 0, m->count, 0xFFFFFFFFull, 0);
        return IGGY_ERR_PAYLOAD_TOO_LARGE;
    }
    uint64_t origin = UINT64_MAX; /* min origin timestamp, :119-123 */
    for (uint64_t i = 0; i < m->count; i++)
        if (m->origin_timestamps[i] < origin) origin = m->origin_timestamps[i];
    uint64_t need = oracle_encoded_batch_size(m);
    if (need > cap) {
        set_err(e, IGGY_ERR_CAPACITY, 0, need, cap, 0);
        return IGGY_ERR_CAPACITY;
    }
    uint64_t pos = HDR, psrc = 0, usrc = 0;
    uint64_t *starts = (uint64_t *)malloc(m->count * sizeof(uint64_t));
    for (uint64_t i = 0; i < m->count; i++) { /* hot loop :131-164 */
        uint64_t delta = m->origin_timestamps[i] - origin;
        if (delta > IGGY_MAX_TIMESTAMP_DELTA_MICROS) {
            set_err(e, IGGY_ERR_INVALID_TIMESTAMP_DELTA, 0, delta, 0, 0);
            free(starts);
            return IGGY_ERR_INVALID_TIMESTAMP_DELTA;
        }
        uint32_t pl = m->payload_lengths[i];
        uint32_t uh = m->user_headers_lengths ? m->user_headers_lengths[i] : 0;
        uint8_t *f = out + pos;
        wr64(f + 0, 0);
        wr64(f + 8, m->ids[2 * i]);
        wr64(f + 16, m->ids[2 * i + 1]);
        wr32(f + 24, (uint32_t)i);
        wr32(f + 28, (uint32_t)delta);
        wr32(f + 32, uh);
        wr32(f + 36, pl);
        wr64(f + 40, 0);
        memcpy(f + FHDR, m->payloads + psrc, pl); /* payload before user headers, :159-160 */
        if (uh) memcpy(f + FHDR + pl, m->user_headers + usrc, uh);
        psrc += pl;
        usrc += uh;
        wr64(f, oracle_xxh3_64(f + 8, 40 + (uint64_t)pl + uh)); /* :162-163 */
        starts[i] = pos - HDR;
        pos += FHDR + (uint64_t)pl + uh;
    }
    /* The SDK caps the batch at u32::MAX (:166-174); the server twin does not. */
    if (partition_id == 0 && pos > 0xFFFFFFFFull) {
        set_err(e, IGGY_ERR_PAYLOAD_TOO_LARGE, 0, pos, 0xFFFFFFFFull, 0);
        free(starts);
        return IGGY_ERR_PAYLOAD_TOO_LARGE;
    }
    iggy_batch_header h;
    memset(&h, 0, sizeof(h));
    h.partition_id = partition_id;
    h.origin_timestamp = origin;
    h.batch_length = pos;
    h.message_count = (uint32_t)m->count;
    h.batch_checksum = hash_checksum_stream(&h, out + HDR, starts, m->count); /* :177 */
    oracle_batch_header_encode(&h, out);
    free(starts);
    if (out_len) *out_len = pos;
    return 0;
}

/* Poll decode.
 * mode SDK:      PolledMessages::messages_from_batches, polled_messages.rs:95-150
 * mode ITERATOR: PolledBatchesIterator, poll_messages.rs:95-165 */
int oracle_poll_decode(const uint8_t *buf, uint64_t len, int mode, iggy_polled_message *out,
                       uint64_t cap, uint64_t *n_out, iggy_wire_error *e) {
    set_err(e, IGGY_OK, 0, 0, 0, 0);
    uint64_t n = 0, position = 0;
    if (n_out) *n_out = 0;
    while (position < len) {
        iggy_batch_header h;
        iggy_wire_error he;
        if (mode == IGGY_POLL_MODE_SDK) {
            if (oracle_batch_header_decode(buf + position, len - position, &h, &he)) {
                set_err(e, IGGY_ERR_INVALID_MESSAGE_PAYLOAD_LENGTH, 0, 0, 0, 0);
                if (n_out) *n_out = 0;
                return IGGY_ERR_INVALID_MESSAGE_PAYLOAD_LENGTH;
            }
            uint64_t batch_end = position + h.batch_length;
            if (batch_end < position || batch_end > len) { /* checked_add + filter, :103-106 */
                set_err(e, IGGY_ERR_INVALID_MESSAGE_PAYLOAD_LENGTH, 0, 0, 0, 0);
                if (n_out) *n_out = 0;
                return IGGY_ERR_INVALID_MESSAGE_PAYLOAD_LENGTH;
            }
            uint64_t cursor = position + HDR;
            while (cursor < batch_end) {
                if (batch_end - cursor < FHDR || rd64(buf + cursor + 40) != 0) {
                    set_err(e, IGGY_ERR_INVALID_MESSAGE_PAYLOAD_LENGTH, 0, 0, 0, 0);
                    if (n_out) *n_out = 0;
                return IGGY_ERR_INVALID_MESSAGE_PAYLOAD_LENGTH;
                }
                const uint8_t *f = buf + cursor;
                uint32_t pl = rd32(f + 36), uh = rd32(f + 32);
                uint64_t ps = cursor + FHDR, pe = ps + pl, ue = pe + uh;
                if (ue > batch_end) {
                    set_err(e, IGGY_ERR_INVALID_MESSAGE_PAYLOAD_LENGTH, 0, 0, 0, 0);
                    if (n_out) *n_out = 0;
                return IGGY_ERR_INVALID_MESSAGE_PAYLOAD_LENGTH;
                }
                if (n >= cap) {
                    set_err(e, IGGY_ERR_CAPACITY, 0, n + 1, cap, 0);
                    return IGGY_ERR_CAPACITY;
                }
                iggy_polled_message *m = &out[n++];
                memset(m, 0, sizeof(*m));
                m->checksum = rd64(f);
                m->id_lo = rd64(f + 8);
                m->id_hi = rd64(f + 16);
                m->offset = h.base_offset + rd32(f + 24);          /* wrapping in release */
                m->timestamp = h.base_timestamp;
                m->origin_timestamp = h.origin_timestamp + rd32(f + 28);
                m->payload_pos = ps;
                m->payload_length = pl;
                m->user_headers_pos = pe;
                m->user_headers_length = uh;
                cursor = ue;
                if (n_out) *n_out = n;
            }
            position = batch_end;
        } else {
            uint64_t tmpn = 0;
            /* advance_batch: decode_batch_slice_with(LayoutOnly), poll_messages.rs:115-129 */
            int rc = oracle_decode_batch_slice_with(buf + position, len - position,
                                                    IGGY_INTEGRITY_LAYOUT_ONLY, &h, NULL, 0,
                                                    &tmpn, e);
            if (rc) return rc;
            const uint8_t *blob = buf + position + HDR;
            uint64_t blob_len = h.batch_length - HDR, pos = 0, end;
            uint32_t pl, uh;
            while (walk_next(blob, blob_len, pos, &end, &pl, &uh)) {
                if (n >= cap) {
                    set_err(e, IGGY_ERR_CAPACITY, 0, n + 1, cap, 0);
                    return IGGY_ERR_CAPACITY;
                }
                const uint8_t *f = blob + pos;
                iggy_polled_message *m = &out[n++];
                memset(m, 0, sizeof(*m));
                m->checksum = rd64(f);
                m->id_lo = rd64(f + 8);
                m->id_hi = rd64(f + 16);
                m->offset = h.base_offset + rd32(f + 24);
                m->timestamp = h.base_timestamp;
                m->origin_timestamp = h.origin_timestamp + rd32(f + 28);
                m->payload_pos = position + HDR + pos + FHDR;
                m->payload_length = pl;
                m->user_headers_pos = m->payload_pos + pl;
                m->user_headers_length = uh;
                if (n_out) *n_out = n;
                pos = end;
            }
            position += h.batch_length;
        }
    }
    if (n_out) *n_out = n;
    return 0;
}

/* stamp_prepare_for_persistence core — server_common/src/send_messages.rs:642-663 */
int oracle_stamp_batch(uint8_t *batch, uint64_t len, uint64_t base_offset,
                       uint64_t base_timestamp, iggy_batch_header *out, iggy_wire_error *e) {
    iggy_batch_header h;
    int rc = oracle_batch_header_decode(batch, len, &h, e);
    if (rc) return rc;
    if (len < h.batch_length) {
        set_err(e, IGGY_ERR_UNEXPECTED_EOF, 0, 0, h.batch_length, len);
        return IGGY_ERR_UNEXPECTED_EOF;
    }
    h.base_offset = base_offset;
    h.base_timestamp = base_timestamp;
    h.batch_checksum = oracle_calculate_batch_checksum(&h, batch + HDR, h.batch_length - HDR);
    oracle_batch_header_encode(&h, batch);
    if (out) *out = h;
    return 0;
}

/* batch_error (core/server_common/src/send_messages.rs:52-66): the two integrity
 * errors keep their payloads, every other wire error is InvalidCommand. */
static int server_error(int rc, iggy_wire_error *e) {
    if (rc == 0 || rc == IGGY_ERR_INVALID_BATCH_CHECKSUM || rc == IGGY_ERR_INVALID_MESSAGE_CHECKSUM) return rc;
    set_err(e, IGGY_ERR_INVALID_COMMAND, 0, 0, 0, 0);
    return IGGY_ERR_INVALID_COMMAND;
}

/* decode_prepare_slice_inner — core/server_common/src/send_messages.rs:581-622 */
int oracle_decode_prepare(const uint8_t *frame, uint64_t len, int validate, iggy_batch_header *h,
                          iggy_wire_error *e) {
    set_err(e, IGGY_OK, 0, 0, 0, 0);
    const uint64_t hs = IGGY_PREPARE_HEADER_SIZE;
    if (len < hs) return server_error(IGGY_ERR_VALIDATION, e);                     /* :586-588 */
    uint32_t total = 0;
    memcpy(&total, frame + IGGY_PREPARE_SIZE_OFFSET, 4);
    if (total < hs || len < total) return server_error(IGGY_ERR_VALIDATION, e);   /* :603-605 */
    const uint8_t *body = frame + hs;
    const uint64_t body_len = total - hs;
    if (body_len < HDR) return server_error(IGGY_ERR_VALIDATION, e);              /* :608-610 */
    int rc = oracle_batch_header_decode(body, HDR, h, e);                         /* :612-613 */
    if (rc) return server_error(rc, e);
    if (body_len != h->batch_length) return server_error(IGGY_ERR_VALIDATION, e); /* :619-621 */
    if (validate) {                                                               /* :625-635 */
        uint64_t computed = 0, n = 0;
        rc = oracle_verify_and_recompute(h, body + HDR, h->batch_length - HDR, &computed, NULL, 0, &n, e);
        if (rc) return server_error(rc, e);
        if (h->batch_checksum != computed) {
            set_err(e, IGGY_ERR_INVALID_BATCH_CHECKSUM, 0, h->batch_checksum, computed, h->base_offset);
            return IGGY_ERR_INVALID_BATCH_CHECKSUM;
        }
    }
    return 0;
}

/* admit_wire_request after the metadata decode — core/server_common/src/send_messages.rs:505-540 */
int oracle_admit_batch(const uint8_t *batch, uint64_t len, uint32_t meta_count, uint64_t partition_id,
                       int checksum_mode, uint8_t *out, uint64_t cap, iggy_batch_header *h,
                       iggy_wire_error *e) {
    uint64_t n = 0;
    int rc = oracle_decode_batch_slice_with(batch, len, IGGY_INTEGRITY_VERIFY, h, NULL, 0, &n, e); /* :505 */
    if (rc) return server_error(rc, e);
    if (h->message_count == 0 || h->message_count != meta_count || len != h->batch_length) {   /* :506-511 */
        set_err(e, IGGY_ERR_INVALID_COMMAND, 0, 0, 0, 0);
        return IGGY_ERR_INVALID_COMMAND;
    }
    if (cap < len) {
        set_err(e, IGGY_ERR_CAPACITY, 0, len, 0, 0);
        return IGGY_ERR_CAPACITY;
    }
    memcpy(out, batch, len);                                                      /* :518-520 */
    h->partition_id = partition_id;                                               /* :524-530 */
    h->batch_checksum = checksum_mode == IGGY_CHECKSUM_COMPUTE
                            ? oracle_calculate_batch_checksum(h, out + HDR, len - HDR)
                            : 0;
    oracle_batch_header_encode(h, out);
    return 0;
}

static uint64_t sat_add_u64(uint64_t a, uint64_t b) { return a + b < a ? ~0ull : a + b; }

/* recover_segment_bounds, index-less arm — core/partitions/src/segment_recovery.rs:425-488 */
int oracle_recover_segment(const uint8_t *messages, uint64_t len, uint64_t start_offset,
                           iggy_segment_recovery *out) {
    memset(out, 0, sizeof(*out));
    uint64_t position = 0, end_offset = start_offset, end_ts = 0, expected = start_offset;
    uint64_t start_ts = 0, batches = 0;
    int have_start = 0;
    while (position < len) {
        iggy_batch_header h;
        iggy_wire_error e;
        if (len - position < HDR) break;                                         /* read_batch_header :532-541 */
        if (oracle_batch_header_decode(messages + position, HDR, &h, &e)) break;
        const uint64_t extent = sat_add_u64(position, h.batch_length);           /* :460-463 */
        if (extent > len) break;
        uint64_t n = 0;                                                          /* :473-476, batch_verifies :518-530 */
        if (h.base_offset != expected ||
            oracle_decode_batch_slice_with(messages + position, h.batch_length, IGGY_INTEGRITY_VERIFY, &h, NULL,
                                           0, &n, &e))
            break;
        if (h.message_count > 0) {                                               /* :477-484 */
            end_offset = sat_add_u64(h.base_offset, (uint64_t)h.message_count - 1);
            end_ts = h.base_timestamp;
            if (!have_start) { start_ts = h.base_timestamp; have_start = 1; }
            expected = sat_add_u64(end_offset, 1);
        }
        ++batches;
        position = extent;
    }
    out->found = (uint64_t)have_start;
    out->start_timestamp = start_ts;
    out->end_timestamp = end_ts;
    out->end_offset = end_offset;
    out->walked_bytes = position;
    out->batches = batches;
    return 0;
}

/* select_batch_slice — core/partitions/src/journal.rs:1025-1086, then the header
 * push_selected_batch_fragments serves (journal.rs:1096-1137): a partial selection
 * gets batch_length = 256 + (end - start), message_count = matched and the batch
 * checksum of the byte range (BatchHeader::checksum_for_blob, batch.rs:174-176 ->
 * calculate_batch_checksum's infallible walk over the slice). */
int oracle_select_batch_slice(const uint8_t *record, uint64_t len, const iggy_slice_query *q,
                              iggy_slice_result *out, uint8_t *header_out) {
    iggy_batch_header h;
    iggy_wire_error e;
    memset(out, 0, sizeof(*out));
    int rc = oracle_batch_header_decode(record, len, &h, &e);
    if (rc) return rc;
    if (len < h.batch_length) return IGGY_ERR_UNEXPECTED_EOF;
    out->header = h;
    uint32_t remaining = q->count > q->already_matched ? q->count - q->already_matched : 0; /* :1030 */
    if (remaining == 0 || h.message_count == 0) return 0;                                   /* :1032 */
    const uint8_t *blob = record + HDR;
    uint64_t blob_len = h.batch_length - HDR, pos = 0, end, start = 0, sel_end = 0, last = 0;
    uint32_t pl, uh, matched = 0;
    int have = 0;
    while (walk_next(blob, blob_len, pos, &end, &pl, &uh)) {                /* iter_with_offsets */
        uint64_t offset = h.base_offset + rd32(blob + pos + 24);          /* :1043, wrapping */
        if (offset > q->ceiling) break;                                   /* :1048 */
        int selected = q->kind == IGGY_LOOKUP_OFFSET ? offset >= q->value  /* :1052-1065 */
                                                     : h.base_timestamp >= q->value;
        if (selected) {
            if (!have) { start = pos; have = 1; }                          /* :1070 */
            sel_end = end;
            matched++;
            last = offset;
            if (matched == remaining) break;                              /* :1075 */
        }
        pos = end;
    }
    if (!have) return 0;                                                  /* `start?` */
    out->selected = 1;
    out->start = start;
    out->end = sel_end;
    out->matched_messages = matched;
    out->last_matching_offset = last;
    out->full_body = start == 0 && sel_end == blob_len;                   /* :1105 */
    iggy_batch_header r = h;
    if (!out->full_body) {                                                /* :1114-1124 */
        r.batch_length = HDR + (sel_end - start);
        r.message_count = matched;
        r.batch_checksum = oracle_calculate_batch_checksum(&r, blob + start, sel_end - start);
    }
    out->header = r;
    if (header_out) {
        if (out->full_body) memcpy(header_out, record, HDR);
        else oracle_batch_header_encode(&r, header_out);
    }
    return 0;
}

/* walk_segment_payload — core/partitions/src/state_transfer.rs:715-833; decode_batch_slice
 * there is server_common's Verify wrapper (errors mapped by batch_error,
 * server_common/src/send_messages.rs:52-66). */
static uint32_t batch_error_kind(int rc) {
    return (rc == IGGY_ERR_INVALID_BATCH_CHECKSUM || rc == IGGY_ERR_INVALID_MESSAGE_CHECKSUM) ? (uint32_t)rc
                                                                                             : IGGY_ERR_INVALID_COMMAND;
}
int oracle_walk_segment_payload(const uint8_t *bytes, uint64_t len, uint64_t base_offset, uint8_t *index_out,
                                uint64_t index_cap, iggy_segment_walk *out) {
    memset(out, 0, sizeof(*out));
    uint64_t position = 0, next_offset = base_offset, indexed = 0, nidx = 0;
    int have_stats = 0, have_index = 0;
    while (position < len) {                                              /* :741 */
        iggy_batch_header h;
        iggy_wire_error e;
        int rc = oracle_decode_batch_slice_with(bytes + position, len - position, IGGY_INTEGRITY_VERIFY, &h, NULL,
                                                0, NULL, &e);
        if (rc) {                                                         /* :750-755 */
            out->error = IGGY_SEG_BATCH;
            out->position = position;
            if (batch_error_kind(rc) == IGGY_ERR_INVALID_COMMAND) set_err(&out->source, IGGY_ERR_INVALID_COMMAND, 0, 0, 0, 0);
            else out->source = e;
            return 0;
        }
        if (!have_stats && h.base_offset != base_offset) {                /* :757-762 */
            out->error = IGGY_SEG_BASE_OFFSET_MISMATCH;
            out->expected = base_offset;
            out->actual = h.base_offset;
            return 0;
        }
        if (h.base_offset != next_offset) {                               /* :763-768 */
            out->error = IGGY_SEG_NON_CONTIGUOUS;
            out->expected = next_offset;
            out->actual = h.base_offset;
            return 0;
        }
        if (h.message_count == 0) {                                       /* :769-774 */
            out->error = IGGY_SEG_BATCH;
            out->position = position;
            set_err(&out->source, IGGY_ERR_INVALID_MESSAGES_COUNT, 0, 0, 0, 0);
            return 0;
        }
        const uint64_t add = (uint64_t)h.message_count - 1;
        if (h.base_offset > UINT64_MAX - add) {                           /* :777-783 checked_add */
            out->error = IGGY_SEG_OFFSET_OVERFLOW;
            out->position = position;
            return 0;
        }
        const uint64_t batch_end = h.base_offset + add, ts = h.base_timestamp;
        if (!have_index || position - indexed >= 64 * 1024) {             /* :799-806, INDEX_STRIDE_BYTES */
            have_index = 1;
            indexed = position;
            if (index_out && nidx < index_cap) {
                wr64(index_out + 24 * nidx + 0, h.base_offset);
                wr64(index_out + 24 * nidx + 8, ts);
                wr64(index_out + 24 * nidx + 16, position);
            }
            nidx++;
        }
        if (!have_stats) {                                                /* :807-820 */
            out->start_timestamp = ts;
            out->max_timestamp = ts;
        } else if (ts > out->max_timestamp) {
            out->max_timestamp = ts;
        }
        have_stats = 1;
        out->end_offset = batch_end;
        out->end_timestamp = ts;
        out->batches++;
        if (batch_end == UINT64_MAX) {                                    /* :821-825 */
            out->error = IGGY_SEG_OFFSET_OVERFLOW;
            out->position = position;
            return 0;
        }
        next_offset = batch_end + 1;
        position += h.batch_length;                                       /* :830 */
    }
    out->index_entries = nidx;
    if (!have_stats) {
        out->error = IGGY_SEG_EMPTY;
        return 0;
    }
    return nidx > index_cap && index_out ? IGGY_ERR_CAPACITY : 0;
}

/* walk_disk_chunk — core/partitions/src/poll_plan.rs:950-1011, with
 * select_batch_slice + push_selected_batch_fragments (core/partitions/src/journal.rs:1025-1137).
 * `decode_batch_slice_with` there is server_common's wrapper (errors mapped by
 * batch_error): InvalidBatchChecksum marks the chunk corrupt at rest (:966-983),
 * every other error is an incomplete tail (:984-987). */
int oracle_walk_disk_chunk(const uint8_t *chunk, uint64_t len, const iggy_slice_query *q, int integrity,
                           iggy_chunk_fragment *frags, uint8_t *headers, uint64_t cap, iggy_chunk_walk *out) {
    memset(out, 0, sizeof(*out));
    uint32_t matched = q->already_matched;
    uint64_t cursor = 0, nfrag = 0;
    while (matched < q->count && cursor + HDR <= len) {                   /* :963 */
        iggy_batch_header h;
        iggy_wire_error e;
        int rc = oracle_decode_batch_slice_with(chunk + cursor, len - cursor, integrity, &h, NULL, 0, NULL, &e);
        if (rc == IGGY_ERR_INVALID_BATCH_CHECKSUM) {                      /* :966-983 */
            out->corrupt = 1;
            out->error = e;
            break;
        }
        if (rc) {                                                         /* :984-987 */
            out->error = e;
            break;
        }
        out->batches++;
        iggy_slice_query qq = *q;
        qq.already_matched = matched;
        iggy_slice_result r;
        uint8_t hb[256];
        oracle_select_batch_slice(chunk + cursor, h.batch_length, &qq, &r, hb);
        if (r.selected) {                                                 /* journal.rs:1096-1137 */
            if (nfrag < cap) {
                iggy_chunk_fragment *f = &frags[nfrag];
                memset(f, 0, sizeof(*f));
                f->batch_pos = cursor;
                f->full_body = r.full_body;
                f->body_start = r.full_body ? cursor : cursor + HDR + r.start;
                f->body_end = r.full_body ? cursor + h.batch_length : cursor + HDR + r.end;
                f->matched_messages = r.matched_messages;
                f->last_matching_offset = r.last_matching_offset;
                if (headers) memcpy(headers + 256 * nfrag, hb, 256);
            }
            nfrag++;
            matched += r.matched_messages;
            out->last_matching_offset = r.last_matching_offset;
            out->has_last_matching_offset = 1;
        }
        cursor += h.batch_length;                                         /* :1003 */
    }
    out->consumed = cursor < len ? cursor : len;
    out->matched = matched;
    out->fragments = nfrag;
    return nfrag > cap ? IGGY_ERR_CAPACITY : 0;
}

/* ---------------------------------------------------- synthetic inputs */
static inline uint64_t splitmix64(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static uint32_t synth_pl(uint64_t *s, uint32_t lo, uint32_t hi) {
    if (hi <= lo) return lo;
    return lo + (uint32_t)(splitmix64(s) % ((uint64_t)hi - lo + 1));
}

uint64_t oracle_synth_batch_size(uint64_t n, uint32_t pl_min, uint32_t pl_max, uint32_t uh_len,
                                 uint64_t seed) {
    uint64_t s = seed ^ 0x5151515151515151ull, total = HDR;
    for (uint64_t i = 0; i < n; i++) total += FHDR + synth_pl(&s, pl_min, pl_max) + uh_len;
    return total;
}

uint64_t oracle_synth_batch(uint8_t *out, uint64_t cap, uint64_t n, uint32_t pl_min,
                            uint32_t pl_max, uint32_t uh_len, uint64_t seed,
                            uint64_t partition_id) {
    uint64_t total = oracle_synth_batch_size(n, pl_min, pl_max, uh_len, seed);
    if (total > cap) return 0;
    uint64_t sl = seed ^ 0x5151515151515151ull; /* lengths stream (same as _size) */
    uint64_t sd = seed;                          /* data stream */
    const uint64_t origin0 = 1700000000000000ull;
    uint64_t pos = HDR;
    uint64_t *starts = (uint64_t *)malloc((n ? n : 1) * sizeof(uint64_t));
    for (uint64_t i = 0; i < n; i++) {
        uint32_t pl = synth_pl(&sl, pl_min, pl_max);
        uint8_t *f = out + pos;
        uint64_t idlo = splitmix64(&sd), idhi = splitmix64(&sd);
        if ((idlo | idhi) == 0) idlo = 1;
        wr64(f + 8, idlo);
        wr64(f + 16, idhi);
        wr32(f + 24, (uint32_t)i);
        wr32(f + 28, (uint32_t)i); /* origin_ts_i = origin0 + i */
        wr32(f + 32, uh_len);
        wr32(f + 36, pl);
        wr64(f + 40, 0);
        uint8_t *d = f + FHDR;
        uint32_t body = pl + uh_len, k = 0;
        for (; k + 8 <= body; k += 8) wr64(d + k, splitmix64(&sd));
        if (k < body) {
            uint64_t r = splitmix64(&sd);
            memcpy(d + k, &r, body - k);
        }
        wr64(f, oracle_xxh3_64_fast(f + 8, 40 + (uint64_t)body));
        starts[i] = pos - HDR;
        pos += FHDR + body;
    }
    iggy_batch_header h;
    memset(&h, 0, sizeof(h));
    h.partition_id = partition_id;
    h.base_offset = 0;
    h.base_timestamp = origin0 + 1000;
    h.origin_timestamp = origin0;
    h.batch_length = pos;
    h.message_count = (uint32_t)n;
    /* fast streaming-equivalent: one-shot over the 44 + 8n concatenation */
    {
        uint64_t tl = 44 + 8 * n;
        uint8_t *buf = (uint8_t *)malloc(tl);
        wr64(buf + 0, h.partition_id); wr64(buf + 8, h.base_offset);
        wr64(buf + 16, h.base_timestamp); wr64(buf + 24, h.origin_timestamp);
        wr64(buf + 32, h.batch_length); wr32(buf + 40, h.message_count);
        for (uint64_t i = 0; i < n; i++) memcpy(buf + 44 + 8 * i, out + HDR + starts[i], 8);
        h.batch_checksum = oracle_xxh3_64_fast(buf, tl);
        free(buf);
    }
    oracle_batch_header_encode(&h, out);
    free(starts);
    return pos;
}

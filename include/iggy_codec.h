/*
 * iggy_codec.h — C ABI of the MI355X-native Iggy message-batch codec.
 *
 * This is the drop-in boundary for Iggy's canonical message batch
 *
 *     batch = [batch header: 256 B][frame_0 ... frame_{n-1}]
 *     frame = [frame header: 48 B][payload][user_headers]
 *
 * (reference: core/binary_protocol/src/batch.rs:18-30). Every entry point is
 * plain C: pointers, sizes, PODs. No torch or HIP types appear in a signature;
 * streams are passed as `void*` (a hipStream_t, NULL = the context's stream).
 *
 * Each function names the reference Rust item it replaces (file:line relative
 * to the apache/iggy tree). INTEGRATION.md shows the Rust `extern "C"` shim a
 * maintainer would add so those Rust bodies become thin dispatchers.
 *
 * Conventions
 *  - return value: 0 = Ok; IGGY_ERR_* otherwise. Wire-format failures also
 *    fill an `iggy_wire_error` that mirrors `WireError`
 *    (core/binary_protocol/src/error.rs:24-68) field by field.
 *  - the caller owns every buffer; the library never frees caller memory.
 *  - host-buffer entry points are synchronous, except the `_submit` /
 *    iggy_codec_poll pair (for shard threads that must never block);
 *    `_device` entry points take device pointers, enqueue on `stream` and
 *    return immediately (results land in a device-resident result struct).
 *  - a context is used by one thread at a time (Iggy shards are
 *    thread-per-core); distinct contexts are independent.
 *  - every enqueue of one context runs in ONE stream order (its scratch is
 *    shared): a `_device` call on another stream than the context's previous
 *    enqueue first waits for that previous stream's work (so that stream must
 *    still exist). Calls on one stream pay nothing for this.
 *  - every entry point makes the context's device current for its duration
 *    and restores the caller's current device on return.
 *  - there is NO CPU fallback: without a usable gfx950 device
 *    iggy_codec_create fails with IGGY_ERR_DEVICE.
 */
#ifndef IGGY_CODEC_H
#define IGGY_CODEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IGGY_CODEC_ABI_VERSION 1u

/* batch.rs:38, :41, :44, :47, :50 */
#define IGGY_BATCH_HEADER_SIZE 256u
#define IGGY_FRAME_HEADER_SIZE 48u
#define IGGY_BATCH_CHECKSUM_OFFSET 40u
#define IGGY_BATCH_MESSAGE_COUNT_OFFSET 48u
#define IGGY_BATCH_RESERVED_OFFSET 52u
/* batch.rs:55 */
#define IGGY_MAX_TIMESTAMP_DELTA_MICROS 0xFFFFFFFFull

/* BatchIntegrity, batch.rs:358-365 */
typedef enum iggy_batch_integrity {
    IGGY_INTEGRITY_VERIFY = 0,
    IGGY_INTEGRITY_LAYOUT_ONLY = 1
} iggy_batch_integrity;

/* WireError variants used by the path (error.rs:27-70) + library failures. */
typedef enum iggy_error_kind {
    IGGY_OK = 0,
    IGGY_ERR_UNEXPECTED_EOF = 1,            /* a=offset b=need c=have      */
    IGGY_ERR_VALIDATION = 2,                /* reason = iggy_validation_reason */
    IGGY_ERR_INVALID_BATCH_CHECKSUM = 3,    /* a=stored b=computed c=base_offset */
    IGGY_ERR_INVALID_MESSAGE_CHECKSUM = 4,  /* a=stored b=computed c=offset */
    IGGY_ERR_INVALID_TIMESTAMP_DELTA = 5,   /* a=delta                     */
    IGGY_ERR_PAYLOAD_TOO_LARGE = 6,         /* a=size b=max                */
    IGGY_ERR_INVALID_UTF8 = 7,              /* a=offset                    */
    IGGY_ERR_UNKNOWN_DISCRIMINANT = 8,      /* a=type (IGGY_TYPE_*) b=value c=offset */
    /* IggyError mapping used by the SDK poll decode (polled_messages.rs:59-60) */
    IGGY_ERR_INVALID_NUMBER_ENCODING = 20,
    IGGY_ERR_INVALID_MESSAGE_PAYLOAD_LENGTH = 21,
    /* IggyError::InvalidCommand: batch_error's mapping of every structural WireError
     * on the server paths (server_common/src/send_messages.rs:52-66) */
    IGGY_ERR_INVALID_COMMAND = 22,
    /* IggyError::InvalidMessagesCount: a transferred segment batch with no messages
     * (core/partitions/src/state_transfer.rs:766-771) */
    IGGY_ERR_INVALID_MESSAGES_COUNT = 23,
    /* IggyError::CannotDecryptData: a section of frame a (b = 0 payload, 1 user
     * headers) is shorter than nonce + tag or fails the GCM tag
     * (core/common/src/utils/crypto.rs:80-90, server_common/src/send_messages.rs:385-399) */
    IGGY_ERR_CANNOT_DECRYPT_DATA = 24,
    /* IggyError::ConnectionClosed / TcpError of the socket framing
     * (core/message_bus/src/framing.rs:165-171) */
    IGGY_ERR_CONNECTION_CLOSED = 25,
    IGGY_ERR_TCP_ERROR = 26,
    /* library-level failures (not wire errors) */
    IGGY_ERR_DEVICE = 100,
    IGGY_ERR_INVALID_ARGUMENT = 101,
    IGGY_ERR_CAPACITY = 102,  /* output capacity too small; a = required */
    IGGY_ERR_TIMEOUT = 103,   /* a device-side bounded wait gave up (bug guard) */
    IGGY_ERR_PENDING = 104,   /* iggy_codec_poll: the operation has not finished yet */
    IGGY_ERR_BUSY = 105       /* every asynchronous slot of the context is in flight */
} iggy_error_kind;

/* The fixed `WireError::Validation` strings of the path, by id. */
typedef enum iggy_validation_reason {
    IGGY_V_NONE = 0,
    IGGY_V_BATCH_LENGTH_SHORT = 1,   /* "batch length must cover the batch header"        batch.rs:109-111 */
    IGGY_V_BATCH_RESERVED = 2,       /* "batch header reserved bytes must be zero"        batch.rs:120-122 */
    IGGY_V_FRAMES_DO_NOT_TILE = 3,   /* "batch frames do not tile message_count exactly"  batch.rs:501-503 */
    IGGY_V_FRAME_RESERVED = 4,       /* "message frame reserved bytes must be zero"       batch.rs:255-257 */
    IGGY_V_EMPTY_BATCH = 5,          /* "cannot encode an empty message batch"  send_messages.rs:97-99 */
    /* SendMessagesHeader metadata (binary_protocol/src/primitives/); a = the length found */
    IGGY_V_NUMERIC_ID_LENGTH = 6,    /* "numeric identifier must be 4 bytes, got {a}"           identifier.rs:202-206 */
    IGGY_V_STRING_ID_EMPTY = 7,      /* "string identifier cannot be empty"                     identifier.rs:215-219 */
    IGGY_V_BALANCED_LENGTH = 8,      /* "balanced partitioning must have length 0, got {a}"     partitioning.rs:111-115 */
    IGGY_V_PARTITION_ID_LENGTH = 9,  /* "partition_id partitioning must have length 4, got {a}" partitioning.rs:119-123 */
    IGGY_V_MESSAGES_KEY_EMPTY = 10   /* "messages_key partitioning cannot have empty key"       partitioning.rs:128-132 */
} iggy_validation_reason;

/* UnknownDiscriminant.type_name (error.rs:39-44) */
#define IGGY_TYPE_WIRE_IDENTIFIER 1u
#define IGGY_TYPE_WIRE_PARTITIONING 2u

typedef struct iggy_wire_error {
    uint32_t kind;    /* iggy_error_kind */
    uint32_t reason;  /* iggy_validation_reason when kind == IGGY_ERR_VALIDATION */
    uint64_t a, b, c;
} iggy_wire_error;

/* BatchHeader (batch.rs:64-73). 64 bytes, little-endian host order. */
typedef struct iggy_batch_header {
    uint64_t partition_id;
    uint64_t base_offset;
    uint64_t base_timestamp;
    uint64_t origin_timestamp;
    uint64_t batch_length;
    uint64_t batch_checksum;
    uint32_t message_count;
    uint32_t _pad0;
    uint64_t _pad1;
} iggy_batch_header;

/* One polled message, deltas resolved (IggyMessageHeader + payload/user
 * header ranges; polled_messages.rs:121-143, poll_messages.rs:75-86).
 * Positions are byte offsets into the caller's input buffer (zero-copy
 * views, like Bytes::slice). 80 bytes. */
typedef struct iggy_polled_message {
    uint64_t checksum;
    uint64_t id_lo, id_hi;      /* u128 id, little-endian halves */
    uint64_t offset;            /* base_offset + offset_delta */
    uint64_t timestamp;         /* base_timestamp (flat per batch) */
    uint64_t origin_timestamp;  /* origin_timestamp + timestamp_delta */
    uint64_t payload_pos;
    uint64_t user_headers_pos;
    uint32_t payload_length;
    uint32_t user_headers_length;
    uint64_t _pad;
} iggy_polled_message;

/* Encoder input, struct-of-arrays form of `&[RawMessage]`
 * (requests/messages/send_messages.rs:37-42). Pointers are host pointers for
 * iggy_codec_encode_batch and device pointers for the _device variant.
 * payloads / user_headers are the concatenation of every message's bytes in
 * message order; user_headers and user_headers_lengths may be NULL (= none). */
typedef struct iggy_raw_messages {
    uint64_t count;
    const uint64_t *ids;                 /* 2*count u64: id_lo, id_hi per message */
    const uint64_t *origin_timestamps;   /* count */
    const uint8_t *payloads;
    const uint32_t *payload_lengths;     /* count */
    const uint8_t *user_headers;
    const uint32_t *user_headers_lengths;/* count */
} iggy_raw_messages;

/* Device-resident result of an asynchronous decode. */
typedef struct iggy_decode_result {
    iggy_batch_header header;
    iggy_wire_error error;
    uint64_t frame_count;        /* frames walked (== message_count on success) */
    uint64_t computed_checksum;  /* recomputed batch checksum (Verify) */
    uint32_t path;               /* 1 = uniform-stride kernel, 2 = general walk */
    uint32_t status;             /* 0 = done; internal otherwise */
    uint64_t covered;            /* end of the last walked frame (blob-relative) */
} iggy_decode_result;

/* Device-resident result of an asynchronous encode. */
typedef struct iggy_encode_result {
    iggy_batch_header header;
    iggy_wire_error error;
    uint64_t batch_length;
    uint64_t _pad[3];
} iggy_encode_result;

typedef struct iggy_codec_ctx iggy_codec_ctx;

/* ---------------------------------------------------------------- context */
uint32_t iggy_codec_abi_version(void);
/* Binds a context to HIP device `device`, creates its stream and scratch.
 * Fails with IGGY_ERR_DEVICE when no gfx950 device is usable. */
int iggy_codec_create(int device, iggy_codec_ctx **out);
void iggy_codec_destroy(iggy_codec_ctx *ctx);
/* Pre-size device scratch for batches up to max_batch_bytes (optional;
 * otherwise grown on demand outside the enqueue path). */
int iggy_codec_reserve(iggy_codec_ctx *ctx, uint64_t max_batch_bytes, uint64_t max_frames);
/* The context's own stream (hipStream_t as void*). */
void *iggy_codec_stream(iggy_codec_ctx *ctx);
/* Blocks until every operation enqueued on the context's stream is done, and every
 * fast-path decode_submit on a slot's own stream (their tickets still need a poll). */
int iggy_codec_synchronize(iggy_codec_ctx *ctx);

/* ------------------------------------------------------------ pure host */
/* BatchHeader::decode (batch.rs:98-134) — 256 bytes, no device work. */
int iggy_batch_header_decode(const uint8_t *bytes, uint64_t len,
                             iggy_batch_header *out, iggy_wire_error *err);
/* BatchHeader::encode_into (batch.rs:138-150). */
void iggy_batch_header_encode(const iggy_batch_header *h, uint8_t out[256]);
/* SendMessagesEncoder::encoded_size, batch part (send_messages.rs:69-79). */
uint64_t iggy_encoded_batch_size(const iggy_raw_messages *msgs);

/* ------------------------------------------------- synchronous (host I/O) */
/* XxHash3_64::oneshot / calculate_checksum (common/src/utils/checksum.rs:20). */
int iggy_codec_xxh3_64(iggy_codec_ctx *ctx, const void *data, uint64_t len, uint64_t *out);

/* decode_batch_slice_with (batch.rs:391-422). On Ok, fills *hdr and, if
 * frame_pos != NULL, the blob-relative start of every frame (up to cap;
 * IGGY_ERR_CAPACITY if more). `body` may extend past batch_length. A single-stride
 * record of <= 4 MiB is read by the kernel in place over the host link: a registered
 * (iggy_codec_host_register) one through its device-mapped address (no copy), a
 * pageable one after a memcpy into the context's own mapped staging (no DMA). */
int iggy_codec_decode_batch(iggy_codec_ctx *ctx, const uint8_t *body, uint64_t len,
                            int integrity, iggy_batch_header *hdr,
                            uint64_t *frame_pos, uint64_t cap, uint64_t *nframes,
                            iggy_wire_error *err);

/* verify_and_recompute_batch_checksum (batch.rs:474-506). */
int iggy_codec_verify_and_recompute_batch_checksum(iggy_codec_ctx *ctx,
                                                   const iggy_batch_header *hdr,
                                                   const uint8_t *blob, uint64_t blob_len,
                                                   uint64_t *out, iggy_wire_error *err);

/* calculate_batch_checksum (batch.rs:439-450): frames found by the infallible
 * walk (BatchIteratorWithOffsets, batch.rs:329-355). */
int iggy_codec_calculate_batch_checksum(iggy_codec_ctx *ctx, const iggy_batch_header *hdr,
                                        const uint8_t *blob, uint64_t blob_len,
                                        uint64_t *out);

/* SendMessagesEncoder::encode batch section (send_messages.rs:89-181) when
 * partition_id == 0; SendMessagesOwned::from_messages
 * (server_common/src/send_messages.rs:104-168) with a namespace partition id
 * otherwise (ids of 0 are NOT minted here: the caller mints, as the SDK does
 * at common/src/traits/binary_impls/messages.rs:343-347). `out` must hold
 * iggy_encoded_batch_size(msgs) bytes. On an error other than capacity its contents
 * are unspecified (a small batch is encoded straight into a registered `out`), as
 * the reference's encoder leaves its partly written buffer to the caller. */
int iggy_codec_encode_batch(iggy_codec_ctx *ctx, const iggy_raw_messages *msgs,
                            uint64_t partition_id, uint8_t *out, uint64_t cap,
                            uint64_t *out_len, iggy_wire_error *err);

/* Poll-side decode of a stream of batch records (the body after the 16-byte
 * PollMessages prefix).
 *  mode 0 = SDK PolledMessages::messages_from_batches
 *           (common/src/types/message/polled_messages.rs:95-150):
 *           errors -> IGGY_ERR_INVALID_MESSAGE_PAYLOAD_LENGTH, no count check.
 *  mode 1 = PolledBatchesIterator (responses/messages/poll_messages.rs:95-165):
 *           each record decoded LayoutOnly; the first framing error is
 *           returned after the messages yielded before it (*n is set). */
#define IGGY_POLL_MODE_SDK 0
#define IGGY_POLL_MODE_ITERATOR 1
int iggy_codec_poll_decode(iggy_codec_ctx *ctx, const uint8_t *records, uint64_t len,
                           int mode, iggy_polled_message *out, uint64_t cap,
                           uint64_t *n, iggy_wire_error *err);

/* stamp_prepare_for_persistence core (server_common/src/send_messages.rs:642-663):
 * write base_offset/base_timestamp into the batch header at `batch` and
 * recompute batch_checksum over its blob. */
int iggy_codec_stamp_batch(iggy_codec_ctx *ctx, uint8_t *batch, uint64_t len,
                           uint64_t base_offset, uint64_t base_timestamp,
                           iggy_batch_header *out, iggy_wire_error *err);

/* ------------------------------------------- asynchronous (device memory) */
/* decode_batch_slice_with on a device-resident record. Enqueues the whole
 * decode on `stream`; the outcome lands in *d_result (device memory). */
int iggy_codec_decode_batch_device(iggy_codec_ctx *ctx, const uint8_t *d_body, uint64_t len,
                                   int integrity, uint64_t *d_frame_pos, uint64_t cap,
                                   iggy_decode_result *d_result, void *stream);

/* SendMessagesEncoder::encode on device-resident SoA input (all pointers in
 * *msgs are device pointers; *msgs itself is a host struct). */
int iggy_codec_encode_batch_device(iggy_codec_ctx *ctx, const iggy_raw_messages *msgs,
                                   uint64_t partition_id, uint8_t *d_out, uint64_t cap,
                                   iggy_encode_result *d_result, void *stream);

/* Batch checksum of a device-resident, already-validated record whose frame
 * starts are known (d_frame_pos, blob-relative); header fields from *hdr.
 * Writes the u64 to *d_out. Used by stamp (a17) and slicing (journal.rs:1119). */
int iggy_codec_batch_checksum_device(iggy_codec_ctx *ctx, const iggy_batch_header *hdr,
                                     const uint8_t *d_blob, const uint64_t *d_frame_pos,
                                     uint64_t nframes, uint64_t *d_out, void *stream);

/* XXH3-64 of n independent byte ranges of d_data (offsets u64, lengths u32). */
int iggy_codec_xxh3_64_ranges_device(iggy_codec_ctx *ctx, const uint8_t *d_data,
                                     const uint64_t *d_offsets, const uint32_t *d_lengths,
                                     uint64_t n, uint64_t *d_out, void *stream);

/* --------------------------------------- at-rest encryption */
/* AES-256-GCM re-encode of a canonical batch record on the device:
 * encrypt_batch_request (core/server_common/src/send_messages.rs:293-355) and
 * decrypt_batch_record (:357-415) with Aes256GcmEncryptor
 * (core/common/src/utils/crypto.rs:47-90). Every message's payload (always) and
 * user headers (when non-empty) become nonce(12) || ciphertext || tag(16) with
 * empty associated data (decrypt: the reverse); id, offset_delta and
 * timestamp_delta are kept, lengths, per-message checksums, batch_length and the
 * batch checksum are restamped; every other header field is kept.
 * Encrypt verifies the input first (decode_batch_slice = Verify; its error comes
 * back as is); decrypt checks layout only and requires len == batch_length
 * (IGGY_ERR_INVALID_COMMAND otherwise). The reference draws each nonce from the
 * OS RNG; here the caller supplies them: d_nonces holds 24 B per message, the
 * payload's nonce then the user headers' (read only when the message has user
 * headers). The encrypted record is at most len + 56 * message_count bytes, the
 * decrypted one at most len. Output [256 B header][frames] at d_out (cap bytes);
 * *d_result is written on the stream. key: 32 host bytes. */
typedef struct iggy_crypt_result {
    iggy_wire_error error;  /* the input's decode error, IGGY_ERR_INVALID_COMMAND,
                               IGGY_ERR_CANNOT_DECRYPT_DATA, IGGY_ERR_CAPACITY (a = bytes needed) */
    uint64_t out_len;        /* bytes of the re-encoded record, header included */
    uint64_t frame_count;
    uint64_t batch_checksum; /* of the re-encoded record */
} iggy_crypt_result;

int iggy_codec_encrypt_batch_device(iggy_codec_ctx *ctx, const uint8_t *key, const uint8_t *d_record,
                                    uint64_t len, const uint8_t *d_nonces, uint8_t *d_out, uint64_t cap,
                                    iggy_crypt_result *d_result, void *stream);
int iggy_codec_decrypt_batch_device(iggy_codec_ctx *ctx, const uint8_t *key, const uint8_t *d_record,
                                    uint64_t len, uint8_t *d_out, uint64_t cap, iggy_crypt_result *d_result,
                                    void *stream);

/* ------------------------------------------------------ poll reply body */
/* One poll fragment (PollFragments, core/server/src/responses.rs:1666-1680): a stored
 * record served whole, or a rewritten 256-B batch header followed by a body slice
 * (journal.rs:1096-1137; iggy_codec_walk_disk_chunk's iggy_chunk_fragment gives both:
 * full body = chunk + batch_pos, else headers[k] then chunk[body_start, body_end)). */
typedef struct iggy_poll_fragment {
    const uint8_t *data;  /* host memory */
    uint64_t len;
} iggy_poll_fragment;

/* build_polled_messages_body (core/server/src/responses.rs:1666-1714) -> out =
 * [partition_id u32][current_offset u64][count u32][records...]: the fragments are
 * concatenated and walked record by record (BatchHeader::decode and the record's end
 * inside the stream, else IGGY_ERR_INVALID_COMMAND); with key (32 B, nullable) every
 * record is decrypted (decrypt_batch_record, server_common/src/send_messages.rs:364-415:
 * IGGY_ERR_CANNOT_DECRYPT_DATA for a failing section, IGGY_ERR_INVALID_COMMAND for a
 * malformed record) on the GPU -- one H2D, every record's decrypt enqueued back to back,
 * one D2H -- else copied as is; count = the records' message_count summed with
 * checked_add (overflow -> IGGY_ERR_INVALID_COMMAND). Errors come in the reference's
 * order (record by record). cap too small -> IGGY_ERR_CAPACITY (err->a = bytes needed).
 * *out_len = the body's length. */
int iggy_codec_build_polled_body(iggy_codec_ctx *ctx, uint32_t partition_id, uint64_t current_offset,
                                 const iggy_poll_fragment *frags, uint64_t nfrags, const uint8_t *key,
                                 uint8_t *out, uint64_t cap, uint64_t *out_len, iggy_wire_error *err);

/* ------------------------------------------------- poll-path slicing (a17+) */
/* MessageLookup (core/partitions/src/journal.rs:68-95). */
#define IGGY_LOOKUP_OFFSET 0
#define IGGY_LOOKUP_TIMESTAMP 1
typedef struct iggy_slice_query {
    uint32_t kind;             /* IGGY_LOOKUP_* */
    uint32_t count;            /* query.count() */
    uint64_t value;            /* offset (>=) or timestamp (base_timestamp >=) */
    uint64_t ceiling;          /* inclusive commit frontier: no offset above it is served */
    uint32_t already_matched;  /* messages matched by earlier batches of this poll */
    uint32_t _pad;
} iggy_slice_query;

/* select_batch_slice (journal.rs:1025-1086) plus the header that
 * push_selected_batch_fragments (journal.rs:1096-1137) serves it with. 128 B. */
typedef struct iggy_slice_result {
    uint32_t selected;             /* 0 = None: nothing of this batch is served */
    uint32_t full_body;            /* 1 = the whole record is forwarded by reference */
    uint64_t start, end;           /* blob-relative byte range of the selection */
    uint32_t matched_messages;
    uint32_t _pad0;
    uint64_t last_matching_offset;
    iggy_batch_header header;      /* rewritten (length, count, checksum) when partial,
                                      the record's own header when full_body */
    uint64_t _pad1[3];
} iggy_slice_result;

/* Select a poll's messages from one decoded record (host buffers): the record is
 * decoded LayoutOnly first (its error is returned if it does not decode), then
 * selected; header_out (nullable, 256 B) receives the header bytes to serve. */
int iggy_codec_select_slice(iggy_codec_ctx *ctx, const uint8_t *record, uint64_t len,
                            const iggy_slice_query *query, iggy_slice_result *out,
                            uint8_t *header_out, iggy_wire_error *err);

/* Device-resident form on a record already decoded by iggy_codec_decode_batch_device
 * (d_frame_pos / nframes are its output): selection, rewritten header and its batch
 * checksum (recomputed over the selected frames, batch.rs:439-450 via
 * BatchHeader::checksum_for_blob, batch.rs:174-176) are enqueued on `stream`;
 * *d_out and d_header_out (nullable, 256 B) are device memory. */
int iggy_codec_select_slice_device(iggy_codec_ctx *ctx, const uint8_t *d_record,
                                   const uint64_t *d_frame_pos, uint64_t nframes,
                                   const iggy_slice_query *query, iggy_slice_result *d_out,
                                   uint8_t *d_header_out, void *stream);

/* ------------------------------------------------------- disk-poll chunk walk */
/* One fragment push_selected_batch_fragments (journal.rs:1096-1137) emits for a
 * selected batch: the whole record by reference (full_body), or the rewritten
 * header (headers[k], 256 B) followed by the chunk bytes [body_start, body_end). 48 B. */
typedef struct iggy_chunk_fragment {
    uint64_t batch_pos;             /* chunk offset of the batch's 256-B header */
    uint32_t full_body;
    uint32_t matched_messages;
    uint64_t body_start, body_end;  /* chunk byte range served (full body: the whole record) */
    uint64_t last_matching_offset;
    uint64_t _pad;
} iggy_chunk_fragment;

/* ChunkWalk plus the walk's carried state (poll_plan.rs:950-1011). 72 B. */
typedef struct iggy_chunk_walk {
    uint64_t consumed;                /* ChunkWalk.consumed: where the caller re-reads from */
    uint32_t corrupt;                 /* ChunkWalk.corrupt: a batch failed its batch checksum */
    uint32_t matched;                 /* `matched` after the walk (query->already_matched before) */
    uint64_t last_matching_offset;    /* valid when has_last_matching_offset */
    uint32_t has_last_matching_offset;
    uint32_t fragments;               /* fragments pushed (may exceed the capacity: then CAPACITY) */
    iggy_wire_error error;            /* the decode error that ended the walk, if any */
    uint64_t batches;                 /* batches decoded and selected from */
} iggy_chunk_walk;

/* walk_disk_chunk (core/partitions/src/poll_plan.rs:950-1011) over one chunk of
 * stamped [256 B header][blob] records read from a segment (host memory). From
 * byte 0, while query->already_matched < query->count and a header fits: decode
 * with `integrity` (Verify when system.partition.validate_checksum); a batch
 * failing its batch checksum stops the walk as corrupt at rest (:966-983), any
 * other decode error as an incomplete tail (:984-987); otherwise
 * select_batch_slice with the running match count (journal.rs:1025-1086) and
 * push its fragments. Every batch is verified and selected on the GPU, the match
 * count carried from batch to batch on the device (one copy in, one sync).
 * frags / headers (nullable, 256 B per fragment) hold up to cap fragments. */
int iggy_codec_walk_disk_chunk(iggy_codec_ctx *ctx, const uint8_t *chunk, uint64_t len,
                               const iggy_slice_query *query, int integrity, iggy_chunk_fragment *frags,
                               uint8_t *headers, uint64_t cap, iggy_chunk_walk *out);

/* stamp_prepare_for_persistence core (server_common/src/send_messages.rs:642-663) on a
 * device-resident record whose frames were walked by a decode (d_frame_pos/nframes):
 * base_offset and base_timestamp written, batch checksum recomputed, header rewritten
 * in place; the new header also lands in *d_header (nullable, device memory). */
int iggy_codec_stamp_batch_device(iggy_codec_ctx *ctx, uint8_t *d_record, const uint64_t *d_frame_pos,
                                  uint64_t nframes, uint64_t base_offset, uint64_t base_timestamp,
                                  iggy_batch_header *d_header, void *stream);

/* ------------------------------------------------- server admission / prepare */
/* PrepareHeader.size (u32) sits at byte 48 of the 256-B consensus header
 * (binary_protocol/src/consensus/header.rs:901-932); the batch header follows it. */
#define IGGY_PREPARE_HEADER_SIZE 256u
#define IGGY_PREPARE_SIZE_OFFSET 48u

/* ChecksumMode (server_common/src/send_messages.rs:416-432) */
typedef enum iggy_checksum_mode {
    IGGY_CHECKSUM_COMPUTE = 0,
    IGGY_CHECKSUM_SKIP = 1
} iggy_checksum_mode;

/* decode_prepare_slice (validate = 1) / decode_prepare_slice_trusted (validate = 0)
 * (server_common/src/send_messages.rs:542-622) on one prepare frame
 * [PrepareHeader 256 B][batch header 256 B][blob] of len bytes. Structural
 * failures (short frame, size outside [256, len], a body that is not exactly
 * batch_length long, a batch header that does not decode, frames that do not
 * tile) return IGGY_ERR_INVALID_COMMAND; validate = 1 also verifies every
 * message checksum and the batch checksum on the GPU (those two errors keep
 * their payloads, as batch_error does); validate = 0 reads the header only. */
int iggy_codec_decode_prepare(iggy_codec_ctx *ctx, const uint8_t *frame, uint64_t len, int validate,
                              iggy_batch_header *hdr_out, iggy_wire_error *err);

/* admit_wire_request's batch half (server_common/src/send_messages.rs:480-540):
 * batch = the wire batch after the metadata section (the caller decoded the
 * metadata and passes its messages_count). Verified as the producer hashed it;
 * an empty batch, a count unlike the metadata's, or a batch that does not fill
 * len exactly is IGGY_ERR_INVALID_COMMAND. On success out (>= len bytes)
 * receives the batch with partition_id stamped and the batch checksum
 * recomputed (IGGY_CHECKSUM_COMPUTE) or zeroed (IGGY_CHECKSUM_SKIP). */
int iggy_codec_admit_batch(iggy_codec_ctx *ctx, const uint8_t *batch, uint64_t len,
                           uint32_t metadata_messages_count, uint64_t partition_id, int checksum_mode,
                           uint8_t *out, uint64_t cap, iggy_batch_header *hdr_out, iggy_wire_error *err);

/* decode_batch_slice_with (batch.rs:391-422) of many records of one host buffer in
 * one call: record k is buf[offsets[k] .. len) (trailing bytes allowed, as the walks
 * over a disk chunk, a segment or a poll body pass each batch; poll_plan.rs:964,
 * segment_recovery.rs:529, state_transfer.rs:751, poll_messages.rs:132). One copy of
 * the buffer, ONE launch for every single-stride record (one workgroup per
 * 128-frame checksum block, decode_records.hip), the single-record decode for the
 * rest, one sync. out[k] receives record k's verdict exactly as
 * iggy_codec_decode_batch_device writes it. */
int iggy_codec_decode_records(iggy_codec_ctx *ctx, const uint8_t *buf, uint64_t len, const uint64_t *offsets,
                              uint64_t nrec, int integrity, iggy_decode_result *out);

/* -------------------------------------------------------- segment recovery */
/* recover_segment_bounds' index-less arm (core/partitions/src/segment_recovery.rs:425-488,
 * batch_verifies :518-530): walk the batches of one segment's messages file from
 * byte 0; a batch is accepted while its header decodes, it fits in the file, its
 * base_offset continues the chain from start_offset and it passes the Verify
 * decode (every message checksum + the batch checksum, on the GPU). 48 B. */
typedef struct iggy_segment_recovery {
    uint64_t found;            /* 0 = None: no accepted batch carried messages */
    uint64_t start_timestamp;  /* base_timestamp of the first accepted batch with messages */
    uint64_t end_timestamp;
    uint64_t end_offset;       /* last offset of the chain (start_offset when none) */
    uint64_t walked_bytes;     /* end of the last accepted batch: the torn tail starts here */
    uint64_t batches;          /* accepted batches */
} iggy_segment_recovery;

int iggy_codec_recover_segment(iggy_codec_ctx *ctx, const uint8_t *messages, uint64_t len,
                               uint64_t start_offset, iggy_segment_recovery *out);

/* SegmentWalkError (core/partitions/src/state_transfer.rs:664-709) */
typedef enum iggy_segment_walk_error {
    IGGY_SEG_OK = 0,
    IGGY_SEG_BATCH = 1,                 /* position, source */
    IGGY_SEG_BASE_OFFSET_MISMATCH = 2,  /* expected (manifest), actual */
    IGGY_SEG_NON_CONTIGUOUS = 3,        /* expected, actual */
    IGGY_SEG_OFFSET_OVERFLOW = 4,       /* position */
    IGGY_SEG_EMPTY = 5
} iggy_segment_walk_error;

/* walk_segment_payload's outcome: SegmentWalkStats + the rebuilt sparse index. 112 B. */
typedef struct iggy_segment_walk {
    uint32_t error;                 /* iggy_segment_walk_error */
    uint32_t _pad;
    uint64_t position;              /* BATCH / OFFSET_OVERFLOW: byte position of the batch */
    uint64_t expected, actual;      /* BASE_OFFSET_MISMATCH / NON_CONTIGUOUS */
    iggy_wire_error source;         /* BATCH: the decode error as batch_error maps it
                                       (server_common/src/send_messages.rs:52-66), or
                                       IGGY_ERR_INVALID_MESSAGES_COUNT */
    uint64_t end_offset, start_timestamp, end_timestamp, max_timestamp;  /* error == OK */
    uint64_t batches;
    uint64_t index_entries;         /* 24-B IggyIndex entries (iggy_index.rs:17-41) produced */
} iggy_segment_walk;

/* walk_segment_payload (core/partitions/src/state_transfer.rs:715-833): every batch
 * of a transferred segment `.log` payload Verify-decoded (all message checksums and
 * the batch checksum, on the GPU: one copy, every batch queued, one sync), offset
 * continuity from the manifest's base_offset, the stats, and the locally rebuilt
 * sparse index: one 24-B (base_offset, base_timestamp, position) entry for the first
 * batch and then every >= 64 KiB (INDEX_STRIDE_BYTES, :2799). index_out (nullable)
 * receives up to index_cap entries (IGGY_ERR_CAPACITY when more were produced). */
int iggy_codec_walk_segment_payload(iggy_codec_ctx *ctx, const uint8_t *bytes, uint64_t len, uint64_t base_offset,
                                    uint8_t *index_out, uint64_t index_cap, iggy_segment_walk *out);

/* MessagesWriter::save_frozen_batches (core/partitions/src/messages_writer.rs:100-118)
 * for stamped batches resident on the device: `len` bytes at d_bytes are copied to
 * the host through the context's pinned staging (two halves in flight: the D2H of
 * one piece overlaps the pwrite of the previous one) and written to the segment
 * file descriptor `fd` at byte `position`; fdatasync afterwards when `fsync` is
 * set. *written = bytes written. IGGY_ERR_DEVICE on an I/O failure (errno kept). */
int iggy_codec_segment_write_device(iggy_codec_ctx *ctx, int fd, uint64_t position, const uint8_t *d_bytes,
                                    uint64_t len, int fsync, uint64_t *written);

/* ------------------------------------------- asynchronous (host buffers) */
/* Server shard threads run one compio reactor each with NO blocking pool
 * (server_common/src/executor.rs:80-88, core/server/src/bootstrap.rs:720-760),
 * so a host-buffer codec call must not block them. A `_submit` copies the
 * caller's buffer to a device slot (async H2D on the context's copy-in
 * stream), enqueues the same kernels as the synchronous call on the context's
 * stream and the result / output copies on its copy-out stream, and returns a
 * ticket at once; iggy_codec_poll tells whether it has finished. Successive
 * submits overlap (one operation's H2D, another's kernels, a third's D2H).
 * Kernels never read host memory. Caller buffers must stay valid (and
 * unmodified, for inputs) until the ticket completes. Pinned caller memory
 * (hipHostMalloc, hipHostRegister, iggy_codec_host_register) is copied by DMA
 * directly. Pageable memory is never a DMA source or target: an input is
 * staged through the context's pinned chunks inside the submit (which blocks
 * for that memcpy), an output lands in the slot's pinned bounce and is copied
 * to the caller by the iggy_codec_poll / _wait that completes the ticket (only
 * on success). Register long-lived buffers (the server's 4096-aligned
 * Owned<MESSAGE_ALIGN> pool, server_common/src/iobuf.rs) once with
 * iggy_codec_host_register. At most 8 operations per context are in flight
 * (IGGY_ERR_BUSY otherwise). */
typedef uint64_t iggy_ticket;
#define IGGY_OP_DECODE 1u
#define IGGY_OP_ENCODE 2u
typedef struct iggy_completion {
    uint32_t op;                  /* IGGY_OP_* */
    uint32_t _pad0;
    iggy_batch_header header;     /* decode: the record's header; encode: the written header */
    iggy_wire_error error;        /* the operation's verdict (kind IGGY_OK = success) */
    uint64_t frame_count;         /* decode: frames walked */
    uint64_t computed_checksum;   /* decode (Verify): recomputed batch checksum */
    uint64_t bytes;               /* encode: batch bytes written to `out` */
    uint64_t _pad1[3];
} iggy_completion;

/* Page-lock a caller buffer for the context's device (hipHostRegister) / undo it.
 * The pages a registration touches ([ptr & ~4095, ptr + len rounded up to 4096)) must
 * not meet those of another live registration (IGGY_ERR_INVALID_ARGUMENT otherwise):
 * the runtime pins whole pages, and two registrations over one page leave a dead
 * mapping behind when either is undone. Register page-aligned buffers (the server's
 * 4096-aligned Owned<MESSAGE_ALIGN> pool). Unregister only through the codec (never a
 * bare hipHostUnregister); ranges a context registered are unregistered when it is
 * destroyed. */
int iggy_codec_host_register(iggy_codec_ctx *ctx, void *ptr, uint64_t len);
int iggy_codec_host_unregister(iggy_codec_ctx *ctx, void *ptr);
/* 1 when every host entry point copies [ptr, ptr + len) by DMA directly (pinned:
 * registered through the codec, hipHostRegister, hipHostMalloc), 0 when it stages the
 * bytes through the context's pinned chunks (pageable memory). Every synchronous
 * host entry point borrows its buffers for the call only (batch.rs:391): nothing of
 * the call touches caller memory after it returns, pinned or not. */
int iggy_codec_host_pinned(const void *ptr, uint64_t len);
/* decode_batch_slice_with (batch.rs:391-422) of a host record; frame_pos
 * (nullable, host) receives up to `cap` blob-relative frame starts (entries
 * past frame_count are unspecified; more frames than cap -> IGGY_ERR_CAPACITY
 * in the completion). A record of <= 16 MiB whose frame 0 sets a stride that
 * tiles it is one k_decode_records launch on the slot's own stream with the slot's
 * own scratch, so such submits run side by side on the device: an input of
 * <= 4 MiB is read in place (the one exception to "kernels never read host memory":
 * pinned memory through its device-mapped address; a pageable input is first copied
 * into the slot's own mapped staging, which the slot keeps until the ticket
 * completes, so submit never waits on the stream), the verdict
 * lands in the slot's completion record and the positions in mapped host memory;
 * if the stride breaks mid-record, the iggy_codec_poll that sees it starts the
 * general walk and the ticket stays pending one more round. */
int iggy_codec_decode_submit(iggy_codec_ctx *ctx, const uint8_t *body, uint64_t len, int integrity,
                             uint64_t *frame_pos, uint64_t cap, iggy_ticket *ticket);
/* SendMessagesEncoder::encode batch section (send_messages.rs:89-181) from host
 * SoA input into `out` (host, cap bytes; a batch larger than cap writes nothing
 * and completes with IGGY_ERR_CAPACITY). A batch whose SoA input is <= 4 MiB is
 * encoded in place on the slot's own stream with the slot's own scratch: the kernels
 * read registered arrays where they are (pageable ones are first copied into the
 * slot's mapped staging) and write the wire bytes and the verdict into mapped host
 * memory (the caller's pinned `out`, else the slot's bounce). Registered inputs
 * stay borrowed until the ticket completes; on an error other than capacity the
 * contents of a pinned `out` are unspecified. */
int iggy_codec_encode_submit(iggy_codec_ctx *ctx, const iggy_raw_messages *msgs, uint64_t partition_id,
                             uint8_t *out, uint64_t cap, iggy_ticket *ticket);
/* 0: finished, *out filled (out->error is the operation's own verdict) and the
 * ticket retired; IGGY_ERR_PENDING: not yet; never blocks. */
int iggy_codec_poll(iggy_codec_ctx *ctx, iggy_ticket ticket, iggy_completion *out);
/* Blocking form of iggy_codec_poll (tests, SDK tasks that may block). */
int iggy_codec_wait(iggy_codec_ctx *ctx, iggy_ticket ticket, iggy_completion *out);

/* ------------------------------------ SDK request body and poll response (a9, a10, a12, a18) */
/* WireIdentifier (binary_protocol/src/primitives/identifier.rs:97-231): kind 1 =
 * numeric (length 4, u32 LE in value[0..4]), kind 2 = string (length 1..255 UTF-8
 * bytes). 264 B. */
#define IGGY_ID_NUMERIC 1u
#define IGGY_ID_STRING 2u
typedef struct iggy_identifier {
    uint32_t kind;
    uint32_t length;
    uint8_t value[256];
} iggy_identifier;

/* WirePartitioning (primitives/partitioning.rs:24-140): kind 1 = balanced
 * (length 0), 2 = partition id (length 4, u32 LE), 3 = messages key (1..255 B). */
#define IGGY_PART_BALANCED 1u
#define IGGY_PART_PARTITION_ID 2u
#define IGGY_PART_MESSAGES_KEY 3u
typedef struct iggy_partitioning {
    uint32_t kind;
    uint32_t length;
    uint8_t value[256];
} iggy_partitioning;

/* SendMessagesHeader (requests/messages/send_messages.rs:189-195). */
typedef struct iggy_send_messages_header {
    iggy_identifier stream_id;
    iggy_identifier topic_id;
    iggy_partitioning partitioning;
    uint32_t messages_count;
    uint32_t _pad;
} iggy_send_messages_header;

/* SendMessagesHeader::metadata_length / WireEncode::encode (send_messages.rs:197-220):
 * the metadata fields without the u32 length prefix. IGGY_ERR_INVALID_ARGUMENT for an
 * identifier or partitioning that its Rust constructor would refuse (a numeric id
 * not 4 bytes long, an empty or > 255-byte name or key, an unknown kind). */
int iggy_send_messages_header_encode(const iggy_send_messages_header *h, uint8_t *out, uint64_t cap,
                                     uint64_t *out_len);
/* WireDecode for SendMessagesHeader (send_messages.rs:222-241), with the
 * identifier / partitioning decode errors of identifier.rs:194-231 and
 * partitioning.rs:106-140 (UnexpectedEof offsets relative to the field being
 * decoded, as the Rust sub-slice decode reports them). *consumed = bytes used. */
int iggy_send_messages_header_decode(const uint8_t *buf, uint64_t len, iggy_send_messages_header *out,
                                     uint64_t *consumed, iggy_wire_error *err);
/* SendMessagesEncoder::encoded_size (send_messages.rs:69-79). */
uint64_t iggy_send_messages_encoded_size(const iggy_send_messages_header *h, const iggy_raw_messages *msgs);
/* SendMessagesEncoder::encode (send_messages.rs:89-181), the whole body:
 * [metadata_length u32][stream_id][topic_id][partitioning][messages_count u32][batch],
 * the batch section encoded on the GPU (h->messages_count is ignored: the count is
 * msgs->count, as the encoder takes it from the slice). */
int iggy_codec_send_messages_encode(iggy_codec_ctx *ctx, const iggy_send_messages_header *h,
                                    const iggy_raw_messages *msgs, uint8_t *out, uint64_t cap,
                                    uint64_t *out_len, iggy_wire_error *err);

/* The PollMessages response prefix (polled_messages.rs:61-83). 16 B. */
typedef struct iggy_polled_prefix {
    uint32_t partition_id;
    uint32_t count;
    uint64_t current_offset;
} iggy_polled_prefix;
/* PolledMessages::from_bytes (common/src/types/message/polled_messages.rs:61-90):
 * fewer than 16 bytes -> IGGY_ERR_INVALID_NUMBER_ENCODING; then the records after the
 * prefix as iggy_codec_poll_decode(IGGY_POLL_MODE_SDK) walks them. payload_pos /
 * user_headers_pos are offsets into `bytes` (prefix included). */
int iggy_codec_polled_messages_from_bytes(iggy_codec_ctx *ctx, const uint8_t *bytes, uint64_t len,
                                          iggy_polled_prefix *prefix, iggy_polled_message *out,
                                          uint64_t cap, uint64_t *n, iggy_wire_error *err);

/* ------------------------------------------ server socket side */
/* The consensus frame header (core/binary_protocol/src/consensus/header.rs:49-78):
 * 256 bytes, the frame's total size a u32 at byte 48. */
#define IGGY_FRAME_HEADER_BYTES 256u
#define IGGY_FRAME_SIZE_OFFSET 48u
#define IGGY_MAX_MESSAGE_SIZE (64ull << 20) /* message_bus framing.rs:40 */
/* GenericHeader.command (consensus/header.rs:201-212: offset 16+16+16+4+4+4 = 60), a
 * #[repr(u8)] Command whose CheckedBitPattern admits 0..=ForwardLogoutResult (29)
 * (consensus/command.rs:24-95) */
#define IGGY_FRAME_COMMAND_OFFSET 60u
#define IGGY_FRAME_COMMAND_MAX 29u

/* read_message (core/message_bus/src/framing.rs:107-164) on a connected blocking
 * stream socket: the 256-B header is read into buf, its size field checked against
 * [256, max_message_size] (IGGY_ERR_INVALID_COMMAND otherwise), then the body is read
 * into the tail of the SAME buffer -- one buffer per frame, no reassembly copy. buf
 * is the caller's (the server's 4096-aligned Owned pool, iobuf.rs), registered once
 * with iggy_codec_host_register so the codec's H2D copy of the frame is DMA. EOF
 * before the frame is complete -> IGGY_ERR_CONNECTION_CLOSED, any other I/O error ->
 * IGGY_ERR_TCP_ERROR. Then Message::<GenericHeader>::try_from (consensus_message.rs:
 * 468-500): the header's checked bit pattern (the command byte at 60 must be a Command
 * discriminant, <= 29; every other GenericHeader field is a plain integer or byte
 * array) and GenericHeader::validate (header.rs:246-248: always Ok) -> a bad command is
 * IGGY_ERR_INVALID_COMMAND, reported, as in the reference, after the body has been
 * consumed (the stream stays in sync; *total_size = the bytes consumed, 0 when the
 * size field itself was refused). *total_size = the frame's size.
 * A frame larger than cap -> IGGY_ERR_CAPACITY (err->a = size, *total_size = size):
 * the 256-B header is in buf and the body is still on the socket. The reference grows
 * its buffer in place (framing.rs:150-160); here the caller takes a buffer of >= size
 * bytes, copies the header into it and finishes the frame with iggy_frame_read_rest.
 * No device work. */
int iggy_frame_read(int fd, uint8_t *buf, uint64_t cap, uint64_t max_message_size, uint64_t *total_size,
                    iggy_wire_error *err);
/* the rest of a frame iggy_frame_read left at IGGY_ERR_CAPACITY: buf[0..256) holds its
 * header (copied by the caller), size = the *total_size it reported; the body is read
 * into buf[256..size) and the header validated as above. */
int iggy_frame_read_rest(int fd, uint8_t *buf, uint64_t size, iggy_wire_error *err);

/* convert_request_message (core/server_common/src/send_messages.rs:459-478) fused
 * with admit_wire_request (:480-540) on one framed SendMessages request
 * [RoutedRequestHeader 256 B][body] of `len` bytes (as iggy_frame_read leaves it):
 *  - a body that is ONE canonical batch (the encrypt ingest path re-entering) is
 *    Verify-decoded on the GPU; it must carry messages, fill the body exactly and
 *    carry this namespace's partition_id (else IGGY_ERR_INVALID_COMMAND); the frame
 *    is kept as is (copied to out);
 *  - otherwise the producer's wire form [u32 metadata_length][SendMessagesHeader]
 *    [batch]: the metadata decoded (iggy_send_messages_header_decode, every failure
 *    IGGY_ERR_INVALID_COMMAND, its length must match), then iggy_codec_admit_batch
 *    with its messages_count (GPU Verify decode, partition stamped, batch checksum
 *    recomputed or zeroed per checksum_mode); out = [the request header with size =
 *    256 + batch_length][the admitted batch].
 * Checksum failures keep their typed errors (batch_error). *out_len = bytes written;
 * hdr_out (nullable) = the batch header of the output. */
int iggy_codec_convert_request(iggy_codec_ctx *ctx, const uint8_t *frame, uint64_t len, uint64_t partition_id,
                               int checksum_mode, uint8_t *out, uint64_t cap, uint64_t *out_len,
                               iggy_batch_header *hdr_out, iggy_wire_error *err);

/* ------------------------------------------ SDK producer batching */
/* The producer's buffering in front of the encoder: the background shard buffer
 * (core/sdk/src/clients/producer_sharding.rs:136-247: one entry per send call,
 * flush when entries >= batch_length or buffered bytes >= batch_size, consecutive
 * same-destination entries merged into one request) and direct sends
 * (producer.rs:406-470: each call split into chunks of batch_length messages,
 * MAX_BATCH_LENGTH = 1 000 000 when 0, clients/mod.rs:41; a failed chunk fails the
 * rest of its call). Message bytes are appended into pinned host staging, so the
 * flush's H2D copies are DMA; every request body is encoded on the GPU through the
 * context's asynchronous slots (up to 8 in flight). */
#define IGGY_MAX_BATCH_LENGTH 1000000ull
typedef struct iggy_producer_config {
    uint64_t batch_length;  /* background: entries that trigger a flush (0 = none); direct: chunk size */
    uint64_t batch_size;    /* background: buffered bytes that trigger a flush (0 = none) */
    uint32_t direct;        /* 1 = direct sends, 0 = background shard buffer */
    uint32_t _pad;
    uint64_t _reserved;
} iggy_producer_config;

/* One request body written by iggy_producer_flush. 72 B. */
typedef struct iggy_producer_request {
    uint64_t offset, length;          /* the SendMessages body at out[offset, offset + length) */
    uint64_t first_message, messages; /* its messages, indices in append order since the last flush */
    uint32_t entry;                   /* the (first) append call it came from */
    uint32_t sent;                    /* 0: not encoded (an earlier chunk of its direct call failed) */
    iggy_wire_error error;            /* the encoder's verdict for this body */
} iggy_producer_request;

typedef struct iggy_producer iggy_producer;
int iggy_producer_create(iggy_codec_ctx *ctx, const iggy_producer_config *cfg, iggy_producer **out);
void iggy_producer_destroy(iggy_producer *p);
/* One send call (a ShardMessage, producer_sharding.rs:91-109): the messages are
 * copied into the staging; *flush_due = the background trigger fired (direct mode:
 * always 1). */
int iggy_producer_append(iggy_producer *p, const iggy_identifier *stream_id, const iggy_identifier *topic_id,
                         const iggy_partitioning *partitioning, const iggy_raw_messages *msgs, int *flush_due);
/* Buffered entries / bytes (ShardMessage::get_size_bytes, producer_sharding.rs:99-109:
 * 2 + identifier length for stream and topic, 64 + payload + user headers per message). */
int iggy_producer_pending(const iggy_producer *p, uint64_t *entries, uint64_t *bytes, uint64_t *messages);
/* flush_buffer (producer_sharding.rs:215-247) / send_internal's chunking
 * (producer.rs:433-455): every request body is encoded into `out` (cap bytes; register
 * it with iggy_codec_host_register for asynchronous copies) and described in reqs
 * (max_reqs). Returns 0 when every body was written (each carries its own verdict in
 * reqs[k].error), IGGY_ERR_CAPACITY (err->a = bytes or requests needed) when out or
 * reqs is too small (nothing is flushed then). The buffer is empty afterwards.
 * When a submit or wait fails part-way (IGGY_ERR_DEVICE, or IGGY_ERR_BUSY when every
 * slot of the context is held by operations the caller has not retired), *nreqs =
 * the requests already written: reqs[0..*nreqs) are complete (each with its own
 * verdict) and are the caller's to send; their messages leave the buffer, which keeps
 * the rest, so a retry never re-sends a request. A failed append leaves the buffer
 * unchanged. */
int iggy_producer_flush(iggy_producer *p, uint8_t *out, uint64_t cap, iggy_producer_request *reqs,
                        uint64_t max_reqs, uint64_t *nreqs, iggy_wire_error *err);

/* ------------------------------------------------------------- profiling */
/* When enabled, the context brackets the dominant kernel of every decode /
 * encode with hipEvents on the launch stream and accumulates its duration. */
int iggy_codec_profile_enable(iggy_codec_ctx *ctx, int enable);
/* Returns the number of bracketed launches and their summed duration (ms)
 * for `which` (0 = decode main kernel, 1 = encode main kernel), then resets. */
int iggy_codec_profile_read(iggy_codec_ctx *ctx, int which, uint64_t *launches, double *total_ms);

/* Host-side counters of a context since its creation (cumulative; diff two reads).
 * The evidence that the asynchronous host API does not serialise its copies: a
 * submit of pinned buffers of a size seen before stages nothing, records no settle
 * event, waits for nothing and allocates nothing. */
typedef struct iggy_host_stats {
    uint64_t pinned_h2d_bytes;   /* caller bytes DMA'd straight from pinned memory */
    uint64_t staged_bytes;       /* pageable caller bytes staged through the context's chunks */
    uint64_t settle_events;      /* events recorded for xfer_settle (staged copies only) */
    uint64_t host_waits;         /* blocking waits inside the codec's copy helpers */
    uint64_t device_allocs;      /* device scratch (re)allocations (process-wide) */
    uint64_t pinned_allocs;      /* pinned / mapped host (re)allocations (process-wide) */
    uint64_t service_posts;      /* records decoded by the resident service (iggy_codec_service_start) */
    uint64_t service_launches;   /* launches of its grid (one per start, and one per idle exit re-entered) */
} iggy_host_stats;
int iggy_codec_host_stats(iggy_codec_ctx *ctx, iggy_host_stats *out);

/* ----------------------------------------------------- resident decode service */
/* Synchronous host decodes of small single-stride records (iggy_codec_decode_batch and
 * the entries built on it: decode_batch_slice_with at C1, batch.rs:391, the reference's
 * own call shape) without a kernel launch per call: the context keeps 8 workgroups
 * resident that poll a host-mapped mailbox, and a record of at most 8 checksum blocks
 * (1 018 frames) that the device can read in place (registered, or copied into the
 * context's mapped staging) is posted to them. Results, errors and positions are those
 * of the launch path. The grid exits after 20 ms without a post and is relaunched by
 * the next call; it holds 8 workgroups of 256 threads (256 VGPRs per wave, 11 KiB of
 * LDS) while alive (the persistent C2 decode grid still fits beside it, measured at the
 * same 0.205 ms). Off by default; _stop (and
 * iggy_codec_destroy) ends it. */
int iggy_codec_service_start(iggy_codec_ctx *ctx);
int iggy_codec_service_stop(iggy_codec_ctx *ctx);

/* Human-readable text for an error kind / validation reason. */
const char *iggy_codec_error_string(uint32_t kind, uint32_t reason);

#ifdef __cplusplus
}
#endif
#endif /* IGGY_CODEC_H */

"""SDK request body, poll prefix and producer batching — TEST INFRASTRUCTURE ONLY.

A pure-Python restatement (small inputs) of the reference's host-side code around
the message batch, used by tests/ as the checker of iggy_amd/csrc/sdk.cpp:

  WireIdentifier encode/decode    core/binary_protocol/src/primitives/identifier.rs:150-231
  WirePartitioning encode/decode  core/binary_protocol/src/primitives/partitioning.rs:42-140
  SendMessagesHeader              core/binary_protocol/src/requests/messages/send_messages.rs:184-241
  SendMessagesEncoder::encode     send_messages.rs:67-181 (the batch section from oracle.encode_batch)
  PolledMessages::from_bytes      core/common/src/types/message/polled_messages.rs:61-90
  Shard buffer / flush_buffer     core/sdk/src/clients/producer_sharding.rs:99-109, 136-247, 288-292
  send_internal chunking          core/sdk/src/clients/producer.rs:406-470 (MAX_BATCH_LENGTH, clients/mod.rs:41)

Pinned by the reference's golden send metadata
(foreign/node/src/wire/message/message-batch.test.ts:98-112: stream 1, topic 2,
balanced, 2 messages -> 120000000104010000000104020000000100 02000000) and the
golden poll body (:62-75, prefix 3 / 101 / 2). Errors are tuples
(kind, reason, a, b, c) with the iggy_error_kind / iggy_validation_reason ids of
include/iggy_codec.h.
"""
from __future__ import annotations

import struct

ERR_UNEXPECTED_EOF, ERR_VALIDATION, ERR_PAYLOAD_TOO_LARGE = 1, 2, 6
ERR_INVALID_UTF8, ERR_UNKNOWN_DISCRIMINANT = 7, 8
ERR_INVALID_NUMBER_ENCODING = 20
V_EMPTY_BATCH, V_NUMERIC_ID_LENGTH, V_STRING_ID_EMPTY = 5, 6, 7
V_BALANCED_LENGTH, V_PARTITION_ID_LENGTH, V_MESSAGES_KEY_EMPTY = 8, 9, 10
TYPE_WIRE_IDENTIFIER, TYPE_WIRE_PARTITIONING = 1, 2
ID_NUMERIC, ID_STRING = 1, 2
PART_BALANCED, PART_PARTITION_ID, PART_MESSAGES_KEY = 1, 2, 3
MAX_BATCH_LENGTH = 1_000_000  # core/sdk/src/clients/mod.rs:41
IGGY_MESSAGE_HEADER_SIZE = 64  # core/common/src/types/message/message_header.rs:23


def eof(offset, need, have):
    return (ERR_UNEXPECTED_EOF, 0, offset, need, max(have, 0))


# ---- fields: (kind, value bytes); identifier.rs:150-162 / partitioning.rs:42-70 encode
def encode_field(kind: int, value: bytes) -> bytes:
    return bytes([kind, len(value)]) + value


def decode_identifier(buf: bytes):
    """identifier.rs:194-231 -> (err | None, (kind, value), consumed)."""
    if len(buf) < 1:
        return eof(0, 1, len(buf)), None, 0
    kind = buf[0]
    if len(buf) < 2:
        return eof(1, 1, len(buf) - 1), None, 0
    length = buf[1]
    if len(buf) - 2 < length:  # read_bytes(buf, 2, length) before the kind match
        return eof(2, length, len(buf) - 2), None, 0
    value = bytes(buf[2:2 + length])
    if kind == ID_NUMERIC:
        if length != 4:
            return (ERR_VALIDATION, V_NUMERIC_ID_LENGTH, length, 0, 0), None, 0
    elif kind == ID_STRING:
        if length == 0:
            return (ERR_VALIDATION, V_STRING_ID_EMPTY, 0, 0, 0), None, 0
        try:
            value.decode("utf-8")
        except UnicodeDecodeError:
            return (ERR_INVALID_UTF8, 0, 2, 0, 0), None, 0
    else:
        return (ERR_UNKNOWN_DISCRIMINANT, 0, TYPE_WIRE_IDENTIFIER, kind, 0), None, 0
    return None, (kind, value), 2 + length


def decode_partitioning(buf: bytes):
    """partitioning.rs:106-140."""
    if len(buf) < 1:
        return eof(0, 1, len(buf)), None, 0
    kind = buf[0]
    if len(buf) < 2:
        return eof(1, 1, len(buf) - 1), None, 0
    length = buf[1]
    if kind == PART_BALANCED:
        if length != 0:
            return (ERR_VALIDATION, V_BALANCED_LENGTH, length, 0, 0), None, 0
        return None, (kind, b""), 2
    if kind == PART_PARTITION_ID:
        if length != 4:
            return (ERR_VALIDATION, V_PARTITION_ID_LENGTH, length, 0, 0), None, 0
        if len(buf) - 2 < 4:  # read_u32_le(buf, 2)
            return eof(2, 4, len(buf) - 2), None, 0
        return None, (kind, bytes(buf[2:6])), 6
    if kind == PART_MESSAGES_KEY:
        if length == 0:
            return (ERR_VALIDATION, V_MESSAGES_KEY_EMPTY, 0, 0, 0), None, 0
        if len(buf) - 2 < length:
            return eof(2, length, len(buf) - 2), None, 0
        return None, (kind, bytes(buf[2:2 + length])), 2 + length
    return (ERR_UNKNOWN_DISCRIMINANT, 0, TYPE_WIRE_PARTITIONING, kind, 0), None, 0


def encode_metadata(stream, topic, part, count: int) -> bytes:
    """SendMessagesHeader::encode (send_messages.rs:214-219)."""
    return encode_field(*stream) + encode_field(*topic) + encode_field(*part) + struct.pack("<I", count)


def decode_metadata(buf: bytes):
    """SendMessagesHeader::decode (send_messages.rs:223-240) -> (err, (stream, topic, part, count), consumed)."""
    e, stream, n = decode_identifier(buf)
    if e:
        return e, None, 0
    pos = n
    e, topic, n = decode_identifier(buf[pos:])
    if e:
        return e, None, 0
    pos += n
    e, part, n = decode_partitioning(buf[pos:])
    if e:
        return e, None, 0
    pos += n
    if len(buf) - pos < 4:
        return eof(pos, 4, len(buf) - pos), None, 0
    count = struct.unpack_from("<I", buf, pos)[0]
    return None, (stream, topic, part, count), pos + 4


def send_messages_body(stream, topic, part, batch: bytes, count: int) -> bytes:
    """SendMessagesEncoder::encode (send_messages.rs:102-117 then the batch): the
    u32 metadata length, the metadata and the batch section."""
    meta = encode_metadata(stream, topic, part, count)
    return struct.pack("<I", len(meta)) + meta + batch


def polled_prefix(buf: bytes):
    """PolledMessages::from_bytes prefix (polled_messages.rs:62-83) -> err | (pid, offset, count)."""
    if len(buf) < 16:
        return (ERR_INVALID_NUMBER_ENCODING, 0, 0, 0, 0)
    return struct.unpack_from("<IQI", buf, 0)


# ---- producer buffering
def shard_message_size(stream, topic, payload_lengths, user_headers_lengths) -> int:
    """ShardMessage::get_size_bytes (producer_sharding.rs:99-109; Identifier length + 2,
    IggyMessage 64 + payload + user headers)."""
    return (len(stream[1]) + 2) + (len(topic[1]) + 2) + sum(
        IGGY_MESSAGE_HEADER_SIZE + p + u for p, u in zip(payload_lengths, user_headers_lengths))


def flush_due(n_entries: int, nbytes: int, batch_length: int, batch_size: int) -> bool:
    """producer_sharding.rs:162-163."""
    return (batch_length != 0 and n_entries >= batch_length) or (batch_size != 0 and nbytes >= batch_size)


def plan_requests(entries, direct: bool, batch_length: int):
    """entries: [(dest, m0, m1)] in append order -> [(entry index, m0, m1)].
    Background: runs of same-destination entries merged (flush_buffer, :226-235;
    same_destination :288-292); direct: each entry in chunks of batch_length
    (MAX_BATCH_LENGTH when 0, producer.rs:436-445). Empty sends are dropped
    (producer.rs:413-415)."""
    plan = []
    if direct:
        mx = batch_length or MAX_BATCH_LENGTH
        for k, (_, m0, m1) in enumerate(entries):
            a = m0
            while a < m1:
                plan.append([k, a, min(a + mx, m1)])
                a += mx
    else:
        for k, (dest, m0, m1) in enumerate(entries):
            if plan and entries[plan[-1][0]][0] == dest:
                plan[-1][2] = m1
                continue
            plan.append([k, m0, m1])
    return [tuple(p) for p in plan if p[2] > p[1]]


# ---- server admission of a framed request: convert_request_message + admit_wire_request
# (core/server_common/src/send_messages.rs:459-540); the batch checks come from the C
# restatement (oracle.decode_batch_slice_with / oracle.admit_batch)
ERR_INVALID_COMMAND = 22


def convert_request(frame: bytes, partition_id: int, checksum_mode: int = 0):
    """-> (rc, err tuple, output bytes)."""
    from oracle import oracle as O

    frame = bytes(frame)
    inv = (ERR_INVALID_COMMAND, (ERR_INVALID_COMMAND, 0, 0, 0, 0), b"")
    if len(frame) < 256:
        return inv
    total = struct.unpack_from("<I", frame, 48)[0]
    if total < 256 or total > len(frame):
        return inv
    body = frame[256:total]
    rc, e, h, _ = O.decode_batch_slice_with(body, 0, want_frames=False)  # decode_batch_slice (Verify)
    if rc == 0:  # :466-476, the canonical-batch shape
        if h.message_count == 0 or len(body) != h.batch_length or h.partition_id != partition_id:
            return inv
        return 0, (0, 0, 0, 0, 0), frame[:total]
    if len(body) < 4:  # admit_wire_request :486-500
        return inv
    mlen = struct.unpack_from("<I", body, 0)[0]
    start = 4 + mlen
    if len(body) < start:
        return inv
    err, meta, consumed = decode_metadata(body[4:start])
    if err or consumed != mlen:
        return inv
    rc, e, ah, admitted = O.admit_batch(body[start:], meta[3], partition_id, checksum_mode)
    if rc:
        return rc, tuple(e.astuple()), b""
    hdr = bytearray(frame[:256])
    struct.pack_into("<I", hdr, 48, 256 + ah.batch_length)
    return 0, (0, 0, 0, 0, 0), bytes(hdr) + admitted


# ---- read_message on a byte stream (core/message_bus/src/framing.rs:107-164) followed by
# Message::<GenericHeader>::try_from (core/server_common/src/consensus_message.rs:468-500)
ERR_CAPACITY, ERR_CONNECTION_CLOSED = 102, 25  # include/iggy_codec.h
COMMAND_OFFSET, COMMAND_MAX = 60, 29  # GenericHeader.command; Command 0..=ForwardLogoutResult


def read_frames(stream: bytes, cap: int, max_message_size: int = 64 << 20):
    """Frames read one after another off `stream` until the first error or its end ->
    [(rc, frame bytes or b"", stream position after the call)]. A frame larger than cap
    is completed as a caller that grows its buffer would (iggy_frame_read_rest)."""
    out, pos = [], 0
    while True:
        if len(stream) - pos < 256:  # read_exact of the header: EOF
            out.append((ERR_CONNECTION_CLOSED, b"", len(stream)))
            return out
        hdr = stream[pos:pos + 256]
        size = struct.unpack_from("<I", hdr, 48)[0]
        if not 256 <= size <= max_message_size:
            out.append((ERR_INVALID_COMMAND, b"", pos + 256))
            return out
        if size > cap:
            out.append((ERR_CAPACITY, b"", pos + 256))  # then the caller resumes the frame
        if len(stream) - pos < size:  # read_exact of the body: EOF
            out.append((ERR_CONNECTION_CLOSED, b"", len(stream)))
            return out
        frame = stream[pos:pos + size]
        pos += size
        if frame[COMMAND_OFFSET] > COMMAND_MAX:  # CheckedBitPattern of Command (command.rs:90-95)
            out.append((ERR_INVALID_COMMAND, b"", pos))
            continue  # the body was consumed: the stream stays in sync
        out.append((0, frame, pos))


# ---- the poll reply body: build_polled_messages_body (core/server/src/responses.rs:1666-1714)
ERR_CANNOT_DECRYPT_DATA = 24
_KEEP = (0, ERR_INVALID_COMMAND, ERR_CANNOT_DECRYPT_DATA, 3, 4)  # + InvalidBatch/MessageChecksum


def build_polled_messages_body(partition_id: int, current_offset: int, fragments, key: bytes | None = None):
    """fragments: [bytes] in order -> (rc, err tuple, body bytes). Decryption through
    the C restatement (oracle.decrypt_batch = decrypt_batch_record); its decode errors
    pass batch_error (server_common/src/send_messages.rs:52-66): InvalidCommand."""
    from oracle import oracle as O

    stream = b"".join(bytes(f) for f in fragments)
    body = bytearray(struct.pack("<IQI", partition_id, current_offset, 0))
    count, pos = 0, 0
    inv = (ERR_INVALID_COMMAND, (ERR_INVALID_COMMAND, 0, 0, 0, 0), b"")
    while pos < len(stream):
        rest = stream[pos:]
        if len(rest) < 256:
            return inv
        bl = struct.unpack_from("<Q", rest, 32)[0]
        if bl < 256 or any(rest[52:256]):
            return inv
        end = pos + bl
        if end > len(stream):
            return inv
        record = stream[pos:end]
        if key is not None:
            rc, e, dec = O.decrypt_batch(key, record)
            if rc:
                kind = rc if rc in _KEEP else ERR_INVALID_COMMAND
                t = tuple(e.astuple()) if kind == rc else (kind, 0, 0, 0, 0)
                return kind, (kind,) + t[1:], b""
            body += dec
        else:
            body += record
        count += struct.unpack_from("<I", rest, 48)[0]
        if count > 0xFFFFFFFF:
            return inv
        pos = end
    struct.pack_into("<I", body, 12, count)
    return 0, (0, 0, 0, 0, 0), bytes(body)

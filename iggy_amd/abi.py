"""ctypes mirrors of the structs declared in include/iggy_codec.h (types only)."""
from __future__ import annotations

import ctypes

u64 = ctypes.c_uint64
u32 = ctypes.c_uint32

# iggy_error_kind
OK = 0
ERR_UNEXPECTED_EOF = 1
ERR_VALIDATION = 2
ERR_INVALID_BATCH_CHECKSUM = 3
ERR_INVALID_MESSAGE_CHECKSUM = 4
ERR_INVALID_TIMESTAMP_DELTA = 5
ERR_PAYLOAD_TOO_LARGE = 6
ERR_INVALID_NUMBER_ENCODING = 20
ERR_INVALID_MESSAGE_PAYLOAD_LENGTH = 21
ERR_INVALID_COMMAND = 22  # IggyError::InvalidCommand (server_common batch_error)
ERR_CONNECTION_CLOSED = 25  # IggyError::ConnectionClosed (message_bus framing.rs:165-171)
ERR_TCP_ERROR = 26
ERR_DEVICE = 100
ERR_INVALID_ARGUMENT = 101
ERR_CAPACITY = 102
ERR_TIMEOUT = 103
ERR_PENDING = 104
ERR_BUSY = 105

OP_DECODE = 1
OP_ENCODE = 2

# iggy_validation_reason
V_NONE = 0
V_BATCH_LENGTH_SHORT = 1
V_BATCH_RESERVED = 2
V_FRAMES_DO_NOT_TILE = 3
V_FRAME_RESERVED = 4
V_EMPTY_BATCH = 5

INTEGRITY_VERIFY = 0
INTEGRITY_LAYOUT_ONLY = 1
POLL_MODE_SDK = 0
POLL_MODE_ITERATOR = 1

BATCH_HEADER_SIZE = 256
FRAME_HEADER_SIZE = 48


class WireError(ctypes.Structure):
    _fields_ = [("kind", u32), ("reason", u32), ("a", u64), ("b", u64), ("c", u64)]

    def astuple(self):
        return (self.kind, self.reason, self.a, self.b, self.c)

    def __repr__(self):
        return f"WireError(kind={self.kind}, reason={self.reason}, a={self.a:#x}, b={self.b:#x}, c={self.c:#x})"


class BatchHeader(ctypes.Structure):
    _fields_ = [
        ("partition_id", u64),
        ("base_offset", u64),
        ("base_timestamp", u64),
        ("origin_timestamp", u64),
        ("batch_length", u64),
        ("batch_checksum", u64),
        ("message_count", u32),
        ("_pad0", u32),
        ("_pad1", u64),
    ]

    def astuple(self):
        return (self.partition_id, self.base_offset, self.base_timestamp, self.origin_timestamp,
                self.batch_length, self.batch_checksum, self.message_count)


class PolledMessage(ctypes.Structure):
    _fields_ = [
        ("checksum", u64),
        ("id_lo", u64),
        ("id_hi", u64),
        ("offset", u64),
        ("timestamp", u64),
        ("origin_timestamp", u64),
        ("payload_pos", u64),
        ("user_headers_pos", u64),
        ("payload_length", u32),
        ("user_headers_length", u32),
        ("_pad", u64),
    ]

    def astuple(self):
        return (self.checksum, self.id_lo, self.id_hi, self.offset, self.timestamp,
                self.origin_timestamp, self.payload_pos, self.user_headers_pos,
                self.payload_length, self.user_headers_length)


class RawMessages(ctypes.Structure):
    _fields_ = [
        ("count", u64),
        ("ids", ctypes.c_void_p),
        ("origin_timestamps", ctypes.c_void_p),
        ("payloads", ctypes.c_void_p),
        ("payload_lengths", ctypes.c_void_p),
        ("user_headers", ctypes.c_void_p),
        ("user_headers_lengths", ctypes.c_void_p),
    ]


class DecodeResult(ctypes.Structure):
    _fields_ = [
        ("header", BatchHeader),
        ("error", WireError),
        ("frame_count", u64),
        ("computed_checksum", u64),
        ("path", u32),
        ("status", u32),
        ("covered", u64),
    ]


class EncodeResult(ctypes.Structure):
    _fields_ = [
        ("header", BatchHeader),
        ("error", WireError),
        ("batch_length", u64),
        ("_pad", u64 * 3),
    ]


LOOKUP_OFFSET = 0
LOOKUP_TIMESTAMP = 1

# ChecksumMode (server_common/src/send_messages.rs:416-432); prepare frame layout
CHECKSUM_COMPUTE = 0
CHECKSUM_SKIP = 1
PREPARE_HEADER_SIZE = 256
PREPARE_SIZE_OFFSET = 48


class SliceQuery(ctypes.Structure):
    """MessageLookup (core/partitions/src/journal.rs:68-95) + already-matched count."""
    _fields_ = [("kind", u32), ("count", u32), ("value", u64), ("ceiling", u64),
                ("already_matched", u32), ("_pad", u32)]


class SliceResult(ctypes.Structure):
    _fields_ = [
        ("selected", u32),
        ("full_body", u32),
        ("start", u64),
        ("end", u64),
        ("matched_messages", u32),
        ("_pad0", u32),
        ("last_matching_offset", u64),
        ("header", BatchHeader),
        ("_pad1", u64 * 3),
    ]

    def astuple(self):
        return (self.selected, self.full_body, self.start, self.end, self.matched_messages,
                self.last_matching_offset) + self.header.astuple()


class Completion(ctypes.Structure):
    """iggy_completion: the outcome of a submitted host-buffer operation."""
    _fields_ = [
        ("op", u32),
        ("_pad0", u32),
        ("header", BatchHeader),
        ("error", WireError),
        ("frame_count", u64),
        ("computed_checksum", u64),
        ("bytes", u64),
        ("_pad1", u64 * 3),
    ]


class HostStats(ctypes.Structure):
    """iggy_host_stats: cumulative host-side counters of a context (diff two reads)."""
    _fields_ = [
        ("pinned_h2d_bytes", u64),
        ("staged_bytes", u64),
        ("settle_events", u64),
        ("host_waits", u64),
        ("device_allocs", u64),
        ("pinned_allocs", u64),
        ("service_posts", u64),
        ("service_launches", u64),
    ]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_ if not k.startswith("_")}


assert ctypes.sizeof(Completion) == 152
assert ctypes.sizeof(HostStats) == 64
assert ctypes.sizeof(SliceQuery) == 32
assert ctypes.sizeof(SliceResult) == 128
assert ctypes.sizeof(BatchHeader) == 64
assert ctypes.sizeof(WireError) == 32
assert ctypes.sizeof(PolledMessage) == 80
assert ctypes.sizeof(DecodeResult) == 128
assert ctypes.sizeof(EncodeResult) == 128


class SegmentRecovery(ctypes.Structure):
    """iggy_segment_recovery (segment_recovery.rs:425-488 index-less walk)."""
    _fields_ = [("found", ctypes.c_uint64), ("start_timestamp", ctypes.c_uint64),
                ("end_timestamp", ctypes.c_uint64), ("end_offset", ctypes.c_uint64),
                ("walked_bytes", ctypes.c_uint64), ("batches", ctypes.c_uint64)]

    def astuple(self):
        return tuple(getattr(self, f) for f, _ in self._fields_)


class ChunkFragment(ctypes.Structure):
    """iggy_chunk_fragment (push_selected_batch_fragments, journal.rs:1096-1137)."""
    _fields_ = [("batch_pos", u64), ("full_body", u32), ("matched_messages", u32), ("body_start", u64),
                ("body_end", u64), ("last_matching_offset", u64), ("_pad", u64)]

    def astuple(self):
        return (self.batch_pos, self.full_body, self.matched_messages, self.body_start, self.body_end,
                self.last_matching_offset)


class ChunkWalk(ctypes.Structure):
    """iggy_chunk_walk (ChunkWalk + carried state, poll_plan.rs:950-1011)."""
    _fields_ = [("consumed", u64), ("corrupt", u32), ("matched", u32), ("last_matching_offset", u64),
                ("has_last_matching_offset", u32), ("fragments", u32), ("error", WireError), ("batches", u64)]

    def astuple(self):
        return (self.consumed, self.corrupt, self.matched,
                self.last_matching_offset if self.has_last_matching_offset else None, self.fragments,
                self.error.astuple(), self.batches)


assert ctypes.sizeof(ChunkFragment) == 48
assert ctypes.sizeof(ChunkWalk) == 72


SEG_OK, SEG_BATCH, SEG_BASE_OFFSET_MISMATCH, SEG_NON_CONTIGUOUS, SEG_OFFSET_OVERFLOW, SEG_EMPTY = range(6)
ERR_INVALID_MESSAGES_COUNT = 23


class SegmentWalk(ctypes.Structure):
    """iggy_segment_walk (walk_segment_payload, state_transfer.rs:715-833)."""
    _fields_ = [("error", u32), ("_pad", u32), ("position", u64), ("expected", u64), ("actual", u64),
                ("source", WireError), ("end_offset", u64), ("start_timestamp", u64), ("end_timestamp", u64),
                ("max_timestamp", u64), ("batches", u64), ("index_entries", u64)]

    def astuple(self):
        return (self.error, self.position, self.expected, self.actual, self.source.astuple(), self.end_offset,
                self.start_timestamp, self.end_timestamp, self.max_timestamp, self.batches, self.index_entries)


assert ctypes.sizeof(SegmentWalk) == 112


ERR_CANNOT_DECRYPT_DATA = 24


class CryptResult(ctypes.Structure):
    """iggy_crypt_result (encrypt_batch_request / decrypt_batch_record,
    server_common/src/send_messages.rs:293-415)."""
    _fields_ = [("error", WireError), ("out_len", u64), ("frame_count", u64), ("batch_checksum", u64)]


assert ctypes.sizeof(CryptResult) == 56


# ---- SDK request body / poll prefix / producer (include/iggy_codec.h "SDK" sections)
ERR_INVALID_UTF8 = 7
ERR_UNKNOWN_DISCRIMINANT = 8
V_NUMERIC_ID_LENGTH = 6
V_STRING_ID_EMPTY = 7
V_BALANCED_LENGTH = 8
V_PARTITION_ID_LENGTH = 9
V_MESSAGES_KEY_EMPTY = 10
TYPE_WIRE_IDENTIFIER = 1
TYPE_WIRE_PARTITIONING = 2
ID_NUMERIC = 1
ID_STRING = 2
PART_BALANCED = 1
PART_PARTITION_ID = 2
PART_MESSAGES_KEY = 3
MAX_BATCH_LENGTH = 1_000_000


class Identifier(ctypes.Structure):
    """WireIdentifier (primitives/identifier.rs:97-180)."""
    _fields_ = [("kind", u32), ("length", u32), ("value", ctypes.c_uint8 * 256)]

    @classmethod
    def numeric(cls, v: int) -> "Identifier":
        return cls.raw(ID_NUMERIC, int(v).to_bytes(4, "little"))

    @classmethod
    def named(cls, s) -> "Identifier":
        return cls.raw(ID_STRING, s.encode() if isinstance(s, str) else bytes(s))

    @classmethod
    def raw(cls, kind: int, value: bytes) -> "Identifier":
        x = cls()
        x.kind, x.length = kind, len(value)
        ctypes.memmove(x.value, value, len(value))
        return x

    def value_bytes(self) -> bytes:
        return bytes(self.value[: self.length])


class Partitioning(Identifier):
    """WirePartitioning (primitives/partitioning.rs:24-100) — same layout."""

    @classmethod
    def balanced(cls) -> "Partitioning":
        return cls.raw(PART_BALANCED, b"")

    @classmethod
    def partition_id(cls, v: int) -> "Partitioning":
        return cls.raw(PART_PARTITION_ID, int(v).to_bytes(4, "little"))

    @classmethod
    def messages_key(cls, key: bytes) -> "Partitioning":
        return cls.raw(PART_MESSAGES_KEY, bytes(key))


class SendMessagesHeader(ctypes.Structure):
    _fields_ = [("stream_id", Identifier), ("topic_id", Identifier), ("partitioning", Partitioning),
                ("messages_count", u32), ("_pad", u32)]


class PolledPrefix(ctypes.Structure):
    _fields_ = [("partition_id", u32), ("count", u32), ("current_offset", u64)]


class ProducerConfig(ctypes.Structure):
    _fields_ = [("batch_length", u64), ("batch_size", u64), ("direct", u32), ("_pad", u32), ("_reserved", u64)]


class ProducerRequest(ctypes.Structure):
    _fields_ = [("offset", u64), ("length", u64), ("first_message", u64), ("messages", u64),
                ("entry", u32), ("sent", u32), ("error", WireError)]


class PollFragment(ctypes.Structure):
    """iggy_poll_fragment: one host span of a poll reply (PollFragments)."""
    _fields_ = [("data", ctypes.c_void_p), ("len", u64)]

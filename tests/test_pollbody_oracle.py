"""The poll reply body restatement (oracle/sdk_ref.build_polled_messages_body,
core/server/src/responses.rs:1666-1714) pinned on the CPU by the reference's own
golden poll body (foreign/node/src/wire/message/message-batch.test.ts:62-75, the same
body in foreign/go/binary_serialization/vsr_response_deserializer_test.go:291-324):
its records, served as fragments of any split, rebuild the body byte for byte."""
import struct

from golden_util import reference_vectors
from oracle import sdk_ref as S


def test_golden_poll_body_from_fragments():
    body = bytes.fromhex(reference_vectors()["poll_body_hex"])
    pid, off, count = struct.unpack_from("<IQI", body, 0)
    records = body[16:]
    for cuts in ([], [256], [100, 300], [len(records) - 1]):
        pts = [0] + cuts + [len(records)]
        frags = [records[a:b] for a, b in zip(pts, pts[1:])]
        rc, e, got = S.build_polled_messages_body(pid, off, frags)
        assert rc == 0 and got == body


def test_truncated_and_malformed_records_are_invalid_command():
    body = bytes.fromhex(reference_vectors()["poll_body_hex"])
    records = body[16:]
    for frags in ([records[:-1]], [records[:200]], [records, b"\x00" * 10]):
        rc, e, got = S.build_polled_messages_body(3, 101, frags)
        assert rc == S.ERR_INVALID_COMMAND and got == b""
    bad = bytearray(records); bad[100] = 1  # reserved header byte
    assert S.build_polled_messages_body(3, 101, [bytes(bad)])[0] == S.ERR_INVALID_COMMAND


def test_count_overflow_is_invalid_command():
    body = bytes.fromhex(reference_vectors()["poll_body_hex"])
    rec = bytearray(body[16:])
    struct.pack_into("<I", rec, 48, 0xFFFFFFFF)
    assert S.build_polled_messages_body(3, 101, [bytes(rec)])[0] == 0
    rc, e, _ = S.build_polled_messages_body(3, 101, [bytes(rec), body[16:]])
    assert rc == S.ERR_INVALID_COMMAND


def test_empty_poll():
    rc, e, got = S.build_polled_messages_body(7, 0, [])
    assert rc == 0 and got == struct.pack("<IQI", 7, 0, 0)

"""CPU checks of the SDK-side host code in the C-ABI library (no device work):
SendMessagesHeader encode/decode (send_messages.rs:184-241 with the identifier /
partitioning codecs of primitives/identifier.rs and partitioning.rs) against the
reference's golden send metadata and the oracle restatement, plus the producer
batching policy of the oracle itself. Byte work: every check is exact."""
import random

import pytest

from golden_util import reference_vectors
from iggy_amd import abi, codec
from oracle import sdk_ref as S

# message-batch.test.ts:98-112 (Rust-generated): stream 1, topic 2, balanced, 2 messages
GOLDEN_METADATA = bytes.fromhex("120000000104010000000104020000000100" + "02000000")


def _hdr(stream, topic, part, count):
    h = abi.SendMessagesHeader()
    h.stream_id = abi.Identifier.raw(*stream)
    h.topic_id = abi.Identifier.raw(*topic)
    h.partitioning = abi.Partitioning.raw(*part)
    h.messages_count = count
    return h


NUM1 = (S.ID_NUMERIC, (1).to_bytes(4, "little"))
NUM2 = (S.ID_NUMERIC, (2).to_bytes(4, "little"))
BAL = (S.PART_BALANCED, b"")


def test_golden_send_metadata():
    meta = codec.send_messages_header_encode(_hdr(NUM1, NUM2, BAL, 2))
    assert len(meta).to_bytes(4, "little") + meta == GOLDEN_METADATA
    # the oracle agrees, and the decode gives it back (send_messages.rs:286-291)
    assert S.send_messages_body(NUM1, NUM2, BAL, b"", 2) == GOLDEN_METADATA
    rc, e, h, n = codec.send_messages_header_decode(GOLDEN_METADATA[4:])
    assert rc == 0 and n == 18 and h.messages_count == 2
    assert (h.stream_id.kind, h.stream_id.value_bytes()) == NUM1
    assert (h.partitioning.kind, h.partitioning.length) == (S.PART_BALANCED, 0)


FIELDS_ID = [NUM1, (S.ID_NUMERIC, b"\xff\xff\xff\xff"), (S.ID_STRING, b"orders"),
             (S.ID_STRING, "strumień-ü".encode()), (S.ID_STRING, b"x" * 255)]
FIELDS_PART = [BAL, (S.PART_PARTITION_ID, (7).to_bytes(4, "little")), (S.PART_MESSAGES_KEY, b"k"),
               (S.PART_MESSAGES_KEY, bytes(range(255)))]


@pytest.mark.parametrize("stream", FIELDS_ID)
@pytest.mark.parametrize("part", FIELDS_PART)
def test_header_roundtrip_matches_oracle(stream, part):
    topic = (S.ID_STRING, b"events")
    meta = codec.send_messages_header_encode(_hdr(stream, topic, part, 123456))
    assert meta == S.encode_metadata(stream, topic, part, 123456)
    rc, e, h, n = codec.send_messages_header_decode(meta + b"trailing batch bytes")
    err, dec, n2 = S.decode_metadata(meta + b"trailing batch bytes")
    assert rc == 0 and err is None and n == n2 == len(meta)
    assert (h.stream_id.kind, h.stream_id.value_bytes()) == dec[0] == stream
    assert (h.partitioning.kind, h.partitioning.value_bytes()) == dec[2] == part
    assert h.messages_count == dec[3] == 123456


def _decode_both(buf):
    rc, e, h, n = codec.send_messages_header_decode(buf)
    err, dec, n2 = S.decode_metadata(buf)
    if err is None:
        assert rc == 0, e
        assert n == n2
    else:
        assert rc == err[0], (e, err)
        assert e.astuple() == err, (buf.hex(), e, err)


# the reference's decode error cases (identifier.rs / partitioning.rs / send_messages.rs tests)
ERROR_CASES = {
    "empty": b"",
    "kind_only": b"\x01",
    "numeric_short_value": b"\x01\x04\x01\x00",
    "numeric_len3": b"\x01\x03\x01\x00\x00",
    "string_empty": b"\x02\x00",
    "string_bad_utf8": b"\x02\x02\xc3\x28",
    "string_overlong": b"\x02\x02\xc0\x80",
    "string_surrogate": b"\x02\x03\xed\xa0\x80",
    "unknown_id_kind": b"\x09\x00",
    "unknown_id_kind_short": b"\x09\x05ab",
    "topic_missing": b"\x01\x04\x01\x00\x00\x00",
    "balanced_len1": b"\x01\x04\x01\x00\x00\x00\x01\x04\x02\x00\x00\x00\x01\x01\x00",
    "pid_len3": b"\x01\x04\x01\x00\x00\x00\x01\x04\x02\x00\x00\x00\x02\x03\x00\x00\x00",
    "pid_short": b"\x01\x04\x01\x00\x00\x00\x01\x04\x02\x00\x00\x00\x02\x04\x07\x00",
    "key_empty": b"\x01\x04\x01\x00\x00\x00\x01\x04\x02\x00\x00\x00\x03\x00",
    "key_short": b"\x01\x04\x01\x00\x00\x00\x01\x04\x02\x00\x00\x00\x03\x05abc",
    "unknown_part": b"\x01\x04\x01\x00\x00\x00\x01\x04\x02\x00\x00\x00\x04\x00",
    "count_short": b"\x01\x04\x01\x00\x00\x00\x01\x04\x02\x00\x00\x00\x01\x00\x02\x00",
}


@pytest.mark.parametrize("name", sorted(ERROR_CASES))
def test_header_decode_errors_match_oracle(name):
    _decode_both(ERROR_CASES[name])


def test_header_decode_fuzz_matches_oracle():
    rng = random.Random(0x1661)
    good = S.encode_metadata((S.ID_STRING, b"stream-a"), NUM2, (S.PART_MESSAGES_KEY, b"key-1"), 9)
    for _ in range(3000):
        b = bytearray(good)
        for _ in range(rng.randint(1, 3)):
            b[rng.randrange(len(b))] = rng.choice([0, 1, 2, 3, 4, 0xC3, 0xFF, rng.randrange(256)])
        _decode_both(bytes(b[: rng.randint(0, len(b))]))


def test_header_encode_refuses_invalid_fields():
    L = codec.lib()
    for bad in [_hdr((S.ID_NUMERIC, b"\x01\x02"), NUM2, BAL, 1), _hdr((S.ID_STRING, b""), NUM2, BAL, 1),
                _hdr((S.ID_STRING, b"\xc3\x28"), NUM2, BAL, 1), _hdr(NUM1, NUM2, (S.PART_BALANCED, b"x"), 1),
                _hdr(NUM1, NUM2, (S.PART_MESSAGES_KEY, b""), 1), _hdr(NUM1, (7, b"ab"), BAL, 1)]:
        with pytest.raises(codec.CodecError) as ei:
            codec.send_messages_header_encode(bad)
        assert ei.value.rc == abi.ERR_INVALID_ARGUMENT


def test_polled_prefix_oracle_on_golden_poll_body():
    ref = reference_vectors()
    body = bytes.fromhex(ref["poll_body_hex"])
    p = ref["poll_prefix"]
    assert S.polled_prefix(body) == (p["partition_id"], p["current_offset"], p["count"])
    assert S.polled_prefix(body[:15])[0] == S.ERR_INVALID_NUMBER_ENCODING


def test_producer_plan_oracle():
    a, b = ("s", "t", "p1"), ("s", "t", "p2")
    entries = [(a, 0, 3), (a, 3, 5), (b, 5, 9), (a, 9, 10), (a, 10, 10)]
    assert S.plan_requests(entries, direct=False, batch_length=0) == [(0, 0, 5), (2, 5, 9), (3, 9, 10)]
    assert S.plan_requests(entries, direct=True, batch_length=2) == [
        (0, 0, 2), (0, 2, 3), (1, 3, 5), (2, 5, 7), (2, 7, 9), (3, 9, 10)]
    assert S.flush_due(3, 10, 3, 0) and not S.flush_due(2, 10, 3, 0) and S.flush_due(1, 100, 0, 100)
    st, tp = (S.ID_STRING, b"ab"), NUM1
    assert S.shard_message_size(st, tp, [10, 0], [0, 5]) == 4 + 6 + 64 * 2 + 15

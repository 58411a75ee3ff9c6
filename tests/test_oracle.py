"""The oracle pinned against the reference's golden vectors and libxxhash
fixtures (CPU only). If these fail, no GPU parity claim stands."""
import struct

import numpy as np
import pytest

from golden_util import batch_cases, expect_matches, reference_vectors, xxh3_vectors
from iggy_amd import abi
from oracle import oracle as O


def test_xxh3_matches_libxxhash_fixtures():
    blob, vecs = xxh3_vectors()
    for v in vecs:
        d = blob[v["offset"]: v["offset"] + v["length"]]
        assert O.xxh3_64(d) == v["xxh3"], v["length"]
        assert O.xxh3_64_fast(d) == v["xxh3"], v["length"]


def test_golden_produce_batch_checksums():
    ref = reference_vectors()
    rec = np.frombuffer(bytes.fromhex(ref["produce_batch_hex"]), dtype=np.uint8)
    rc, e, h, frames = O.decode_batch_slice_with(rec, abi.INTEGRITY_VERIFY)
    assert rc == 0, e
    assert h.batch_checksum == ref["produce_batch_checksum"]
    assert h.message_count == 2 and h.origin_timestamp == 1000 and h.partition_id == 0
    for i, m in enumerate(ref["messages"]):
        assert struct.unpack_from("<Q", rec, 256 + int(frames[i]))[0] == m["checksum"]


def test_golden_produce_batch_encodes_byte_for_byte():
    ref = reference_vectors()
    msgs = ref["messages"]
    ids = np.array([m["id"] & (2**64 - 1) for m in msgs for _ in (0,)], dtype=np.uint64)
    ids = np.array([[m["id"], 0] for m in msgs], dtype=np.uint64).reshape(-1)
    ots = np.array([m["origin_timestamp"] for m in msgs], dtype=np.uint64)
    payloads = np.frombuffer(b"".join(m["payload"].encode() for m in msgs), dtype=np.uint8).copy()
    pls = np.array([len(m["payload"]) for m in msgs], dtype=np.uint32)
    uhs = np.frombuffer(b"".join(m["user_headers"].encode() for m in msgs), dtype=np.uint8).copy()
    uhl = np.array([len(m["user_headers"]) for m in msgs], dtype=np.uint32)
    raw = abi.RawMessages(2, ids.ctypes.data, ots.ctypes.data, payloads.ctypes.data,
                          pls.ctypes.data, uhs.ctypes.data, uhl.ctypes.data)
    rc, e, out = O.encode_batch(raw)
    assert rc == 0, e
    assert out.hex() == ref["produce_batch_hex"]


def test_golden_poll_body_sdk_and_iterator():
    ref = reference_vectors()
    body = bytes.fromhex(ref["poll_body_hex"])
    pid, cur, cnt = struct.unpack_from("<IQI", body, 0)
    assert (pid, cur, cnt) == (3, 101, 2)
    recs = np.frombuffer(body[16:], dtype=np.uint8)
    for mode in (abi.POLL_MODE_SDK, abi.POLL_MODE_ITERATOR):
        rc, e, msgs = O.poll_decode(recs, mode)
        assert rc == 0, e
        assert len(msgs) == 2
        for got, m in zip(msgs, ref["messages"]):
            assert got.id_lo == m["id"] and got.id_hi == 0
            assert got.offset == m["offset"] and got.timestamp == m["timestamp"]
            assert got.origin_timestamp == m["origin_timestamp"]
            assert got.checksum == m["checksum"]
            assert bytes(recs[got.payload_pos: got.payload_pos + got.payload_length]) == m["payload"].encode()
            assert bytes(recs[got.user_headers_pos: got.user_headers_pos + got.user_headers_length]) == m["user_headers"].encode()
    # the record itself verifies (stamped checksum from the Rust server)
    rc, e, h, _ = O.decode_batch_slice_with(recs, abi.INTEGRITY_VERIFY)
    assert rc == 0, e
    assert h.batch_checksum == ref["poll_record_checksum"]


def test_golden_poll_rejects_nonzero_frame_reserved():
    """message-batch.test.ts:140-147"""
    ref = reference_vectors()
    body = bytearray(bytes.fromhex(ref["poll_body_hex"]))
    body[16 + 256 + 40] = 1
    rc, e, _ = O.poll_decode(np.frombuffer(bytes(body[16:]), dtype=np.uint8), abi.POLL_MODE_SDK)
    assert rc == abi.ERR_INVALID_MESSAGE_PAYLOAD_LENGTH


@pytest.mark.parametrize("case", batch_cases(), ids=lambda c: c["name"])
def test_oracle_against_fixture_cases(case):
    rc, e, h, frames = O.decode_batch_slice_with(case["data"], case["integrity"])
    assert expect_matches(case["expect"], e), (case["name"], e)
    assert rc == case["expect"]["kind"]
    if rc == 0 and case["frames"] is not None:
        assert list(frames) == case["frames"]


def test_stamp_matches_recompute():
    rec = O.synth_batch(50, 100, 300)
    rc, e, h, stamped = O.stamp_batch(rec.copy(), 123, 456)
    assert rc == 0
    rc2, e2, h2, _ = O.decode_batch_slice_with(np.frombuffer(stamped, dtype=np.uint8), 0)
    assert rc2 == 0, e2
    assert (h2.base_offset, h2.base_timestamp) == (123, 456)


def test_synth_batches_verify():
    for n, lo, hi in [(1, 0, 0), (30, 1024, 1024), (200, 64, 4096), (100, 10, 250)]:
        rec = O.synth_batch(n, lo, hi)
        rc, e, h, frames = O.decode_batch_slice_with(rec, 0)
        assert rc == 0, (n, lo, hi, e)
        assert len(frames) == n

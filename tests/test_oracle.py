"""The oracle pinned against the reference's golden vectors and libxxhash
fixtures (CPU only). If these fail, no GPU parity claim stands."""
import struct

import numpy as np
import pytest

from golden_util import batch_cases, expect_matches, reference_vectors, xxh3_vectors
from iggy_amd import abi
from oracle import oracle as O


def _prepare_frame(batch, size=None, trailing=b""):
    """[PrepareHeader 256 B (size at 48)][batch][trailing], as server_common's
    prepare_from_owned builds it (send_messages.rs:690-705)."""
    body = bytes(batch) + trailing
    hdr = bytearray(256)
    struct.pack_into("<I", hdr, 48, 256 + len(body) if size is None else size)
    return np.frombuffer(bytes(hdr) + body, dtype=np.uint8).copy()


def _wire_batch(n=7, seed=3):
    from iggy_amd.codec import raw_messages
    rng = np.random.default_rng(seed)
    pls = rng.integers(1, 300, size=n).astype(np.uint32)
    ids = rng.integers(1, 2**63, size=2 * n, dtype=np.uint64)
    ots = (1_700_000_000_000_000 + np.arange(n)).astype(np.uint64)
    pay = rng.integers(0, 256, size=int(pls.sum()), dtype=np.uint8)
    rc, e, out = O.encode_batch(raw_messages(ids, ots, pay, pls), 0)
    assert rc == 0, e
    return np.frombuffer(out, dtype=np.uint8).copy()


def test_decode_prepare_mirrors_server_common_tests():
    # send_messages.rs:721-745: trusted and validating agree on a stamped batch
    rec = O.synth_batch(40, 10, 500, 0)
    fr = _prepare_frame(rec)
    rc, e, h = O.decode_prepare(fr, True)
    rc2, e2, h2 = O.decode_prepare(fr, False)
    assert rc == 0 and rc2 == 0, (e, e2)
    assert h.astuple() == h2.astuple() and h.message_count == 40
    # :747-766: a mutated stored batch checksum fails only the validating decode
    bad = fr.copy()
    bad[256 + 40] ^= 0xFF
    assert O.decode_prepare(bad, True)[0] == abi.ERR_INVALID_BATCH_CHECKSUM
    assert O.decode_prepare(bad, False)[0] == 0
    # :769-782: size below the header size
    for size in (0, 255):
        assert O.decode_prepare(_prepare_frame(rec, size=size), True)[0] == abi.ERR_INVALID_COMMAND
    # :947-966: payload corruption under an intact checksum field
    bad = fr.copy()
    bad[512 + 48] ^= 0xFF
    assert O.decode_prepare(bad, True)[0] == abi.ERR_INVALID_MESSAGE_CHECKSUM
    assert O.decode_prepare(bad, False)[0] == 0
    # :1292-1307: trailing bytes past batch_length (size covers them)
    for junk in (b"\x00", b"\x01" * 7, b"\x00" * 64):
        assert O.decode_prepare(_prepare_frame(rec, trailing=junk), True)[0] == abi.ERR_INVALID_COMMAND
    # a size that overruns the buffer, and a tiling break (structural -> InvalidCommand)
    assert O.decode_prepare(_prepare_frame(rec, size=256 + rec.size + 1), True)[0] == abi.ERR_INVALID_COMMAND
    brk = fr.copy()
    brk[512 + 44] = 1  # first frame's reserved bytes
    assert O.decode_prepare(brk, True)[0] == abi.ERR_INVALID_COMMAND


def test_admit_batch_mirrors_server_common_tests():
    wire = _wire_batch()
    # :1053-1090: admitted, partition stamped, checksum recomputed over the stamped header
    rc, e, h, out = O.admit_batch(wire, 7, 5, abi.CHECKSUM_COMPUTE)
    assert rc == 0, e
    assert h.partition_id == 5
    stamped = O.decode_batch_slice_with(np.frombuffer(out, dtype=np.uint8), abi.INTEGRITY_VERIFY)
    assert stamped[0] == 0 and stamped[2].partition_id == 5
    assert out[256:] == wire[256:].tobytes()
    # :1121-1150: Skip leaves the checksum zero until stamp
    rc, e, h, out = O.admit_batch(wire, 7, 5, abi.CHECKSUM_SKIP)
    assert rc == 0 and h.batch_checksum == 0 and struct.unpack_from("<Q", out, 40)[0] == 0
    # :1093-1104: a tampered body keeps its integrity error
    bad = wire.copy()
    bad[256 + 48 + 3] ^= 0x10
    assert O.admit_batch(bad, 7, 5)[0] == abi.ERR_INVALID_MESSAGE_CHECKSUM
    # :1106-1119: metadata count mismatch
    assert O.admit_batch(wire, 6, 5)[0] == abi.ERR_INVALID_COMMAND
    # trailing bytes past batch_length (:1260-1278 at the wire form)
    assert O.admit_batch(np.concatenate([wire, np.zeros(3, dtype=np.uint8)]), 7, 5)[0] == abi.ERR_INVALID_COMMAND
    # :1015-1050: an empty batch (header only, valid checksum) is rejected
    empty = np.zeros(256, dtype=np.uint8)
    struct.pack_into("<Q", empty, 32, 256)
    hdr = abi.BatchHeader()
    hdr.batch_length = 256
    struct.pack_into("<Q", empty, 40, O.calculate_batch_checksum(hdr, b""))
    assert O.decode_batch_slice_with(empty, abi.INTEGRITY_VERIFY)[0] == 0
    assert O.admit_batch(empty, 0, 5)[0] == abi.ERR_INVALID_COMMAND


def _segment(sizes, start_offset=100, seed=1):
    """Batches stamped back to back as a partition's segment file (base offsets
    contiguous from start_offset)."""
    recs, off = [], start_offset
    for k, (n, pl) in enumerate(sizes):
        r = O.synth_batch(n, pl, pl + 50, 0, seed=seed + k)
        rc, e, h, r2 = O.stamp_batch(r, off, 1_000 + k)
        assert rc == 0, e
        recs.append(np.frombuffer(r2, dtype=np.uint8))
        off += n
    return np.concatenate(recs), recs


def test_recover_segment_walk():
    seg, recs = _segment([(5, 100), (7, 300), (3, 10), (9, 2000)])
    rc, out = O.recover_segment(seg, 100)
    assert rc == 0 and out.found == 1 and out.batches == 4
    assert out.end_offset == 100 + 5 + 7 + 3 + 9 - 1 and out.walked_bytes == seg.size
    assert out.start_timestamp == 1000 and out.end_timestamp == 1003
    # torn tail: the last batch cut short stops the walk before it
    rc, out = O.recover_segment(seg[:-10], 100)
    assert out.batches == 3 and out.walked_bytes == seg.size - recs[-1].size
    # a corrupt payload in batch 2 (index 1) stops the walk after batch 1
    bad = seg.copy()
    bad[recs[0].size + 256 + 48 + 5] ^= 1
    rc, out = O.recover_segment(bad, 100)
    assert out.batches == 1 and out.end_offset == 104
    # an offset gap (wrong start offset from the file name) accepts nothing
    rc, out = O.recover_segment(seg, 99)
    assert out.found == 0 and out.batches == 0 and out.walked_bytes == 0 and out.end_offset == 99


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


# ---- poll-path slicing (core/partitions/src/journal.rs:1025-1137)
def _stamped(n, lo, hi, base_offset, base_ts, seed=7):
    rec = O.synth_batch(n, lo, hi, 0, seed=seed)
    rc, e, h, out = O.stamp_batch(rec.copy(), base_offset, base_ts)
    assert rc == 0, e
    return np.frombuffer(out, dtype=np.uint8).copy()


def test_select_slice_timestamp_at_exact_broker_time():
    """journal.rs:1496-1533: three 8-byte messages, producer clock 900+i, broker
    base_timestamp 1000; a poll at 1000 takes the whole batch, at 1001 nothing."""
    ids = np.array([1, 0, 2, 0, 3, 0], dtype=np.uint64)
    ots = np.array([900, 901, 902], dtype=np.uint64)
    pay = np.frombuffer(b"abcdefgh" * 3, dtype=np.uint8).copy()
    pls = np.full(3, 8, dtype=np.uint32)
    raw = abi.RawMessages(3, ids.ctypes.data, ots.ctypes.data, pay.ctypes.data, pls.ctypes.data, None, None)
    rc, e, enc = O.encode_batch(raw, 1)
    assert rc == 0, e
    rc, e, h, rec = O.stamp_batch(np.frombuffer(enc, dtype=np.uint8).copy(), 0, 1000)
    rec = np.frombuffer(rec, dtype=np.uint8)
    rc, r, hdr = O.select_slice(rec, abi.LOOKUP_TIMESTAMP, 1000, 10)
    assert rc == 0 and r.selected and r.matched_messages == 3 and r.full_body
    assert hdr == bytes(rec[:256])
    rc, r, hdr = O.select_slice(rec, abi.LOOKUP_TIMESTAMP, 1001, 10)
    assert rc == 0 and not r.selected and hdr is None


def test_selected_slices_are_valid_batches():
    """A partial selection is served as [rewritten header][blob slice]: it must decode
    (Verify) on its own, with the clamped count and recomputed checksum."""
    rec = _stamped(400, 10, 700, 5000, 77)
    n_ok = 0
    for value, count, ceiling in [(5000, 10, 2**64 - 1), (5123, 57, 2**64 - 1), (5390, 100, 2**64 - 1),
                                  (5100, 1000, 5200), (4000, 3, 2**64 - 1), (5399, 1, 2**64 - 1)]:
        rc, r, hdr = O.select_slice(rec, abi.LOOKUP_OFFSET, value, count, ceiling)
        assert rc == 0 and r.selected
        if r.full_body:
            continue
        sliced = np.frombuffer(hdr + bytes(rec[256 + r.start: 256 + r.end]), dtype=np.uint8)
        rc2, e2, h2, frames = O.decode_batch_slice_with(sliced, abi.INTEGRITY_VERIFY)
        assert rc2 == 0, (value, count, ceiling, e2)
        assert h2.message_count == r.matched_messages and h2.base_offset == 5000
        assert h2.batch_checksum == r.header.batch_checksum
        n_ok += 1
    assert n_ok >= 4


def test_select_slice_non_monotone_offsets_keep_unselected_inside():
    """A frame whose offset is below the query between two selected ones stays in the
    byte range (and in the checksum walk) but not in matched_messages."""
    rec = _stamped(6, 100, 100, 0, 1)
    S = 48 + 100
    for i, d in enumerate([0, 9, 3, 9, 9, 1]):  # offset_delta rewrite (layout stays valid)
        struct.pack_into("<I", rec, 256 + i * S + 24, d)
    rc, r, hdr = O.select_slice(rec, abi.LOOKUP_OFFSET, 5, 3)
    assert rc == 0 and r.selected
    assert (r.start, r.end, r.matched_messages, r.last_matching_offset) == (1 * S, 5 * S, 3, 9)
    assert r.header.message_count == 3 and r.header.batch_length == 256 + 4 * S


def test_oracle_walk_disk_chunk_semantics():
    """poll_plan.rs:950-1011 on composed chunks: fragments follow select_batch_slice per
    batch with the running match count; Verify stops on a batch checksum as corrupt."""
    recs, off = [], 100
    for k, n in enumerate((10, 20, 5)):
        r = O.synth_batch(n, 50, 50, 0, seed=k)
        rc, e, h, out = O.stamp_batch(r, off, 1000 + k)
        recs.append(np.frombuffer(out, dtype=np.uint8).copy())
        off += n
    chunk = np.concatenate(recs)
    starts = np.cumsum([0] + [r.size for r in recs])
    rc, w, fr, hd = O.walk_disk_chunk(chunk, abi.LOOKUP_OFFSET, 105, 12)
    assert rc == 0 and w.matched == 12 and w.fragments == 2 and w.batches == 2
    assert w.consumed == starts[2]            # stopped by the count before batch 2
    assert fr[0].full_body == 0 and fr[0].matched_messages == 5 and fr[1].matched_messages == 7
    assert w.last_matching_offset == 116
    bad = chunk.copy()
    bad[starts[1] + 41] ^= 1                  # batch 1's checksum byte
    rc, w, fr, hd = O.walk_disk_chunk(bad, abi.LOOKUP_OFFSET, 0, 100, integrity=0)
    assert w.corrupt == 1 and w.consumed == starts[1] and w.fragments == 1
    rc, w, fr, hd = O.walk_disk_chunk(bad, abi.LOOKUP_OFFSET, 0, 100, integrity=1)
    assert w.corrupt == 0 and w.consumed == chunk.size and w.matched == 35


def test_oracle_walk_segment_payload_semantics():
    """state_transfer.rs:715-833: stats, a 24-B index entry for the first batch and
    every >= 64 KiB, and the first invalid byte's error."""
    recs, off = [], 500
    for k, (n, pl) in enumerate(((100, 1000), (30, 50), (200, 1000), (10, 10))):
        r = O.synth_batch(n, pl, pl, 0, seed=k)
        rc, e, h, out = O.stamp_batch(r, off, 2000 + (k * 7) % 3)
        recs.append(np.frombuffer(out, dtype=np.uint8).copy())
        off += n
    seg = np.concatenate(recs)
    starts = np.cumsum([0] + [r.size for r in recs])
    rc, w, idx = O.walk_segment_payload(seg, 500)
    assert rc == 0 and w.error == abi.SEG_OK and w.batches == 4 and w.end_offset == 839
    assert (w.start_timestamp, w.end_timestamp, w.max_timestamp) == (2000, 2000, 2002)
    ents = [struct.unpack_from("<QQQ", idx, 24 * i) for i in range(w.index_entries)]
    assert ents[0] == (500, 2000, 0)
    assert all(e[2] in starts for e in ents) and ents[1][2] >= 65536
    rc, w, _ = O.walk_segment_payload(seg, 501)
    assert w.error == abi.SEG_BASE_OFFSET_MISMATCH and (w.expected, w.actual) == (501, 500)
    rc, w, _ = O.walk_segment_payload(seg[: starts[2] + 10], 500)
    assert w.error == abi.SEG_BATCH and w.position == starts[2] and w.source.kind == abi.ERR_INVALID_COMMAND
    rc, w, _ = O.walk_segment_payload(seg[:0], 500)
    assert w.error == abi.SEG_EMPTY

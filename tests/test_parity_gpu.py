"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the
golden fixtures. Integer/byte work, so every comparison is bit-exact."""
import ctypes
import struct

import numpy as np
import pytest

from golden_util import batch_cases, expect_matches, reference_vectors, xxh3_vectors
from iggy_amd import abi
from iggy_amd.torch_io import to_device, to_host
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cx():
    from iggy_amd.codec import Codec
    c = Codec(0)
    yield c
    c.close()


def _same(a_rc, a_e, b_rc, b_e):
    assert a_rc == b_rc, (a_e, b_e)
    assert a_e.astuple() == b_e.astuple()


@pytest.mark.parametrize("case", batch_cases(), ids=lambda c: c["name"])
@pytest.mark.parametrize("integrity", [0, 1])
def test_fixture_cases(cx, case, integrity):
    rc, e, h, frames = cx.decode_batch_slice_with(case["data"], integrity)
    orc, oe, oh, of = O.decode_batch_slice_with(case["data"], integrity)
    _same(rc, e, orc, oe)
    if integrity == case["integrity"]:
        assert expect_matches(case["expect"], e)
    if rc == 0:
        assert h.astuple() == oh.astuple()
        assert list(frames) == list(of)


def test_golden_produce_and_poll(cx):
    ref = reference_vectors()
    rec = np.frombuffer(bytes.fromhex(ref["produce_batch_hex"]), dtype=np.uint8)
    rc, e, h, _ = cx.decode_batch_slice_with(rec, 0)
    assert rc == 0, e
    assert h.batch_checksum == ref["produce_batch_checksum"]
    body = bytes.fromhex(ref["poll_body_hex"])
    recs = np.frombuffer(body[16:], dtype=np.uint8)
    for mode in (0, 1):
        rc, e, msgs = cx.poll_decode(recs, mode)
        assert rc == 0, e
        orc, oe, om = O.poll_decode(recs, mode)
        assert [m.astuple() for m in msgs] == [m.astuple() for m in om]
        assert msgs[1].checksum == 0xc0b78e751c7e6bd6 and msgs[1].offset == 101


def test_xxh3_one_shot_vectors(cx):
    blob, vecs = xxh3_vectors()
    for v in vecs[::7] + vecs[-6:]:
        d = blob[v["offset"]: v["offset"] + v["length"]]
        assert cx.xxh3_64(d) == v["xxh3"], v["length"]


def _check_decode(cx, rec):
    for integ in (0, 1):
        rc, e, h, frames = cx.decode_batch_slice_with(rec, integ)
        orc, oe, oh, of = O.decode_batch_slice_with(rec, integ)
        _same(rc, e, orc, oe)
        if rc == 0:
            assert np.array_equal(frames, of)


@pytest.mark.parametrize("n,pl", [(1, 0), (1, 200), (7, 1024), (24, 64), (25, 64), (120, 16),
                                  (122, 1024), (123, 1024), (250, 1024), (251, 1024), (506, 1024),
                                  (3000, 1024), (4097, 256), (20000, 1024), (1000, 256),
                                  (300, 193), (301, 5000), (64, 1000),
                                  # grids sized to small records (<= one producer WG per 128
                                  # frames of 48 B): frames at or near that bound
                                  (30000, 0), (70000, 8)])
def test_uniform_random_batches(cx, n, pl):
    rec = O.synth_batch(n, pl, pl, 0, seed=0x16619E3779B97F4A ^ n)
    _check_decode(cx, rec)


@pytest.mark.parametrize("n,lo,hi,uh", [(200, 64, 4096, 0), (1000, 0, 300, 7), (50, 5000, 70000, 0),
                                        (5000, 64, 4096, 0), (333, 1, 2, 3),
                                        # small variable frames: a general grid of one WG per 64 KiB
                                        (40000, 0, 40, 0)])
def test_variable_random_batches(cx, n, lo, hi, uh):
    rec = O.synth_batch(n, lo, hi, uh, seed=0xABCDEF ^ n)
    _check_decode(cx, rec)


def _device_decode(cx, rec, integrity, cap=None):
    """decode_device on a torch-resident copy of rec: (result, positions[:frame_count])."""
    import torch
    n = rec.size // 48 + 1 if cap is None else cap
    d_rec = to_device(rec)
    d_pos = torch.zeros(max(n, 1), dtype=torch.int64, device="cuda")
    d_res = torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()
    assert cx.decode_device(d_rec.data_ptr(), rec.size, integrity, d_pos.data_ptr(), n, d_res.data_ptr(), s) == 0
    torch.cuda.synchronize()
    r = abi.DecodeResult.from_buffer_copy(to_host(d_res).tobytes())
    return r, to_host(d_pos[: min(r.frame_count, n)])


@pytest.mark.parametrize("shape", ["sealed_2000", "c3_120k", "small_frames_600k"])
@pytest.mark.parametrize("integrity", [abi.INTEGRITY_LAYOUT_ONLY, abi.INTEGRITY_VERIFY])
def test_general_walk_large_grids_device(cx, shape, integrity):
    """The general walk on device-resident records far above the 3-12-WG grids of
    test_configs_gpu: the sealed record of GPUTEST_r03's decrypt fault (4.3 MB, user
    headers, ~68 WGs), a C3-shaped 120,000-frame record (~255 MB, every WG of the chip)
    and 600,000 small frames (tiles of 16 frames). Positions and results exact."""
    if shape == "sealed_2000":
        from crypt_util import key_for, nonces_for, raw_record
        raw = raw_record(2000, 64, 4096, seed=11 * 2000 + 64, uh_max=20)
        rc, e, sealed = O.encrypt_batch(key_for(2003), raw, nonces_for(2000, 2004))
        assert rc == 0
        rec = np.frombuffer(sealed, dtype=np.uint8).copy()
        assert rec.size == 4_325_343
    elif shape == "c3_120k":
        rec = O.synth_batch(120_000, 64, 4096, 0, seed=0xC3)
    else:
        rec = O.synth_batch(600_000, 0, 90, 0, seed=0x600)
    r, pos = _device_decode(cx, rec, integrity)
    orc, oe, oh, of = O.decode_batch_slice_with(rec, integrity)
    assert (r.error.kind, r.frame_count) == (orc, len(of)), r.error.astuple()
    assert r.header.astuple() == oh.astuple()
    assert np.array_equal(pos, np.asarray(of, dtype=np.int64))
    # a frame length broken three quarters in: the walk stops or re-routes there
    bad = rec.copy()
    struct.pack_into("<I", bad, 256 + int(of[3 * len(of) // 4]) + 36, 5)
    r, pos = _device_decode(cx, bad, integrity)
    orc, oe, oh, of2 = O.decode_batch_slice_with(bad, integrity)
    assert r.error.astuple() == oe.astuple()
    if orc == 0:
        assert np.array_equal(pos, np.asarray(of2, dtype=np.int64))


@pytest.mark.parametrize("shift", [1, 3, 8, 13])
def test_unaligned_host_buffer(cx, shift):
    """The host-buffer entry point reading a caller buffer at an odd host address
    (the H2D copy's source alignment). Device-side misalignment of the record itself
    is covered by test_robust_gpu.py::test_misaligned_device_records."""
    rec = O.synth_batch(700, 1024, 1024)
    buf = np.zeros(rec.size + shift, dtype=np.uint8)
    buf[shift:] = rec
    view = buf[shift:]
    assert view.ctypes.data % 16 == shift % 16
    _check_decode(cx, view)


def test_corruption_sweep(cx):
    rng = np.random.default_rng(5)
    base = O.synth_batch(300, 1024, 1024)
    for trial in range(40):
        rec = base.copy()
        k = int(rng.integers(0, 3))
        for _ in range(k + 1):
            p = int(rng.integers(0, rec.size))
            rec[p] ^= np.uint8(1 << int(rng.integers(0, 8)))
        _check_decode(cx, rec)


def test_count_and_stride_breaks(cx):
    base = O.synth_batch(600, 1024, 1024)
    # message_count off by one (checksum also stale -> tile error first)
    r = base.copy(); struct.pack_into("<I", r, 48, 599); _check_decode(cx, r)
    # a frame's reserved field nonzero mid-batch -> walk stops there
    r = base.copy(); r[256 + 1072 * 333 + 44] = 1; _check_decode(cx, r)
    # a frame length changed mid-batch (stride break, walk continues elsewhere)
    r = base.copy(); struct.pack_into("<I", r, 256 + 1072 * 100 + 36, 1000); _check_decode(cx, r)
    # truncated record
    _check_decode(cx, base[:-5])
    # trailing bytes
    _check_decode(cx, np.concatenate([base, np.full(77, 9, dtype=np.uint8)]))


def _prepare_frame(batch, size=None, trailing=b""):
    body = bytes(batch) + trailing
    hdr = bytearray(256)
    struct.pack_into("<I", hdr, 48, 256 + len(body) if size is None else size)
    return np.frombuffer(bytes(hdr) + body, dtype=np.uint8).copy()


def test_decode_prepare_matches_oracle(cx):
    recs = [O.synth_batch(40, 10, 500, 0), O.synth_batch(3000, 1024, 1024, 0), O.synth_batch(500, 0, 5000, 3)]
    for rec in recs:
        fr = _prepare_frame(rec)
        cases = [fr, _prepare_frame(rec, size=0), _prepare_frame(rec, size=255),
                 _prepare_frame(rec, size=256 + rec.size + 1), _prepare_frame(rec, trailing=b"\x00" * 9)]
        for off in (256 + 40, 512 + 48, 512 + 44, 256 + 32, 256 + 60):
            b = fr.copy()
            b[off] ^= 0x5A
            cases.append(b)
        for c in cases:
            for validate in (True, False):
                rc, e, h = cx.decode_prepare(c, validate)
                orc, oe, oh = O.decode_prepare(c, validate)
                _same(rc, e, orc, oe)
                if rc == 0:
                    assert h.astuple() == oh.astuple()


def test_admit_batch_matches_oracle(cx):
    from iggy_amd.codec import raw_messages
    rng = np.random.default_rng(11)
    for n, lo, hi in ((7, 1, 300), (2000, 1024, 1024), (900, 0, 3000)):
        pls = rng.integers(lo, hi + 1, size=n).astype(np.uint32)
        ids = rng.integers(1, 2**63, size=2 * n, dtype=np.uint64)
        ots = (1_700_000_000_000_000 + np.arange(n)).astype(np.uint64)
        pay = rng.integers(0, 256, size=int(pls.sum()), dtype=np.uint8)
        rc, e, out = O.encode_batch(raw_messages(ids, ots, pay, pls), 0)
        wire = np.frombuffer(out, dtype=np.uint8).copy()
        bad = wire.copy()
        bad[256 + 48 + 3] ^= 0x10
        for batch, count in ((wire, n), (wire, n - 1), (bad, n), (np.concatenate([wire, np.zeros(3, np.uint8)]), n)):
            for mode in (abi.CHECKSUM_COMPUTE, abi.CHECKSUM_SKIP):
                got = cx.admit_batch(batch, count, 9, mode)
                exp = O.admit_batch(batch, count, 9, mode)
                _same(got[0], got[1], exp[0], exp[1])
                if got[0] == 0:
                    assert got[2].astuple() == exp[2].astuple()
                    assert got[3] == exp[3]


def test_recover_segment_matches_oracle(cx):
    recs, off = [], 500
    for k, (n, lo, hi) in enumerate([(40, 10, 900), (3000, 1024, 1024), (0, 0, 0), (700, 0, 5000), (1, 3, 3),
                                     (20000, 64, 64)]):
        if n == 0:  # a header-only batch with no messages (count 0) still chains
            r = np.zeros(256, dtype=np.uint8)
            struct.pack_into("<QQQQQ", r, 0, 1, off, 7, 0, 256)
            h = abi.BatchHeader()
            h.partition_id, h.base_offset, h.base_timestamp, h.batch_length = 1, off, 7, 256
            struct.pack_into("<Q", r, 40, O.calculate_batch_checksum(h, b""))
            recs.append(r)
            continue
        r = O.synth_batch(n, lo, hi, 0, seed=k)
        rc, e, h, r2 = O.stamp_batch(r, off, 2_000 + k)
        recs.append(np.frombuffer(r2, dtype=np.uint8))
        off += n
    seg = np.concatenate(recs)
    starts = np.cumsum([0] + [r.size for r in recs])
    cases = [(seg, 500), (seg, 501), (seg[:-1], 500), (seg[: starts[3] + 100], 500)]
    for k in range(len(recs)):
        b = seg.copy()
        b[starts[k] + 256 + (48 + 2 if recs[k].size > 256 else -216)] ^= 0x40
        cases.append((b, 500))
    for buf, so in cases:
        rc, out = cx.recover_segment(buf, so)
        orc, oout = O.recover_segment(buf, so)
        assert rc == orc == 0
        assert out.astuple() == oout.astuple()


def _crafted_record(n, lo, hi, fill, seed):
    """A stamped record whose payloads defeat the tile speculation: "zero" payloads
    (every offset inside them is a candidate frame start) or "fake" payloads that
    carry chains of well-formed fake frame headers every 100 B (confirmed false
    starts), so the link phase must repair groups exactly."""
    from iggy_amd.codec import raw_messages
    rng = np.random.default_rng(seed)
    pls = rng.integers(lo, hi + 1, size=n).astype(np.uint32)
    ids = rng.integers(0, 2**63, size=2 * n, dtype=np.uint64)
    ots = (1_700_000_000_000_000 + np.arange(n)).astype(np.uint64)
    if fill == "zero":
        pay = np.zeros(int(pls.sum()), dtype=np.uint8)
    else:
        pay = rng.integers(0, 256, size=int(pls.sum()), dtype=np.uint8)
        fake = np.zeros(48, dtype=np.uint8)
        struct.pack_into("<II", fake, 32, 0, 52)  # user headers 0, payload 52: a 100-B frame
        starts = np.concatenate([[0], np.cumsum(pls)[:-1]]).astype(np.int64)
        for st, ln in zip(starts, pls):
            for o in range(int(rng.integers(0, 100)), int(ln) - 48, 100):
                pay[st + o: st + o + 48] = fake
    raw = raw_messages(ids, ots, pay, pls)
    rc, e, out = O.encode_batch(raw, 1)
    assert rc == 0, e
    return np.frombuffer(out, dtype=np.uint8).copy()


@pytest.mark.parametrize("n,lo,hi,fill", [(3000, 64, 4096, "zero"), (20000, 0, 600, "zero"),
                                          (3000, 64, 4096, "fake"), (20000, 100, 700, "fake"),
                                          (60, 50000, 300000, "fake"), (40, 100000, 200000, "zero")])
def test_adversarial_variable_batches(cx, n, lo, hi, fill):
    rec = _crafted_record(n, lo, hi, fill, seed=n ^ lo)
    _check_decode(cx, rec)
    # and with a break in the middle: a frame's reserved bytes set
    rc, e, h, frames = O.decode_batch_slice_with(rec, 0)
    assert rc == 0, e
    r = rec.copy()
    r[256 + int(frames[len(frames) // 2]) + 41] = 7
    _check_decode(cx, r)


def _raw_from_arrays(n, pls, uhl, rng):
    ids = rng.integers(0, 2**63, size=2 * n, dtype=np.uint64)
    ots = (1_700_000_000_000_000 + rng.integers(0, 10**6, size=n)).astype(np.uint64)
    pay = rng.integers(0, 256, size=int(pls.sum()), dtype=np.uint8)
    uhb = rng.integers(0, 256, size=int(uhl.sum()), dtype=np.uint8) if uhl is not None else None
    return ids, ots, pay, uhb


@pytest.mark.parametrize("n,lo,hi,with_uh", [(1, 0, 0, False), (2, 5, 6, True), (100, 64, 4096, False),
                                             (3000, 64, 4096, True), (500, 0, 250, True),
                                             (2049, 1024, 1024, False), (40, 5000, 9000, False),
                                             # lane-group encode edges: tiny payloads (the s = 32 piece and the
                                             # clamped, realigned last piece), the 240-B short/long boundary,
                                             # a payload area under 16 B (fallback kernel)
                                             (300, 0, 20, False), (64, 0, 3, False), (5, 1, 2, False),
                                             (1000, 195, 206, False), (777, 1015, 1033, False),
                                             # unsegmented (< 2^18 messages) with a checksum chain of
                                             # 1 172 blocks: three chunks through k_bsum_chain's LDS stager
                                             (150_000, 0, 200, False)])
@pytest.mark.parametrize("partition_id", [0, 3])
def test_encode_matches_oracle(cx, n, lo, hi, with_uh, partition_id):
    from iggy_amd.codec import raw_messages
    rng = np.random.default_rng(n * 7 + lo)
    pls = rng.integers(lo, hi + 1, size=n).astype(np.uint32)
    uhl = rng.integers(0, 40, size=n).astype(np.uint32) if with_uh else None
    ids, ots, pay, uhb = _raw_from_arrays(n, pls, uhl, rng)
    raw = raw_messages(ids, ots, pay, pls, uhb, uhl)
    rc, e, out = cx.encode_batch(raw, partition_id)
    orc, oe, oout = O.encode_batch(raw, partition_id)
    _same(rc, e, orc, oe)
    assert out == oout
    # and it decodes
    rc, e, h, fr = cx.decode_batch_slice_with(np.frombuffer(out, dtype=np.uint8), 0)
    assert rc == 0, e


@pytest.mark.parametrize("n,lo,hi", [(300_000, 0, 64), (262_144, 100, 1100)])
def test_encode_segmented_matches_oracle(cx, n, lo, hi):
    """Batches of >= 2^18 messages encode in segments with the checksum chain of
    earlier segments on the side stream: byte-identical to the oracle."""
    from iggy_amd.codec import raw_messages
    rng = np.random.default_rng(n + lo)
    pls = rng.integers(lo, hi + 1, size=n).astype(np.uint32)
    ids, ots, pay, _ = _raw_from_arrays(n, pls, None, rng)
    raw = raw_messages(ids, ots, pay, pls)
    rc, e, out = cx.encode_batch(raw, 4)
    orc, oe, oout = O.encode_batch(raw, 4)
    _same(rc, e, orc, oe)
    assert out == oout


@pytest.mark.parametrize("pay_shift,out_shift", [(0, 0), (0, 5), (7, 7), (3, 12)])
def test_encode_segmented_device_alignments(cx, pay_shift, out_shift):
    """Segmented device encodes with payloads and output at every congruence: the writer-
    wave ring when P - out = 0 mod 16 (shifts (0, 0) and (7, 7)), the one-role ring
    otherwise: byte-identical to the oracle either way (encode.hip k_enc_ring)."""
    import torch
    from iggy_amd.codec import raw_messages
    n = 262_144
    rng = np.random.default_rng(n + pay_shift * 16 + out_shift)
    pls = rng.integers(100, 1101, size=n).astype(np.uint32)
    ids, ots, pay, _ = _raw_from_arrays(n, pls, None, rng)
    raw = raw_messages(ids, ots, pay, pls)
    orc, oe, oout = O.encode_batch(raw, 6)
    assert orc == 0
    d_ids = to_device(ids.view(np.int64))
    d_ots = to_device(ots.view(np.int64))
    d_pls = to_device(pls.view(np.int32))
    d_payb = torch.zeros(pay.size + 64, dtype=torch.uint8, device="cuda")
    d_payb[pay_shift: pay_shift + pay.size] = to_device(pay)
    need = len(oout)
    d_outb = torch.full((need + 64,), 0xCD, dtype=torch.uint8, device="cuda")
    d_res = torch.zeros(ctypes.sizeof(abi.EncodeResult), dtype=torch.uint8, device="cuda")
    draw = abi.RawMessages(n, d_ids.data_ptr(), d_ots.data_ptr(), d_payb.data_ptr() + pay_shift, d_pls.data_ptr(),
                           None, None)
    s = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()
    assert cx.encode_device(draw, 6, d_outb.data_ptr() + out_shift, need, d_res.data_ptr(), s) == 0
    torch.cuda.synchronize()
    er = abi.EncodeResult.from_buffer_copy(to_host(d_res).tobytes())
    assert er.error.kind == 0 and er.batch_length == need
    got = to_host(d_outb)
    assert got[out_shift: out_shift + need].tobytes() == oout
    assert (got[:out_shift] == 0xCD).all() and (got[out_shift + need:] == 0xCD).all()


def test_encode_errors(cx):
    from iggy_amd.codec import raw_messages
    rng = np.random.default_rng(1)
    n = 5
    pls = np.full(n, 10, dtype=np.uint32)
    ids, ots, pay, _ = _raw_from_arrays(n, pls, None, rng)
    ots[:] = 1000
    ots[3] = 1000 + 2**32  # delta > u32::MAX (send_messages.rs:132-135)
    raw = raw_messages(ids, ots, pay, pls)
    rc, e, _ = cx.encode_batch(raw)
    orc, oe, _ = O.encode_batch(raw)
    _same(rc, e, orc, oe)
    assert rc == abi.ERR_INVALID_TIMESTAMP_DELTA and e.a == 2**32
    empty = raw_messages(ids[:0], ots[:0], pay[:0], pls[:0])
    rc, e, _ = cx.encode_batch(empty)
    assert rc == abi.ERR_VALIDATION and e.reason == abi.V_EMPTY_BATCH


def test_stamp_and_calculate(cx):
    rec = O.synth_batch(777, 64, 2000, 3)
    rc, e, h, out = cx.stamp_batch(rec, 1234, 5678)
    orc, oe, oh, oout = O.stamp_batch(rec.copy(), 1234, 5678)
    assert rc == orc == 0
    assert out == oout
    # calculate over a blob with a broken tail: infallible walk semantics
    blob = rec[256:].copy()
    blob[-3] = 0xFF
    struct.pack_into("<I", blob, len(blob) - 500, 0xFFFF)
    hh = abi.BatchHeader()
    O.lib().oracle_batch_header_decode(rec.ctypes.data, rec.size, ctypes.byref(hh), None)
    assert cx.calculate_batch_checksum(hh, blob) == O.calculate_batch_checksum(hh, blob)


@pytest.mark.parametrize("mode", [0, 1])
def test_poll_multi_record(cx, mode):
    recs = [O.synth_batch(n, lo, hi, uh, seed=n) for n, lo, hi, uh in
            [(10, 100, 100, 0), (300, 1, 900, 5), (1, 0, 0, 0), (2000, 1024, 1024, 0)]]
    body = np.concatenate(recs)
    rc, e, msgs = cx.poll_decode(body, mode)
    orc, oe, om = O.poll_decode(body, mode)
    _same(rc, e, orc, oe)
    assert [m.astuple() for m in msgs] == [m.astuple() for m in om]
    # corrupt the third record's frame: SDK maps to InvalidMessagePayloadLength,
    # the iterator yields what came before, then the error
    bad = body.copy()
    off = recs[0].size + recs[1].size + 256 + 40
    bad[off] = 1
    rc, e, msgs = cx.poll_decode(bad, mode)
    orc, oe, om = O.poll_decode(bad, mode)
    _same(rc, e, orc, oe)
    assert len(msgs) == len(om)


# ---- full-size parity (BASELINE config C2 and a 256K-message record): many more
# chunks than producer waves, every LDS ring slot of the chain reused, and the
# per-call epoch tags exercised by repeated calls on one context
@pytest.fixture(scope="module")
def big_record():
    return O.synth_batch(1 << 18, 1024, 1024, 0, seed=0x5EED)


def test_c2_full_size_decode(cx):
    rec = O.synth_batch(1 << 20, 1024, 1024, 0, seed=0x16619E3779B97F4A)
    assert rec.size == 1_124_073_728
    orc, oe, oh, of = O.decode_batch_slice_with(rec, 0)
    assert orc == 0
    for _ in range(2):
        rc, e, h, frames = cx.decode_batch_slice_with(rec, 0)
        assert rc == 0, e
        assert h.astuple() == oh.astuple()
        assert np.array_equal(frames, of)


def test_large_uniform_repeated(cx, big_record):
    orc, oe, oh, of = O.decode_batch_slice_with(big_record, 0)
    for integrity in (0, 1, 0, 0):
        rc, e, h, frames = cx.decode_batch_slice_with(big_record, integrity)
        assert rc == orc == 0, e
        assert h.astuple() == oh.astuple()
        assert np.array_equal(frames, of)


@pytest.mark.parametrize("where", ["payload_late", "payload_first", "stored_cs_mid", "batch_cs",
                                   "reserved_late", "count", "last_frame_byte", "two_errors"])
def test_large_uniform_corruption(cx, big_record, where):
    rec = big_record.copy()
    S = 1072
    if where == "payload_late":
        rec[256 + S * 250_000 + 500] ^= 0x40
    elif where == "payload_first":
        rec[256 + 100] ^= 1
    elif where == "stored_cs_mid":
        rec[256 + S * 131_071 + 3] ^= 0x10
    elif where == "batch_cs":
        rec[56] ^= 0x80
    elif where == "reserved_late":
        rec[256 + S * 200_000 + 45] = 7
    elif where == "count":
        struct.pack_into("<I", rec, 48, (1 << 18) - 1)
    elif where == "last_frame_byte":
        rec[-1] ^= 0xFF
    elif where == "two_errors":
        rec[256 + S * 180_000 + 300] ^= 2
        rec[256 + S * 70_000 + 900] ^= 4
    for integrity in (0, 1):
        _check_decode_integrity(cx, rec, integrity)


def _check_decode_integrity(cx, rec, integrity):
    rc, e, h, frames = cx.decode_batch_slice_with(rec, integrity)
    orc, oe, oh, of = O.decode_batch_slice_with(rec, integrity)
    _same(rc, e, orc, oe)
    if rc == 0:
        assert h.astuple() == oh.astuple()
        assert np.array_equal(frames, of)


# ---- poll-path slicing and device stamp
def _stamped_rec(n, lo, hi, base_offset, base_ts, seed):
    rec = O.synth_batch(n, lo, hi, 0, seed=seed)
    rc, e, h, out = O.stamp_batch(rec.copy(), base_offset, base_ts)
    assert rc == 0
    return np.frombuffer(out, dtype=np.uint8).copy()


_SLICE_QUERIES = [
    (abi.LOOKUP_OFFSET, 0, 10**9, 2**64 - 1), (abi.LOOKUP_OFFSET, 7000, 25, 2**64 - 1),
    (abi.LOOKUP_OFFSET, 7000, 10**6, 2**64 - 1), (abi.LOOKUP_OFFSET, 9000, 5000, 12000),
    (abi.LOOKUP_OFFSET, 5000, 1, 2**64 - 1), (abi.LOOKUP_OFFSET, 10**9, 5, 2**64 - 1),
    (abi.LOOKUP_OFFSET, 6000, 3000, 5500), (abi.LOOKUP_OFFSET, 6024, 1024, 2**64 - 1),
    (abi.LOOKUP_TIMESTAMP, 4242, 10, 2**64 - 1), (abi.LOOKUP_TIMESTAMP, 4243, 10, 2**64 - 1),
    (abi.LOOKUP_TIMESTAMP, 0, 10**9, 6100),
]


@pytest.mark.parametrize("shape", [(3000, 1024, 1024), (2500, 10, 900), (40, 300, 300)])
@pytest.mark.parametrize("q", _SLICE_QUERIES)
def test_select_slice_matches_oracle(cx, shape, q):
    n, lo, hi = shape
    rec = _stamped_rec(n, lo, hi, 5000, 4242, seed=n)
    kind, value, count, ceiling = q
    for already in (0, 3):
        rc, e, r, hdr = cx.select_slice(rec, kind, value, count, ceiling, already)
        orc, orr, ohdr = O.select_slice(rec, kind, value, count, ceiling, already)
        assert rc == orc == 0, e
        assert r.astuple() == orr.astuple()
        assert hdr == ohdr


def test_select_slice_non_monotone_and_errors(cx):
    rec = _stamped_rec(5000, 100, 100, 0, 1, seed=9)
    S = 148
    rng = np.random.default_rng(4)
    for i in range(5000):  # scrambled offset deltas: unselected frames inside selections
        struct.pack_into("<I", rec, 256 + i * S + 24, int(rng.integers(0, 6000)))
    for value, count, ceiling in [(3000, 7, 2**64 - 1), (100, 2000, 5000), (5990, 4, 2**64 - 1), (0, 1, 10)]:
        rc, e, r, hdr = cx.select_slice(rec, abi.LOOKUP_OFFSET, value, count, ceiling)
        orc, orr, ohdr = O.select_slice(rec, abi.LOOKUP_OFFSET, value, count, ceiling)
        assert rc == orc == 0 and r.astuple() == orr.astuple() and hdr == ohdr
    bad = rec.copy()
    bad[256 + 40] = 1  # frame 0 reserved: the batch does not decode -> its error, nothing selected
    rc, e, r, hdr = cx.select_slice(bad, abi.LOOKUP_OFFSET, 0, 10)
    orc, oe, _, _ = O.decode_batch_slice_with(bad, abi.INTEGRITY_LAYOUT_ONLY)
    assert rc == orc != 0 and e.astuple() == oe.astuple()


def test_device_select_and_stamp(cx):
    import torch
    rec = _stamped_rec(20000, 64, 2000, 100, 200, seed=11)
    n = 20000
    d_rec = to_device(rec, "cuda:0")
    d_pos = torch.zeros(n, dtype=torch.int64, device="cuda:0")
    d_res = torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device="cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    assert cx.decode_device(d_rec.data_ptr(), rec.size, 0, d_pos.data_ptr(), n, d_res.data_ptr(), s) == 0
    d_sr = torch.zeros(ctypes.sizeof(abi.SliceResult), dtype=torch.uint8, device="cuda:0")
    d_hdr = torch.zeros(256, dtype=torch.uint8, device="cuda:0")
    q = abi.SliceQuery(abi.LOOKUP_OFFSET, 777, 5100, 2**64 - 1, 0, 0)
    assert cx.select_slice_device(d_rec.data_ptr(), d_pos.data_ptr(), n, q, d_sr.data_ptr(), d_hdr.data_ptr(), s) == 0
    # stamp the same record in place (new base values), then re-verify it
    d_h = torch.zeros(64, dtype=torch.uint8, device="cuda:0")
    assert cx.stamp_device(d_rec.data_ptr(), d_pos.data_ptr(), n, 424242, 999, d_h.data_ptr(), s) == 0
    torch.cuda.synchronize()
    sr = abi.SliceResult.from_buffer_copy(to_host(d_sr).tobytes())
    orc, orr, ohdr = O.select_slice(rec, abi.LOOKUP_OFFSET, 5100, 777)
    assert sr.astuple() == orr.astuple() and to_host(d_hdr).tobytes() == ohdr
    stamped = to_host(d_rec)
    orc, oe, oh, oout = O.stamp_batch(rec.copy(), 424242, 999)
    assert stamped.tobytes() == oout
    h = abi.BatchHeader.from_buffer_copy(to_host(d_h).tobytes())
    assert h.astuple() == oh.astuple()
    rc, e, hh, _ = cx.decode_batch_slice_with(stamped, abi.INTEGRITY_VERIFY)
    assert rc == 0, e


# ---- BASELINE config C3 at full size: 1,048,576 messages, payloads U[64, 4096] B
# (~2.23 GB batch). The encode takes the segmented path (4 frame segments, the
# batch-checksum chain of earlier segments on the side stream) and the decode the
# general walk (variable frame sizes), at the sizes the bench times.
@pytest.fixture(scope="module")
def c3_raw():
    from iggy_amd.codec import raw_messages
    n = 1 << 20
    rng = np.random.default_rng(0x16619E3779B97F4A)
    pls = (64 + rng.integers(0, 4033, size=n)).astype(np.uint32)
    ids = rng.integers(1, 2**63, size=2 * n, dtype=np.uint64)
    ots = (1_700_000_000_000_000 + np.arange(n)).astype(np.uint64)
    pay = rng.integers(0, 256, size=int(pls.sum()), dtype=np.uint8)
    keep = (ids, ots, pay, pls)
    return raw_messages(ids, ots, pay, pls), keep


def test_c3_full_size_encode_decode(cx, c3_raw):
    raw, _keep = c3_raw
    rc, e, out = cx.encode_batch(raw, 1)
    orc, oe, oout = O.encode_batch(raw, 1)
    assert rc == orc == 0, e
    assert len(out) == len(oout) > 2_000_000_000
    assert out == oout
    del oout
    rec = np.frombuffer(out, dtype=np.uint8)
    for integ in (abi.INTEGRITY_VERIFY, abi.INTEGRITY_LAYOUT_ONLY):
        rc, e, h, frames = cx.decode_batch_slice_with(rec, integ)
        orc, oe, oh, of = O.decode_batch_slice_with(rec, integ)
        _same(rc, e, orc, oe)
        assert rc == 0 and h.astuple() == oh.astuple()
        assert np.array_equal(frames, of)
    # a body byte near the end and a frame length mid-batch
    bad = rec.copy()
    bad[-100] ^= 0x10
    _check_decode_integrity(cx, bad, abi.INTEGRITY_VERIFY)
    bad = rec.copy()
    _, _, _, of = O.decode_batch_slice_with(rec, abi.INTEGRITY_LAYOUT_ONLY)
    struct.pack_into("<I", bad, 256 + int(of[600_000]) + 36, 77)
    for integ in (abi.INTEGRITY_VERIFY, abi.INTEGRITY_LAYOUT_ONLY):
        _check_decode_integrity(cx, bad, integ)


# ---- walk_disk_chunk: core/partitions/src/poll_plan.rs:950-1011
def _segment_chunk(shapes, base_offset=1000, seed=3):
    """Consecutive stamped batches (offsets continue across batches), as a segment
    chunk reads them from disk; -> (chunk, batch starts)."""
    recs, off = [], base_offset
    for k, (n, lo, hi) in enumerate(shapes):
        r = O.synth_batch(n, lo, hi, 0, seed=seed * 100 + k)
        rc, e, h, out = O.stamp_batch(r, off, 5000 + 10 * k)
        recs.append(np.frombuffer(out, dtype=np.uint8).copy())
        off += n
    starts = np.cumsum([0] + [r.size for r in recs])
    return np.concatenate(recs), starts


_CHUNK_SHAPES = [(40, 10, 900), (3000, 1024, 1024), (1, 5, 5), (700, 0, 3000), (25, 64, 64), (5000, 100, 100)]


def _walk_same(cx, chunk, *args, **kw):
    rc, w, fr, hd = cx.walk_disk_chunk(chunk, *args, **kw)
    orc, ow, ofr, ohd = O.walk_disk_chunk(chunk, *args, **kw)
    assert rc == orc, (w.astuple(), ow.astuple())
    assert w.astuple() == ow.astuple()
    assert [f.astuple() for f in fr] == [f.astuple() for f in ofr]
    assert hd == ohd
    return w


@pytest.mark.parametrize("q", [(abi.LOOKUP_OFFSET, 0, 10**9, 2**64 - 1), (abi.LOOKUP_OFFSET, 1020, 30, 2**64 - 1),
                               (abi.LOOKUP_OFFSET, 1030, 5000, 2**64 - 1), (abi.LOOKUP_OFFSET, 2000, 10**6, 4200),
                               (abi.LOOKUP_OFFSET, 4040, 1, 2**64 - 1), (abi.LOOKUP_OFFSET, 10**9, 5, 2**64 - 1),
                               (abi.LOOKUP_TIMESTAMP, 5015, 100, 2**64 - 1), (abi.LOOKUP_TIMESTAMP, 0, 3500, 2**64 - 1)])
@pytest.mark.parametrize("integrity", [0, 1])
def test_walk_disk_chunk_clean(cx, q, integrity):
    chunk, starts = _segment_chunk(_CHUNK_SHAPES)
    kind, value, count, ceiling = q
    for already in (0, 7):
        _walk_same(cx, chunk, kind, value, count, ceiling, already, integrity)


def test_walk_disk_chunk_tails_and_corruption(cx):
    chunk, starts = _segment_chunk(_CHUNK_SHAPES)
    q = (abi.LOOKUP_OFFSET, 1000, 10**9)
    cases = []
    cases.append(chunk[: starts[3] + 1000])          # torn tail inside batch 3
    cases.append(chunk[: starts[4] + 100])           # torn inside a header
    cases.append(chunk[: starts[2] + 255])           # less than a header left
    b = chunk.copy(); b[starts[2] + 40] ^= 1; cases.append(b)          # batch checksum: corrupt at rest (Verify)
    b = chunk.copy(); b[starts[1] + 256 + 1072 * 7 + 500] ^= 4; cases.append(b)  # body byte: message checksum
    b = chunk.copy(); b[starts[3] + 100] = 9; cases.append(b)           # reserved header byte: tail
    b = chunk.copy(); b[starts[4] + 256 + 40] = 1; cases.append(b)      # frame reserved: layout break
    cases.append(np.concatenate([chunk, np.zeros(300, dtype=np.uint8)]))  # zero padding after the last batch
    for c in cases:
        for integrity in (0, 1):
            w = _walk_same(cx, c, *q, integrity=integrity)
    # the batch-checksum case is corrupt under Verify only, and consumed stops at that batch
    b = chunk.copy(); b[starts[2] + 40] ^= 1
    w = _walk_same(cx, b, *q, integrity=0)
    assert w.corrupt == 1 and w.consumed == starts[2] and w.error.kind == abi.ERR_INVALID_BATCH_CHECKSUM
    w = _walk_same(cx, b, *q, integrity=1)
    assert w.corrupt == 0 and w.consumed == len(b)
    # a message-checksum failure is an incomplete tail, not corruption (poll_plan.rs:984-987)
    b = chunk.copy(); b[starts[1] + 256 + 1072 * 7 + 500] ^= 4
    w = _walk_same(cx, b, *q, integrity=0)
    assert w.corrupt == 0 and w.consumed == starts[1] and w.error.kind == abi.ERR_INVALID_MESSAGE_CHECKSUM


def test_walk_disk_chunk_capacity_and_matched(cx):
    chunk, starts = _segment_chunk(_CHUNK_SHAPES)
    rc, w, fr, hd = cx.walk_disk_chunk(chunk, abi.LOOKUP_OFFSET, 0, 10**9, cap=2)
    orc, ow, ofr, ohd = O.walk_disk_chunk(chunk, abi.LOOKUP_OFFSET, 0, 10**9, cap=2)
    assert rc == orc == abi.ERR_CAPACITY and w.astuple() == ow.astuple() and len(fr) == 2
    # already matched everything: nothing decoded, nothing consumed
    w = _walk_same(cx, chunk, abi.LOOKUP_OFFSET, 0, 50, 2**64 - 1, 50)
    assert w.consumed == 0 and w.batches == 0 and w.fragments == 0


# ---- state-transfer segment verify + segment writer:
# core/partitions/src/state_transfer.rs:715-833, messages_writer.rs:100-118
def _empty_batch(base_offset, ts):
    r = np.zeros(256, dtype=np.uint8)
    struct.pack_into("<QQQQQ", r, 0, 1, base_offset, ts, 0, 256)
    h = abi.BatchHeader()
    h.partition_id, h.base_offset, h.base_timestamp, h.batch_length = 1, base_offset, ts, 256
    struct.pack_into("<Q", r, 40, O.calculate_batch_checksum(h, b""))
    return r


def test_walk_segment_payload_matches_oracle(cx):
    seg, starts = _segment_chunk([(3000, 1024, 1024), (40, 10, 900), (700, 0, 3000), (1, 5, 5), (20000, 64, 64),
                                  (300, 100, 5000)], base_offset=7000, seed=5)
    cases = [(seg, 7000), (seg, 7001), (seg[:0], 7000), (seg[: starts[3] + 77], 7000), (seg[: starts[4]], 7000)]
    for k in range(len(starts) - 1):
        b = seg.copy(); b[starts[k] + 256 + 48 + 3] ^= 0x20; cases.append((b, 7000))   # message checksum
        b = seg.copy(); b[starts[k] + 41] ^= 2; cases.append((b, 7000))                 # batch checksum
    # a gap in the offsets, an empty batch, an offset overflow
    gap = np.concatenate([seg[: starts[2]], _segment_chunk([(50, 10, 10)], base_offset=9999)[0]])
    cases.append((gap, 7000))
    cases.append((np.concatenate([seg[: starts[1]], _empty_batch(10000, 3)]), 7000))
    big = _segment_chunk([(10, 10, 10)], base_offset=2**64 - 5)[0]
    cases.append((big, 2**64 - 5))
    for payload, base in cases:
        rc, w, idx = cx.walk_segment_payload(payload, base)
        orc, ow, oidx = O.walk_segment_payload(payload, base)
        assert rc == orc, (w.astuple(), ow.astuple())
        assert w.astuple() == ow.astuple()
        assert idx == oidx
    rc, w, idx = cx.walk_segment_payload(seg, 7000)
    assert w.error == abi.SEG_OK and w.index_entries >= 2


def test_segment_write_device_then_verify(cx, tmp_path):
    """Device-resident stamped batches appended to a segment file through the pinned
    staging (several 8 MiB pieces), read back byte-exact, then verified by the
    state-transfer walk and the boot-recovery walk."""
    import os
    import torch
    seg, starts = _segment_chunk([(20000, 1024, 1024), (3000, 10, 3000), (5000, 100, 100)], base_offset=0, seed=9)
    d = to_device(seg, "cuda:0")
    torch.cuda.synchronize()
    path = str(tmp_path / "00000000000000000000.log")
    fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o644)
    try:
        head = 4096
        os.pwrite(fd, b"\x00" * head, 0)  # the writer appends at its cursor: here past 4 KiB of prior data
        n = cx.segment_write_device(fd, head, d.data_ptr(), seg.size, fsync=True)
        assert n == seg.size
        got = np.fromfile(path, dtype=np.uint8)[head:]
    finally:
        os.close(fd)
    assert np.array_equal(got, seg)
    rc, w, idx = cx.walk_segment_payload(got, 0)
    assert rc == 0 and w.error == abi.SEG_OK and w.end_offset == 27999
    rc, rec = cx.recover_segment(got, 0)
    assert rc == 0 and rec.batches == 3 and rec.walked_bytes == seg.size

"""GPU tests of the boundary's robustness and of the entry points the parity suite
does not reach: the asynchronous submit/poll host API, the device entry points
(encode, batch checksum, XXH3 ranges, verify-and-recompute) against the oracle,
misaligned device records, one context on two streams, two contexts decoding
variable-size records concurrently, device-encode capacity, and recovery after a
timed-out decode (diagnostic build). Integer byte work: every check is bit-exact."""
import ctypes
import struct
import threading

import numpy as np
import pytest

from golden_util import reference_vectors
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


def _torch():
    import os
    if os.environ.get("IGGY_TEST_DIAG"):  # diagnostics: the HIP state torch will initialise on top of
        hip = ctypes.CDLL("libamdhip64.so")
        n = ctypes.c_int(-1)
        rc = hip.hipGetDeviceCount(ctypes.byref(n))
        print(f"\n[diag] peek={hip.hipPeekAtLastError()} getDeviceCount rc={rc} n={n.value} "
              f"HIP_VISIBLE_DEVICES={os.environ.get('HIP_VISIBLE_DEVICES')} "
              f"ROCR_VISIBLE_DEVICES={os.environ.get('ROCR_VISIBLE_DEVICES')} "
              f"CUDA_VISIBLE_DEVICES={os.environ.get('CUDA_VISIBLE_DEVICES')}", flush=True)
    import torch
    return torch


def _res(t):
    return abi.DecodeResult.from_buffer_copy(to_host(t).tobytes())


def _same(a_rc, a_e, b_rc, b_e):
    assert a_rc == b_rc, (a_e, b_e)
    assert a_e.astuple() == b_e.astuple()


def _raw(n, lo, hi, seed, uh=False):
    from iggy_amd.codec import raw_messages
    rng = np.random.default_rng(seed)
    pls = rng.integers(lo, hi + 1, size=n).astype(np.uint32)
    ids = rng.integers(0, 2**63, size=2 * n, dtype=np.uint64)
    ots = (1_700_000_000_000_000 + rng.integers(0, 10**6, size=n)).astype(np.uint64)
    pay = rng.integers(0, 256, size=int(pls.sum()), dtype=np.uint8)
    uhl = rng.integers(0, 40, size=n).astype(np.uint32) if uh else None
    uhb = rng.integers(0, 256, size=int(uhl.sum()), dtype=np.uint8) if uh else None
    keep = (ids, ots, pay, pls, uhb, uhl)
    return raw_messages(ids, ots, pay, pls, uhb, uhl), keep


# ------------------------------------------------------------ submit / poll
def test_submit_poll_decode_matches_oracle(cx):
    recs = [O.synth_batch(3000, 1024, 1024, seed=1), O.synth_batch(900, 0, 5000, 3, seed=2),
            O.synth_batch(1, 5, 5, seed=3)]
    bad = recs[0].copy()
    bad[256 + 1072 * 1234 + 600] ^= 4
    recs.append(bad)
    tickets = []
    for rec in recs:  # all in flight together
        for integ in (abi.INTEGRITY_VERIFY, abi.INTEGRITY_LAYOUT_ONLY):
            if len(tickets) == 8:
                break
            pos = np.zeros(rec.size // 48 + 1, dtype=np.uint64)
            tickets.append((cx.decode_submit(rec, integ, pos), rec, integ, pos))
    for t, rec, integ, pos in tickets:
        c = None
        while c is None:
            c = cx.poll(t)
        orc, oe, oh, of = O.decode_batch_slice_with(rec, integ)
        assert c.op == abi.OP_DECODE
        assert c.error.kind == orc and c.error.astuple() == oe.astuple()
        if orc == 0:
            assert c.header.astuple() == oh.astuple() and c.frame_count == len(of)
            assert np.array_equal(pos[: len(of)], of)
    # a retired ticket is not valid any more
    with pytest.raises(Exception):
        cx.poll(tickets[0][0])


def test_submit_registered_buffers_and_busy(cx):
    from iggy_amd.codec import host_buffer, page_aligned
    rec = O.synth_batch(20000, 100, 2000, seed=9)
    buf = page_aligned(rec)
    pos = host_buffer(20000, np.uint64)
    cx.host_register(buf)
    cx.host_register(pos)
    try:
        ts = [cx.decode_submit(buf, abi.INTEGRITY_VERIFY, pos if k == 0 else None) for k in range(8)]
        from iggy_amd.codec import CodecError
        with pytest.raises(CodecError) as ei:
            cx.decode_submit(buf, abi.INTEGRITY_VERIFY)
        assert ei.value.rc == abi.ERR_BUSY
        orc, oe, oh, of = O.decode_batch_slice_with(rec, 0)
        for t in ts:
            c = cx.wait(t)
            assert c.error.kind == 0 and c.header.astuple() == oh.astuple()
        assert np.array_equal(pos, of)
    finally:
        cx.host_unregister(buf)
        cx.host_unregister(pos)
    # frame capacity too small for the record
    short = np.zeros(10, dtype=np.uint64)  # kept alive until the ticket completes (the API's contract)
    t = cx.decode_submit(rec, abi.INTEGRITY_VERIFY, short)
    assert cx.wait(t).error.kind == abi.ERR_CAPACITY


@pytest.mark.parametrize("n,lo,hi,uh", [(3000, 64, 4096, False), (500, 0, 250, True), (262_144, 100, 1100, False)])
def test_submit_encode_matches_oracle(cx, n, lo, hi, uh):
    raw, keep = _raw(n, lo, hi, seed=n + lo, uh=uh)
    need = O.lib().oracle_encoded_batch_size(ctypes.byref(raw))
    out = np.zeros(need, dtype=np.uint8)
    t = cx.encode_submit(raw, 5, out)
    c = cx.wait(t)
    orc, oe, oout = O.encode_batch(raw, 5)
    assert c.op == abi.OP_ENCODE and c.error.kind == orc == 0, c.error
    assert c.bytes == need and out.tobytes() == oout
    # too small: nothing written, capacity error from the device
    small = np.full(need - 1, 0xAB, dtype=np.uint8)
    c = cx.wait(cx.encode_submit(raw, 5, small))
    assert c.error.kind == abi.ERR_CAPACITY and c.error.a == need
    assert (small == 0xAB).all()


# ---------------------------------------------------------- device entry points
def test_encode_device_matches_oracle_and_capacity(cx):
    torch = _torch()
    for n, lo, hi, uh in [(5000, 64, 4096, False), (700, 0, 300, True), (2049, 1024, 1024, False)]:
        raw, keep = _raw(n, lo, hi, seed=7 * n, uh=uh)
        ids, ots, pay, pls, uhb, uhl = keep
        d = lambda a: to_device(a.view(np.uint8), "cuda:0") if a is not None and a.size else None
        dids, dots, dpay, dpls, duhb, duhl = (d(a) for a in keep)
        draw = abi.RawMessages(n, dids.data_ptr(), dots.data_ptr(), dpay.data_ptr() if dpay is not None else None,
                               dpls.data_ptr(), duhb.data_ptr() if duhb is not None else None,
                               duhl.data_ptr() if duhl is not None else None)
        orc, oe, oout = O.encode_batch(raw, 0)
        need = len(oout)
        out = torch.full((need + 64,), 0xCD, dtype=torch.uint8, device="cuda:0")
        res = torch.zeros(ctypes.sizeof(abi.EncodeResult), dtype=torch.uint8, device="cuda:0")
        s = torch.cuda.current_stream().cuda_stream
        assert cx.encode_device(draw, 0, out.data_ptr(), need, res.data_ptr(), s) == 0
        torch.cuda.synchronize()
        er = abi.EncodeResult.from_buffer_copy(to_host(res).tobytes())
        assert er.error.kind == 0 and er.batch_length == need
        got = to_host(out)
        assert got[:need].tobytes() == oout and (got[need:] == 0xCD).all()
        # capacity one byte short: the device reports it and writes nothing
        out.fill_(0xCD)
        assert cx.encode_device(draw, 0, out.data_ptr(), need - 1, res.data_ptr(), s) == 0
        torch.cuda.synchronize()
        er = abi.EncodeResult.from_buffer_copy(to_host(res).tobytes())
        assert er.error.kind == abi.ERR_CAPACITY and er.error.a == need and er.error.b == need - 1
        assert (to_host(out) == 0xCD).all()


def test_golden_produce_vector_encoded_on_gpu(cx):
    """The Rust-generated produce batch (message-batch.test.ts:47-60), byte for byte."""
    ref = reference_vectors()
    msgs = ref["messages"]
    ids = np.array([[m["id"], 0] for m in msgs], dtype=np.uint64).reshape(-1)
    ots = np.array([m["origin_timestamp"] for m in msgs], dtype=np.uint64)
    pay = np.frombuffer(b"".join(m["payload"].encode() for m in msgs), dtype=np.uint8).copy()
    pls = np.array([len(m["payload"]) for m in msgs], dtype=np.uint32)
    uhs = np.frombuffer(b"".join(m["user_headers"].encode() for m in msgs), dtype=np.uint8).copy()
    uhl = np.array([len(m["user_headers"]) for m in msgs], dtype=np.uint32)
    raw = abi.RawMessages(2, ids.ctypes.data, ots.ctypes.data, pay.ctypes.data, pls.ctypes.data,
                          uhs.ctypes.data if uhs.size else None, uhl.ctypes.data)
    rc, e, out = cx.encode_batch(raw)
    assert rc == 0, e
    assert out.hex() == ref["produce_batch_hex"]
    # and through the asynchronous host API
    buf = np.zeros(len(out), dtype=np.uint8)
    c = cx.wait(cx.encode_submit(raw, 0, buf))
    assert c.error.kind == 0 and buf.tobytes().hex() == ref["produce_batch_hex"]


def test_verify_and_recompute_matches_oracle(cx):
    for rec in (O.synth_batch(3000, 1024, 1024, seed=4), O.synth_batch(777, 0, 3000, 2, seed=5),
                O.synth_batch(3, 10, 10, seed=6)):
        h = abi.BatchHeader()
        O.lib().oracle_batch_header_decode(rec.ctypes.data, rec.size, ctypes.byref(h), None)
        blob = rec[256:].copy()
        cases = [blob]
        b = blob.copy(); b[len(b) // 2] ^= 1; cases.append(b)           # body byte
        b = blob.copy(); b[40] = 3; cases.append(b)                      # frame 0 reserved
        cases.append(blob[:-1].copy())                                   # torn tail
        for bl in cases:
            rc, e, v = cx.verify_and_recompute_batch_checksum(h, bl)
            oe = abi.WireError()
            ov = ctypes.c_uint64(0)
            orc = O.lib().oracle_verify_and_recompute(ctypes.byref(h), bl.ctypes.data, bl.size, ctypes.byref(ov),
                                                      None, 0, None, ctypes.byref(oe))
            _same(rc, e, orc, oe)
            if rc == 0:
                assert v == ov.value


def test_batch_checksum_and_xxh3_ranges_device(cx):
    torch = _torch()
    rec = O.synth_batch(50_000, 10, 900, 4, seed=12)
    rc, e, h, frames = O.decode_batch_slice_with(rec, 1)
    assert rc == 0
    d_rec = to_device(rec, "cuda:0")
    d_pos = to_device(frames.view(np.int64), "cuda:0")
    d_out = torch.zeros(4, dtype=torch.int64, device="cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    h2 = abi.BatchHeader.from_buffer_copy(bytes(h))
    h2.base_offset, h2.base_timestamp = 77, 88
    for n in (len(frames), 1, 7, 25, 1000):
        assert cx._L.iggy_codec_batch_checksum_device(cx.handle, ctypes.byref(h2), d_rec.data_ptr() + 256,
                                                      d_pos.data_ptr(), n, d_out.data_ptr(), s) == 0
        torch.cuda.synchronize()
        blob = rec[256: 256 + (int(frames[n]) if n < len(frames) else rec.size - 256)]
        assert int(d_out[0].item()) & (2**64 - 1) == O.calculate_batch_checksum(h2, blob)
    # XXH3 of every frame's hashed range (frame[8..end]) equals its stored checksum
    lens = np.array([struct.unpack_from("<I", rec, 256 + int(p) + 36)[0] +
                     struct.unpack_from("<I", rec, 256 + int(p) + 32)[0] + 40 for p in frames], dtype=np.uint32)
    offs = (frames + 256 + 8).astype(np.uint64)
    d_offs = to_device(offs.view(np.int64), "cuda:0")
    d_lens = to_device(lens.view(np.int32), "cuda:0")
    d_h = torch.zeros(len(frames), dtype=torch.int64, device="cuda:0")
    assert cx.xxh3_ranges_device(d_rec.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), len(frames),
                                 d_h.data_ptr(), s) == 0
    torch.cuda.synchronize()
    got = to_host(d_h).view(np.uint64)
    stored = np.array([struct.unpack_from("<Q", rec, 256 + int(p))[0] for p in frames], dtype=np.uint64)
    assert np.array_equal(got, stored)


@pytest.mark.parametrize("shift", [1, 3, 8, 13])
@pytest.mark.parametrize("shape", [(700, 1024, 1024), (900, 64, 4096)])
def test_misaligned_device_records(cx, shift, shape):
    """Records at byte offsets 1/3/8/13 of a device allocation (frames at every
    alignment), through the device entry point."""
    torch = _torch()
    n, lo, hi = shape
    rec = O.synth_batch(n, lo, hi, seed=shift * 31 + n)
    buf = torch.zeros(rec.size + 64, dtype=torch.uint8, device="cuda:0")
    buf[shift: shift + rec.size] = to_device(rec, "cuda:0")
    d_pos = torch.zeros(n, dtype=torch.int64, device="cuda:0")
    d_res = torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device="cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    bad = rec.copy()
    bad[256 + rec.size // 2 - 128] ^= 0x20
    for r in (rec, bad):
        buf[shift: shift + rec.size] = to_device(r, "cuda:0")
        for integ in (0, 1):
            assert cx.decode_device(buf.data_ptr() + shift, r.size, integ, d_pos.data_ptr(), n, d_res.data_ptr(), s) == 0
            torch.cuda.synchronize()
            res = _res(d_res)
            orc, oe, oh, of = O.decode_batch_slice_with(r, integ)
            assert res.error.kind == orc and res.error.astuple() == oe.astuple()
            if orc == 0:
                assert np.array_equal(to_host(d_pos).astype(np.uint64), of)


def test_one_context_two_streams(cx):
    """Enqueues of one context alternate between two streams: the context orders
    them (its scratch is shared), so every result stays exact."""
    torch = _torch()
    recs = [O.synth_batch(4000, 1024, 1024, seed=21), O.synth_batch(3000, 64, 4096, seed=22)]
    bad = recs[1].copy()
    bad[256 + 5000] ^= 1
    recs.append(bad)
    drecs = [to_device(r, "cuda:0") for r in recs]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    res = [torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device="cuda:0") for _ in range(12)]
    torch.cuda.synchronize()
    for k in range(12):
        r = recs[k % 3]
        assert cx.decode_device(drecs[k % 3].data_ptr(), r.size, 0, None, 0, res[k].data_ptr(),
                                streams[k % 2].cuda_stream) == 0
    torch.cuda.synchronize()
    for k in range(12):
        orc, oe, _, _ = O.decode_batch_slice_with(recs[k % 3], 0)
        got = _res(res[k])
        assert got.error.kind == orc and got.error.astuple() == oe.astuple()


def test_two_contexts_concurrent_variable_decodes():
    """Variable-size (general-walk) decodes from two contexts on two streams at
    once, each from its own host thread: the general kernel's barriers count only
    the workgroups that joined, so neither waits for the other (no timeout) and
    both results are exact."""
    torch = _torch()
    from iggy_amd.codec import Codec
    recs = [O.synth_batch(60_000, 64, 4096, seed=31), O.synth_batch(40_000, 0, 3000, 2, seed=32)]
    expect = [O.decode_batch_slice_with(r, 0) for r in recs]
    ctxs = [Codec(0), Codec(0)]
    errors = []

    def run(k):
        try:
            s = torch.cuda.Stream()
            d = to_device(recs[k], "cuda:0")
            n = int(expect[k][2].message_count)
            pos = torch.zeros(n, dtype=torch.int64, device="cuda:0")
            res = torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device="cuda:0")
            torch.cuda.synchronize()
            for it in range(6):
                assert ctxs[k].decode_device(d.data_ptr(), recs[k].size, it & 1, pos.data_ptr(), n, res.data_ptr(),
                                             s.cuda_stream) == 0
            s.synchronize()
            got = _res(res)
            assert got.error.kind == 0, got.error
            assert got.path == 2
            assert np.array_equal(to_host(pos).astype(np.uint64), expect[k][3])
        except Exception as ex:  # surfaced below
            errors.append(ex)

    th = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for c in ctxs:
        c.close()
    assert not errors, errors


def test_recovery_after_timed_out_decode():
    """Diagnostic build only: a decode whose consumer gives up at once (as a
    timed-out wait does) while its producers run on must not leak into the next
    decode on the context: a flipped body byte is still InvalidMessageChecksum."""
    import os
    from iggy_amd import codec as C
    if not os.path.exists(C.DIAG_LIB_PATH):
        pytest.skip("diagnostic build not present")
    torch = _torch()
    L = C.load(C.DIAG_LIB_PATH)
    cx = C.Codec(0, library=L)
    try:
        rec = O.synth_batch(200_000, 1024, 1024, seed=41)
        bad = rec.copy()
        bad[256 + 1072 * 150_000 + 700] ^= 8  # body byte: stored checksums intact
        d_good = to_device(rec, "cuda:0")
        d_bad = to_device(bad, "cuda:0")
        res = torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device="cuda:0")
        s = torch.cuda.current_stream().cuda_stream
        L.iggy_codec_debug_set(cx.handle, 4096)
        assert cx.decode_device(d_good.data_ptr(), rec.size, 0, None, 0, res.data_ptr(), s) == 0
        torch.cuda.synchronize()
        assert _res(res).error.kind == abi.ERR_TIMEOUT
        L.iggy_codec_debug_set(cx.handle, 0)
        for _ in range(2):
            assert cx.decode_device(d_bad.data_ptr(), bad.size, 0, None, 0, res.data_ptr(), s) == 0
            torch.cuda.synchronize()
            orc, oe, _, _ = O.decode_batch_slice_with(bad, 0)
            got = _res(res)
            assert orc == abi.ERR_INVALID_MESSAGE_CHECKSUM
            assert got.error.astuple() == oe.astuple()
            assert cx.decode_device(d_good.data_ptr(), rec.size, 0, None, 0, res.data_ptr(), s) == 0
            torch.cuda.synchronize()
            assert _res(res).error.kind == 0
    finally:
        cx.close()


@pytest.mark.parametrize("shift", [0, 5])
def test_register_verify_loop_fallback(shift):
    """Diagnostic build only: the register verify loop of the general walk (the form
    records of 4 GiB and more take, forced by debug bit 0x200000) gives the same
    verdicts as the LDS-ring loop on variable-size records, clean and with a body
    byte flipped, at a misaligned record start."""
    import os
    from iggy_amd import codec as C
    if not os.path.exists(C.DIAG_LIB_PATH):
        pytest.skip("diagnostic build not present")
    torch = _torch()
    L = C.load(C.DIAG_LIB_PATH)
    cx = C.Codec(0, library=L)
    try:
        n = 3000
        rec = O.synth_batch(n, 64, 4096, seed=77 + shift)
        bad = rec.copy()
        bad[256 + rec.size // 3] ^= 0x10
        buf = torch.zeros(rec.size + 64, dtype=torch.uint8, device="cuda:0")
        d_pos = torch.zeros(n, dtype=torch.int64, device="cuda:0")
        res = torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device="cuda:0")
        s = torch.cuda.current_stream().cuda_stream
        for bits in (0x200000, 0):
            L.iggy_codec_debug_set(cx.handle, bits)
            for r in (rec, bad):
                buf[shift: shift + r.size] = to_device(r, "cuda:0")
                assert cx.decode_device(buf.data_ptr() + shift, r.size, 0, d_pos.data_ptr(), n, res.data_ptr(), s) == 0
                torch.cuda.synchronize()
                got = _res(res)
                orc, oe, _, of = O.decode_batch_slice_with(r, 0)
                assert got.error.kind == orc and got.error.astuple() == oe.astuple(), (bits, got.error.astuple())
                if orc == 0:
                    assert np.array_equal(to_host(d_pos).astype(np.uint64), of)
        L.iggy_codec_debug_set(cx.handle, 0)
    finally:
        cx.close()

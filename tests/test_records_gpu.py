"""GPU parity of the one-launch multi-record decode (decode_records.hip) and the
one-launch disk-chunk walk (slice.hip k_chunk_walk) behind the walks over
sequences of batches: walk_disk_chunk (poll_plan.rs:950-1011), recover_segment
(segment_recovery.rs:425-530), walk_segment_payload (state_transfer.rs:715-833)
and poll_decode (poll_messages.rs:95-165 / polled_messages.rs:95-150), each
against the oracle. The records are single-stride (the one-launch path) unless a
case says otherwise: short and long frames, 1..24-frame records (the short batch-
checksum input), empty payloads, a stride that breaks mid-record and continues
(the general walk takes over), corruption of every kind. Byte work: all exact."""
import struct

import numpy as np
import pytest

from iggy_amd import abi
from iggy_amd.codec import raw_messages
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cx():
    from iggy_amd.codec import Codec
    c = Codec(0)
    yield c
    c.close()


def _record(pls, seed, base_offset, base_ts):
    """A stamped record with exactly these payload lengths."""
    pls = np.asarray(pls, dtype=np.uint32)
    n = pls.size
    rng = np.random.default_rng(seed)
    ids = rng.integers(1, 2**63, size=2 * n, dtype=np.uint64)
    ots = (1_700_000_000_000_000 + np.arange(n)).astype(np.uint64)
    pay = rng.integers(0, 256, size=int(pls.sum()), dtype=np.uint8)
    rc, e, out = O.encode_batch(raw_messages(ids, ots, pay, pls), 1)
    assert rc == 0, e
    rc, e, h, st = O.stamp_batch(np.frombuffer(out, dtype=np.uint8).copy(), base_offset, base_ts)
    assert rc == 0, e
    return np.frombuffer(st, dtype=np.uint8).copy()


def _stride_break(n=1000, pl=256, at=500):
    """Single-stride length overall (batch_length % S == 0) but frame `at` is 8 B
    shorter and frame at+1 8 B longer: the speculation breaks and the walk goes on."""
    pls = [pl] * n
    pls[at] -= 8
    pls[at + 1] += 8
    return pls


def _chunk(shapes, base_offset=1000, seed=11):
    """shapes: payload-length lists (or (n, pl) pairs) -> consecutive stamped batches."""
    recs, off = [], base_offset
    for k, sh in enumerate(shapes):
        pls = [sh[1]] * sh[0] if isinstance(sh, tuple) else sh
        recs.append(_record(pls, seed * 131 + k, off, 5000 + 10 * k))
        off += len(pls)
    starts = np.cumsum([0] + [r.size for r in recs])
    return np.concatenate(recs), starts


C1_CHUNK = [(1000, 256)] * 3 + [(449, 256)]   # ~1 MiB of C1 producer batches
MIXED = [(30, 64), (1, 5), (24, 100), (25, 100), (2000, 1024), (1000, 0), (300, 200), (7, 4000)]


def _walk_same(cx, chunk, *args, **kw):
    rc, w, fr, hd = cx.walk_disk_chunk(chunk, *args, **kw)
    orc, ow, ofr, ohd = O.walk_disk_chunk(chunk, *args, **kw)
    assert rc == orc, (w.astuple(), ow.astuple())
    assert w.astuple() == ow.astuple()
    assert [f.astuple() for f in fr] == [f.astuple() for f in ofr]
    assert hd == ohd
    return w


@pytest.mark.parametrize("shapes", [C1_CHUNK, MIXED], ids=["c1", "mixed"])
@pytest.mark.parametrize("q", [(abi.LOOKUP_OFFSET, 0, 10**9, 2**64 - 1), (abi.LOOKUP_OFFSET, 1500, 30, 2**64 - 1),
                               (abi.LOOKUP_OFFSET, 1999, 1002, 2**64 - 1), (abi.LOOKUP_OFFSET, 1000, 10**6, 2600),
                               (abi.LOOKUP_OFFSET, 3400, 1, 2**64 - 1), (abi.LOOKUP_OFFSET, 10**9, 5, 2**64 - 1),
                               (abi.LOOKUP_TIMESTAMP, 5015, 100, 2**64 - 1), (abi.LOOKUP_TIMESTAMP, 0, 2500, 1999)])
@pytest.mark.parametrize("integrity", [0, 1])
def test_chunk_one_launch(cx, shapes, q, integrity):
    chunk, starts = _chunk(shapes)
    kind, value, count, ceiling = q
    for already in (0, 7):
        _walk_same(cx, chunk, kind, value, count, ceiling, already, integrity)
    _walk_same(cx, chunk, kind, value, count, ceiling, 0, integrity, cap=1)


def test_chunk_one_launch_tails_corruption_and_general(cx):
    chunk, starts = _chunk(C1_CHUNK)
    q = (abi.LOOKUP_OFFSET, 1000, 10**9)
    S = 48 + 256
    cases = [chunk[: starts[2] + 1000], chunk[: starts[3] + 100], chunk[: starts[1] + 255],
             np.concatenate([chunk, np.zeros(300, dtype=np.uint8)])]
    b = chunk.copy(); b[starts[2] + 40] ^= 1; cases.append(b)                   # batch checksum
    b = chunk.copy(); b[starts[1] + 256 + S * 7 + 200] ^= 4; cases.append(b)    # message checksum
    b = chunk.copy(); b[starts[1] + 256 + S * 999 + 200] ^= 4; cases.append(b)  # the last frame's
    b = chunk.copy(); b[starts[0] + 100] = 9; cases.append(b)                   # header reserved byte
    b = chunk.copy(); b[starts[2] + 256 + S * 600 + 40] = 1; cases.append(b)    # frame reserved: walk stops
    b = chunk.copy(); struct.pack_into("<I", b, starts[1] + 48, 999); cases.append(b)  # count off by one
    # a stride break that the walk continues through: the general walk decides
    gen, gst = _chunk([(1000, 256), _stride_break(), (1000, 256)])
    cases.append(gen)
    b = gen.copy(); b[gst[1] + 256 + S * 700 + 100] ^= 2; cases.append(b)
    for c in cases:
        for integrity in (0, 1):
            _walk_same(cx, c, *q, integrity=integrity)
            _walk_same(cx, c, abi.LOOKUP_OFFSET, 1990, 1500, integrity=integrity)


def _segment(shapes, base_offset):
    return _chunk(shapes, base_offset=base_offset, seed=17)


def test_recover_and_walk_segment_one_launch(cx):
    shapes = [(1000, 256)] * 20 + [(24, 100), (1, 0), (3000, 1024), _stride_break(), (500, 64)]
    seg, starts = _segment(shapes, 500)
    cases = [seg, seg[:-1], seg[: starts[7] + 5000]]
    for k in (0, 6, 20, 23, 24):
        b = seg.copy(); b[starts[k] + 256 + 48 + 3] ^= 0x20; cases.append(b)    # message checksum
        b = seg.copy(); b[starts[k] + 41] ^= 2; cases.append(b)                  # batch checksum
    for buf in cases:
        for so in (500, 501):
            rc, out = cx.recover_segment(buf, so)
            orc, oout = O.recover_segment(buf, so)
            assert rc == orc == 0
            assert out.astuple() == oout.astuple()
        rc, w, idx = cx.walk_segment_payload(buf, 500)
        orc, ow, oidx = O.walk_segment_payload(buf, 500)
        assert rc == orc, (w.astuple(), ow.astuple())
        assert w.astuple() == ow.astuple() and idx == oidx


def test_segment_of_many_c1_batches(cx):
    """A 61 MB segment of 200 C1 batches: 1 600 workgroups of one launch."""
    shapes = [(1000, 256)] * 200
    recs, off = [], 0
    base = _record([256] * 1000, 7, 0, 1)
    for k in range(200):  # the same payloads, restamped per batch (fast to build)
        rc, e, h, st = O.stamp_batch(base, off, 10 + k)
        recs.append(np.frombuffer(st, dtype=np.uint8).copy())
        off += 1000
    seg = np.concatenate(recs)
    rc, w, idx = cx.walk_segment_payload(seg, 0)
    orc, ow, oidx = O.walk_segment_payload(seg, 0)
    assert rc == orc == 0 and w.astuple() == ow.astuple() and idx == oidx
    assert w.batches == 200 and w.end_offset == 199_999
    b = seg.copy(); b[304256 * 150 + 256 + 304 * 999 + 100] ^= 1
    rc, out = cx.recover_segment(b, 0)
    orc, oout = O.recover_segment(b, 0)
    assert out.astuple() == oout.astuple() and out.batches == 150


@pytest.mark.parametrize("mode", [0, 1])
def test_poll_one_launch(cx, mode):
    body, starts = _chunk([(10, 100), (300, 900), (1, 0), (2000, 1024), (24, 16)])
    for b in (body, body[:-1]):
        rc, e, msgs = cx.poll_decode(b, mode)
        orc, oe, om = O.poll_decode(b, mode)
        assert rc == orc and e.astuple() == oe.astuple()
        assert [m.astuple() for m in msgs] == [m.astuple() for m in om]
    # a stride break continued by the walk, between single-stride records
    body2, st2 = _chunk([(100, 100), _stride_break(300, 50, 120), (40, 1000)])
    bad = body2.copy(); bad[st2[2] + 256 + 40] = 1   # frame reserved in the third record
    for b in (body2, bad):
        rc, e, msgs = cx.poll_decode(b, mode)
        orc, oe, om = O.poll_decode(b, mode)
        assert rc == orc and e.astuple() == oe.astuple()
        assert [m.astuple() for m in msgs] == [m.astuple() for m in om]


def test_completion_flag_sequence_wrap():
    """Diagnostic build only: the host-mapped completion flags' sequence wraps (2^32
    values, 0 skipped) in the middle of a run of one-launch chunk walks and segment
    recoveries; every result still matches the oracle."""
    import os
    from iggy_amd import codec as C
    if not os.path.exists(C.DIAG_LIB_PATH):
        pytest.skip("diagnostic build not present")
    L = C.load(C.DIAG_LIB_PATH)
    c = C.Codec(0, library=L)
    try:
        chunk, starts = _chunk(C1_CHUNK)
        seg, _ = _segment([(1000, 256)] * 3 + [(24, 100)], 500)
        L.iggy_codec_debug_set(c.handle, 0x40000000)
        for k in range(40):
            _walk_same(c, chunk, abi.LOOKUP_OFFSET, 1000 + 37 * k, 500, integrity=k & 1)
            if k % 4 == 0:
                rc, out = c.recover_segment(seg, 500)
                orc, oout = O.recover_segment(seg, 500)
                assert rc == orc == 0 and out.astuple() == oout.astuple()
    finally:
        c.close()


def test_segment_above_zero_copy_table_limit(cx):
    """A segment whose one launch needs more than 4,096 workgroups (560 C1 batches,
    170 MB): the task table and workgroup map go up with one H2D copy instead of being
    read from host-mapped memory. Walk, recovery and a corruption near the end exact."""
    base = _record([256] * 1000, 9, 0, 1)
    recs, off = [], 0
    for k in range(560):
        rc, e, h, st = O.stamp_batch(base, off, 10 + k)
        recs.append(np.frombuffer(st, dtype=np.uint8).copy())
        off += 1000
    seg = np.concatenate(recs)
    rc, w, idx = cx.walk_segment_payload(seg, 0)
    orc, ow, oidx = O.walk_segment_payload(seg, 0)
    assert rc == orc == 0 and w.astuple() == ow.astuple() and idx == oidx
    assert w.batches == 560
    b = seg.copy(); b[304256 * 541 + 256 + 304 * 17 + 100] ^= 1
    rc, out = cx.recover_segment(b, 0)
    orc, oout = O.recover_segment(b, 0)
    assert out.astuple() == oout.astuple() and out.batches == 541

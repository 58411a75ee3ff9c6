"""The resident decode service (iggy_codec_service_start, decode_records.hip
k_decode_service): synchronous host decodes of small single-stride records posted to
resident workgroups instead of a launch per call. Every verdict, header and position
list must be the launch path's and the oracle's (decode_batch_slice_with,
core/binary_protocol/src/batch.rs:391-506), including the records the service does not
take (too many blocks, a stride that breaks mid-record) and the grid's idle exit."""
import time

import numpy as np
import pytest

from iggy_amd import abi
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture
def cx():
    from iggy_amd.codec import Codec
    c = Codec(0)
    yield c
    c.close()


def _stride_break_record():
    from iggy_amd.codec import raw_messages
    n = 600
    rng = np.random.default_rng(7)
    pls = np.full(n, 200, dtype=np.uint32)
    pls[300], pls[301] = 216, 184  # same blob length as all-200, the walk finds the break
    ids = rng.integers(1, 2**63, size=2 * n, dtype=np.uint64)
    ots = (1_700_000_000_000_000 + np.arange(n)).astype(np.uint64)
    pay = rng.integers(0, 256, size=int(pls.sum()), dtype=np.uint8)
    rc, e, out = O.encode_batch(raw_messages(ids, ots, pay, pls), 0)
    assert rc == 0
    return np.frombuffer(out, dtype=np.uint8).copy()


def _records():
    clean = O.synth_batch(1000, 256, seed=11)           # C1: 8 blocks, the service's largest
    bad = clean.copy()
    bad[256 + 304 * 777 + 100] ^= 0x20                  # one payload bit of frame 777
    badcs = O.synth_batch(500, 100, 900, seed=12)       # variable sizes: not single-stride
    tiny = O.synth_batch(4, 256, seed=13)
    short = O.synth_batch(30, 40, seed=14)              # hashed <= 240 B: one lane per frame
    big = O.synth_batch(1200, 256, seed=15)             # 10 blocks: the launch path
    hdr_bad = clean.copy()
    hdr_bad[60] = 1                                     # batch header reserved byte
    trunc = clean[: clean.size - 10].copy()             # UnexpectedEof / tiling
    return [clean, bad, badcs, tiny, short, big, hdr_bad, trunc, _stride_break_record()]


def _check(cx, rec, integrity, pos):
    want = O.decode_batch_slice_with(rec, integrity)
    h, e = abi.BatchHeader(), abi.WireError()
    rc, nf = cx.decode_batch_into(rec, integrity, pos, h, e)
    assert rc == want[0] and e.astuple() == want[1].astuple() and h.astuple() == want[2].astuple(), (rc, want[0])
    if rc == 0:
        assert nf == len(want[3]) and np.array_equal(pos[:nf], np.asarray(want[3], dtype=np.uint64))


@pytest.mark.parametrize("registered", [False, True])
def test_service_matches_oracle(cx, registered):
    from iggy_amd.codec import host_buffer, page_aligned
    recs = [page_aligned(r) for r in _records()]
    poss = [host_buffer(r.size // 48 + 1, np.uint64) for r in recs]
    if registered:
        for a in recs + poss:
            cx.host_register(a)
    try:
        cx.service_start()
        s0 = cx.host_stats()
        for rnd in range(3):
            for integrity in (abi.INTEGRITY_VERIFY, abi.INTEGRITY_LAYOUT_ONLY):
                for r, p in zip(recs, poss):
                    p[:] = 0
                    _check(cx, r, integrity, p)
        s1 = cx.host_stats()
        assert s1["service_posts"] > s0["service_posts"]  # the small single-stride records went to it
        cx.service_stop()
        for r, p in zip(recs, poss):  # and the launch path after the stop
            _check(cx, r, abi.INTEGRITY_VERIFY, p)
        assert cx.host_stats()["service_posts"] == s1["service_posts"]
    finally:
        if registered:
            for a in recs + poss:
                cx.host_unregister(a)


@pytest.mark.parametrize("registered", [False, True])
def test_service_back_to_back_posts_of_one_shape(cx, registered):
    """Records of one shape posted back to back, each verdict judged against its own
    oracle result: a clean record, the same with one payload bit of a late block flipped
    (its stored checksums unchanged, so only that block's first-bad word tells them
    apart), and the same with another base offset (only the relayed prefix differs).
    A stale relay granule or block record from the previous post would pass one for the
    other."""
    from iggy_amd.codec import host_buffer, page_aligned
    clean = O.synth_batch(1000, 256, seed=51)
    bad = clean.copy()
    bad[256 + 304 * 990 + 200] ^= 0x01                  # frame 990: block 7, the last
    moved = clean.copy()
    moved[8:16].view(np.uint64)[0] += 1000
    recs = [page_aligned(r) for r in (clean, bad, moved)]
    wants = [O.decode_batch_slice_with(r, abi.INTEGRITY_VERIFY) for r in recs]
    assert wants[0][0] == 0 and wants[1][0] != 0
    pos = host_buffer(clean.size // 48 + 1, np.uint64)
    if registered:
        for a in recs + [pos]:
            cx.host_register(a)
    try:
        cx.service_start()
        h, e = abi.BatchHeader(), abi.WireError()
        for k in range(300):
            i = (k * 7 + k // 3) % 3
            rc, nf = cx.decode_batch_into(recs[i], abi.INTEGRITY_VERIFY, pos, h, e)
            want = wants[i]
            assert rc == want[0] and e.astuple() == want[1].astuple() and h.astuple() == want[2].astuple(), (k, i, rc)
            if rc == 0:
                assert nf == len(want[3]) and np.array_equal(pos[:nf], np.asarray(want[3], dtype=np.uint64))
        cx.service_stop()
    finally:
        if registered:
            for a in recs + [pos]:
                cx.host_unregister(a)


@pytest.mark.parametrize("registered", [False, True])
def test_service_header_prefix_follows_each_post(cx, registered):
    """The post carries the record's first 304 B (batch header + frame 0's header) to
    the workgroups: the same buffer rewritten between calls (header fields, a reserved
    byte, frame 0's lengths, its checksum) must be judged on its new bytes every time."""
    from iggy_amd.codec import host_buffer, page_aligned
    base = O.synth_batch(1000, 256, seed=41)
    rec = page_aligned(base)
    pos = host_buffer(rec.size // 48 + 1, np.uint64)
    if registered:
        cx.host_register(rec)
        cx.host_register(pos)
    try:
        cx.service_start()
        edits = [
            lambda r: r[8:16].view(np.uint64).__setitem__(0, 123456789),   # base_offset
            lambda r: r.__setitem__(200, 7),                                 # reserved byte
            lambda r: r.__setitem__(256 + 3, r[256 + 3] ^ 0x40),             # frame 0 checksum
            lambda r: r[256 + 36:256 + 40].view(np.uint32).__setitem__(0, 255),  # frame 0 payload_length
            lambda r: r[256 + 24:256 + 28].view(np.uint32).__setitem__(0, 9),    # frame 0 offset_delta
            lambda r: r.__setitem__(256 + 44, 1),                                # frame 0 reserved
            lambda r: None,                                                  # back to clean
        ]
        for rnd in range(2):
            for ed in edits:
                rec[:] = base
                ed(rec)
                _check(cx, rec, abi.INTEGRITY_VERIFY, pos)
                _check(cx, rec, abi.INTEGRITY_LAYOUT_ONLY, pos)
        cx.service_stop()
    finally:
        if registered:
            cx.host_unregister(pos)
            cx.host_unregister(rec)


def test_service_idle_exit_and_relaunch(cx):
    """The grid exits after 20 ms without a post; the next call relaunches it and its
    post is decoded once (the results are the oracle's)."""
    rec = O.synth_batch(1000, 256, seed=21)
    pos = np.zeros(rec.size // 48 + 1, dtype=np.uint64)
    cx.service_start()
    _check(cx, rec, abi.INTEGRITY_VERIFY, pos)
    l0 = cx.host_stats()["service_launches"]
    for _ in range(3):
        time.sleep(0.06)
        _check(cx, rec, abi.INTEGRITY_VERIFY, pos)
    st = cx.host_stats()
    assert st["service_launches"] >= l0 + 3 and st["service_posts"] >= 4
    cx.service_stop()


def test_service_beside_device_decodes_and_destroy():
    """A context with the service running decodes device-resident records (the
    persistent grids beside the resident workgroups) and is destroyed with the service
    still running; a second context then decodes as usual."""
    import ctypes

    import torch

    from iggy_amd.codec import Codec
    from iggy_amd.torch_io import to_device, to_host
    c = Codec(0)
    c.service_start()
    small = O.synth_batch(1000, 256, seed=31)
    pos = np.zeros(small.size // 48 + 1, dtype=np.uint64)
    _check(c, small, abi.INTEGRITY_VERIFY, pos)
    rec = O.synth_batch(200_000, 1024, seed=32)  # 215 MB: the persistent uniform grid
    d = to_device(rec)
    d_res = torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device="cuda")
    d_pos = torch.zeros(200_000, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        assert c.decode_device(d.data_ptr(), rec.size, 0, d_pos.data_ptr(), 200_000, d_res.data_ptr(), s) == 0
        _check(c, small, abi.INTEGRITY_VERIFY, pos)
    torch.cuda.synchronize()
    r = abi.DecodeResult.from_buffer_copy(to_host(d_res).tobytes())
    assert r.error.kind == 0 and r.frame_count == 200_000
    c.close()  # service still running: destroy stops it first
    c2 = Codec(0)
    try:
        _check(c2, small, abi.INTEGRITY_VERIFY, pos)
    finally:
        c2.close()

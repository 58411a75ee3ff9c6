"""Caller host memory at the boundary.

The reference borrows `&[u8]` for the call only (core/binary_protocol/src/batch.rs:391):
the caller may free or reuse a buffer the moment a codec call returns. These tests run
with the HIP runtime's defaults (no GPU_PINNED_MIN_XFER_SIZE override) and drive every
host entry point with freshly allocated PAGEABLE numpy buffers that are freed right
after the call, interleaved with torch's own pageable copies into new allocations --
the sequence that faulted in rounds 3-4 -- and check each result against the oracle.
They also pin the codec's pinned / pageable classification (iggy_codec_host_pinned)."""
import ctypes
import gc
import os

import numpy as np
import pytest

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


def test_runtime_defaults_in_this_process():
    assert "GPU_PINNED_MIN_XFER_SIZE" not in os.environ


def test_host_pinned_classification(cx):
    import torch
    from iggy_amd.codec import host_buffer
    a = np.zeros(1 << 20, dtype=np.uint8)
    assert not cx.host_pinned(a.ctypes.data, a.size)
    b = host_buffer(3 << 20)
    cx.host_register(b)
    try:
        assert cx.host_pinned(b.ctypes.data, b.size)
        assert cx.host_pinned(b.ctypes.data + 4097, 1000)
        assert not cx.host_pinned(b.ctypes.data + 4096, b.size)  # runs past the range
    finally:
        cx.host_unregister(b)
    assert not cx.host_pinned(b.ctypes.data, b.size)
    t = torch.empty(1 << 20, dtype=torch.uint8).pin_memory()  # hipHostMalloc
    assert cx.host_pinned(t.data_ptr(), t.numel())
    assert cx.host_pinned(t.data_ptr() + 100, 1000)
    assert cx.host_pinned(0, 0)  # nothing to copy


def _fresh(rec):
    """A new pageable copy of rec (a new allocation, freed by the caller's del)."""
    x = np.empty(rec.size, dtype=np.uint8)
    x[:] = rec
    return x


def test_pageable_buffers_freed_after_every_call(cx):
    import torch
    big = O.synth_batch(150_000, 1024, seed=5)            # 161 MB: persistent decode path
    small = O.synth_batch(3000, 200, 300, seed=6)         # < 16 MiB: host-flag path
    # 8 batches with contiguous offsets (recover_segment walks them all)
    seg = np.concatenate([np.frombuffer(O.stamp_batch(O.synth_batch(1000, 256, seed=s), 1000 * s, 10 + s)[3],
                                        dtype=np.uint8) for s in range(8)])
    ob = O.decode_batch_slice_with(big, 0)
    osm = O.decode_batch_slice_with(small, 0)
    dev = torch.randint(0, 255, (64 << 20,), dtype=torch.uint8, device="cuda")
    ref_sum = int(dev.sum().item())
    for it in range(4):
        x = _fresh(big)
        rc, e, h, f = cx.decode_batch_slice_with(x, abi.INTEGRITY_VERIFY)
        del x
        assert (rc, h.astuple()) == (ob[0], ob[2].astuple()) and np.array_equal(f, ob[3])
        # the caller's own copies between (through pinned staging, iggy_amd/torch_io.py)
        host = to_host(dev)
        assert int(host.sum(dtype=np.uint64)) == ref_sum
        back = to_device(host.copy())
        assert torch.equal(back, dev)
        del host, back
        x = _fresh(small)
        rc, e, h, f = cx.decode_batch_slice_with(x, abi.INTEGRITY_VERIFY)
        del x
        assert (rc, h.astuple()) == (osm[0], osm[2].astuple()) and np.array_equal(f, osm[3])
        x = _fresh(seg)
        rc, rec = cx.recover_segment(x, 0)
        del x
        orc, orec = O.recover_segment(seg, 0)
        assert rc == orc == 0 and rec.batches == orec.batches == 8 and rec.walked_bytes == orec.walked_bytes == seg.size
        gc.collect()


def test_pageable_submit_outputs(cx):
    """Asynchronous submits with pageable inputs and outputs: nothing lands in the
    caller's output before the ticket completes, and only on success."""
    rec = O.synth_batch(20000, 100, 2000, seed=19)
    orc, oe, oh, of = O.decode_batch_slice_with(rec, 0)
    pos = np.full(20000, 7, dtype=np.uint64)
    body = _fresh(rec)
    t = cx.decode_submit(body, abi.INTEGRITY_VERIFY, pos)
    del body  # the input was staged inside the submit
    c = cx.wait(t)
    assert c.error.kind == 0 and c.header.astuple() == oh.astuple()
    assert np.array_equal(pos, of)
    # frame capacity too small: a capacity error and the caller's array untouched
    short = np.full(10, 7, dtype=np.uint64)
    t = cx.decode_submit(rec, abi.INTEGRITY_VERIFY, short)
    assert cx.wait(t).error.kind == abi.ERR_CAPACITY
    assert (short == 7).all()


def test_registered_record_read_in_place(cx):
    """A registered record of <= 4 MiB is decoded in place (the kernel reads the
    host-mapped bytes, no H2D): same verdicts as the oracle, at the start of the
    registered range and at an interior, unaligned offset, clean and corrupted, and a
    larger registered record (copied as before)."""
    from iggy_amd.codec import host_buffer
    recs = [O.synth_batch(1000, 256, seed=31), O.synth_batch(700, 100, 900, seed=32),
            O.synth_batch(1500, 1024, seed=33),  # 1.6 MB: in place
            O.synth_batch(5000, 1024, seed=34)]  # 5.4 MB: above the in-place limit, copied
    bad = recs[0].copy()
    bad[256 + 48 * 500 + 60] ^= 0x40  # one payload bit of frame 500
    recs.append(bad)
    for rec in recs:
        want = O.decode_batch_slice_with(rec, 0)
        for off in (0, 4099):
            buf = host_buffer(off + rec.size + 64)
            buf[off:off + rec.size] = rec
            pos = host_buffer(rec.size // 48 + 1, np.uint64)
            cx.host_register(buf)
            cx.host_register(pos)
            try:
                view = buf[off:off + rec.size]
                assert cx.host_pinned(view.ctypes.data, view.size)
                h, e = abi.BatchHeader(), abi.WireError()
                rc, nf = cx.decode_batch_into(view, abi.INTEGRITY_VERIFY, pos, h, e)
            finally:
                cx.host_unregister(pos)
                cx.host_unregister(buf)
            assert rc == want[0] and e.astuple() == want[1].astuple() and h.astuple() == want[2].astuple()
            if rc == 0:
                assert np.array_equal(pos[:nf], np.asarray(want[3], dtype=np.uint64))


def _stride_break_record():
    """1000 frames: 256-B payloads, except frames 500 / 501 (272 / 240 B), so the blob
    is still a multiple of frame 0's size and only the walk finds the break."""
    from iggy_amd.codec import raw_messages
    n = 1000
    rng = np.random.default_rng(41)
    pls = np.full(n, 256, dtype=np.uint32)
    pls[500], pls[501] = 272, 240
    ids = rng.integers(1, 2**63, size=2 * n, dtype=np.uint64)
    ots = (1_700_000_000_000_000 + np.arange(n)).astype(np.uint64)
    pay = rng.integers(0, 256, size=int(pls.sum()), dtype=np.uint8)
    rc, e, out = O.encode_batch(raw_messages(ids, ots, pay, pls), 0)
    assert rc == 0
    return np.frombuffer(out, dtype=np.uint8).copy()


@pytest.mark.parametrize("registered", [False, True])
def test_submit_single_stride_fast_path(cx, registered):
    """decode_submit of records <= 16 MiB (one k_decode_records launch on the context's
    stream, the verdict straight into the slot's host-mapped record, k_decode_general
    behind it): clean, corrupted and stride-breaking records, with and without
    positions, several in flight, each against the oracle."""
    clean = O.synth_batch(1000, 256, seed=43)
    bad = clean.copy()
    bad[256 + 304 * 700 + 100] ^= 1
    from iggy_amd.codec import host_buffer, page_aligned
    recs = [clean, bad, _stride_break_record(), O.synth_batch(3000, 1000, seed=44),  # 3.1 MB: in place
            O.synth_batch(5000, 1000, seed=45)]  # 5.2 MB: copied (pageable: from the slot's staging)
    recs = [page_aligned(r) for r in recs]  # (registrations may not share a page)
    poss = [host_buffer(r.size // 48 + 1, np.uint64) for r in recs]
    if registered:
        for a in recs + poss:
            cx.host_register(a)
    try:
        for with_pos in (True, False):
            tks = [cx.decode_submit(r, abi.INTEGRITY_VERIFY, p if with_pos else None) for r, p in zip(recs, poss)]
            for tk, r, p in zip(tks, recs, poss):
                c = cx.wait(tk)
                orc, oe, oh, of = O.decode_batch_slice_with(r, 0)
                assert c.error.astuple() == oe.astuple()
                assert c.header.astuple() == oh.astuple()
                if orc == 0:
                    assert c.frame_count == len(of)
                    if with_pos:
                        assert np.array_equal(p[:c.frame_count], np.asarray(of, dtype=np.uint64))
    finally:
        if registered:
            for a in recs + poss:
                cx.host_unregister(a)


def test_pageable_submit_buffers_reused_at_once(cx):
    """Pageable records submitted back to back (8 in flight, the slots' own mapped
    staging) while the caller overwrites each input right after its submit returns
    (batch.rs:391 borrows for the call only): every verdict and position list is the
    oracle's for the bytes the caller passed. Sizes on both sides of the in-place limit
    (4 MiB), a corrupted record among them, and the slots reused with other records."""
    recs = [O.synth_batch(1000, 256, seed=50 + k) for k in range(4)]          # C1 shapes, in place
    recs += [O.synth_batch(2000, 1000, seed=60),                                # 2 MB, in place
             O.synth_batch(4500, 1000, seed=61)]                                # 4.7 MB, staging + DMA
    bad = O.synth_batch(1000, 256, seed=62)
    bad[256 + 304 * 10 + 70] ^= 0x10
    recs += [bad, O.synth_batch(30, 4000, seed=63)]
    wants = [O.decode_batch_slice_with(r, 0) for r in recs]
    for rnd in range(3):
        order = list(range(len(recs)))[rnd:] + list(range(len(recs)))[:rnd]  # other slot per record
        bufs, poss, tks = [], [], []
        for i in order:
            b = _fresh(recs[i])
            p = np.zeros(recs[i].size // 48 + 1, dtype=np.uint64)
            tks.append(cx.decode_submit(b, abi.INTEGRITY_VERIFY, p))
            b[:] = 0xA5  # the caller reuses its buffer at once
            bufs.append(b)
            poss.append(p)
        for tk, i, p in zip(tks, order, poss):
            c = cx.wait(tk)
            orc, oe, oh, of = wants[i]
            assert c.error.astuple() == oe.astuple(), (rnd, i)
            assert c.header.astuple() == oh.astuple(), (rnd, i)
            if orc == 0:
                assert c.frame_count == len(of)
                assert np.array_equal(p[:c.frame_count], np.asarray(of, dtype=np.uint64)), (rnd, i)
        del bufs
        gc.collect()


def test_pageable_sync_decode_around_in_place_limit(cx):
    """The synchronous decode of pageable records on both sides of the in-place limit
    (4 MiB: one memcpy into the context's mapped staging, read in place; above it, the
    two staging chunks and a DMA), clean and with one corrupted payload byte, against
    the oracle; the staging is reused call after call with other bytes."""
    for n, pl in ((1500, 1000), (3800, 1024), (4400, 1000)):  # 1.5 / 3.9 / 4.4 MB
        rec = O.synth_batch(n, pl, seed=n)
        bad = rec.copy()
        bad[256 + (48 + pl) * (n - 3) + 100] ^= 0x08
        for r in (rec, bad, rec):
            want = O.decode_batch_slice_with(r, 0)
            x = _fresh(r)
            pos = np.zeros(r.size // 48 + 1, dtype=np.uint64)
            h, e = abi.BatchHeader(), abi.WireError()
            rc, nf = cx.decode_batch_into(x, abi.INTEGRITY_VERIFY, pos, h, e)
            del x
            assert rc == want[0] and e.astuple() == want[1].astuple() and h.astuple() == want[2].astuple()
            if rc == 0:
                assert np.array_equal(pos[:nf], np.asarray(want[3], dtype=np.uint64))


def test_destroy_with_fast_submits_in_flight():
    """A context destroyed while fast-path submits (each on its slot's own stream) are
    still in flight drains those streams before it frees their staging and results; a
    new context then decodes as usual."""
    from iggy_amd.codec import Codec
    recs = [O.synth_batch(1000, 256, seed=70 + k) for k in range(6)]
    poss = [np.zeros(r.size // 48 + 1, dtype=np.uint64) for r in recs]
    c = Codec(0)
    for r, p in zip(recs, poss):
        c.decode_submit(r, abi.INTEGRITY_VERIFY, p)
    c.close()  # no wait: the destroy drains the slot streams
    c2 = Codec(0)
    try:
        want = O.decode_batch_slice_with(recs[0], 0)
        rc, e, h, f = c2.decode_batch_slice_with(recs[0], abi.INTEGRITY_VERIFY)
        assert rc == want[0] == 0 and np.array_equal(f, want[3])
    finally:
        c2.close()


def _soa(n, lo, hi, seed, uh=False):
    """SoA arrays in page-aligned buffers (registrations may not share a page)."""
    from iggy_amd.codec import page_aligned, raw_messages
    rng = np.random.default_rng(seed)
    ids = page_aligned(rng.integers(1, 2**63, size=2 * n, dtype=np.uint64))
    ots = page_aligned((1_700_000_000_000_000 + rng.integers(0, 10**6, size=n)).astype(np.uint64))
    pls = page_aligned(rng.integers(lo, hi + 1, size=n).astype(np.uint32))
    pay = page_aligned(rng.integers(0, 256, size=int(pls.sum()), dtype=np.uint8))
    arrs = [ids, ots, pay, pls]
    if uh:
        uhl = page_aligned(rng.integers(0, 40, size=n).astype(np.uint32))
        uhb = page_aligned(rng.integers(0, 256, size=int(uhl.sum()), dtype=np.uint8))
        arrs += [uhb, uhl]
        return arrs, raw_messages(ids, ots, pay, pls, uhb, uhl)
    return arrs, raw_messages(ids, ots, pay, pls)


@pytest.mark.parametrize("registered", [False, True])
def test_encode_submit_small_batches_in_place(cx, registered):
    """encode_submit of small batches (SoA input of <= 4 MiB: the kernels read it over
    the host link -- registered arrays where they are, pageable ones from the slot's
    staging -- and write the wire bytes into mapped host memory): 8 in flight, with and
    without user headers, empty payloads, the caller's SoA arrays overwritten right
    after each submit, each output byte-exact against the oracle; plus one batch whose
    output capacity is too small (nothing written, capacity error)."""
    from iggy_amd.codec import page_aligned
    cases = [(1000, 256, 256, False), (700, 0, 300, True), (3000, 1, 900, False), (64, 0, 0, False),
             (1000, 256, 256, True), (5, 2000, 5000, False), (2000, 100, 1000, True), (1, 17, 17, False)]
    wants, outs, tks, keep = [], [], [], []
    for k, (n, lo, hi, uh) in enumerate(cases):
        arrs, raw = _soa(n, lo, hi, 80 + k, uh)
        rc, e, w = O.encode_batch(raw, 3)
        assert rc == 0
        wants.append(np.frombuffer(w, dtype=np.uint8))
        out = page_aligned(np.full(len(w) + 32, 0xEE, dtype=np.uint8))
        outs.append(out)
        if registered:
            for a in arrs + [out]:
                if a.size:
                    cx.host_register(a)
        tks.append(cx.encode_submit(raw, 3, out))
        if not registered:
            for a in arrs:
                a[...] = 0x5A  # the caller reuses its arrays at once (they were staged)
        keep.append(arrs)
    try:
        for tk, w, out in zip(tks, wants, outs):
            c = cx.wait(tk)
            assert c.error.kind == 0 and c.bytes == w.size, c.error
            assert np.array_equal(out[:w.size], w)
            assert (out[w.size:] == 0xEE).all()
    finally:
        if registered:
            for arrs, out in zip(keep, outs):
                for a in arrs + [out]:
                    if a.size:
                        cx.host_unregister(a)
    arrs, raw = _soa(500, 10, 50, 99)
    small = np.full(100, 0xEE, dtype=np.uint8)
    c = cx.wait(cx.encode_submit(raw, 0, small))
    assert c.error.kind == abi.ERR_CAPACITY and (small == 0xEE).all()


def test_pinned_submits_never_wait(cx):
    """The asynchronous host API on pinned buffers issues no wait, settle event, staging
    or allocation inside a submit (iggy_codec_host_stats diffed around the submits), so
    one batch's H2D, another's kernels and a third's D2H overlap (C4, VERDICT r05 item 1:
    a settle event recorded after every pinned H2D serialised the copies, 24.7 -> 17.6
    GiB/s). C4-shaped batches (64 K x 1 KiB: the copy path of both submits) plus a
    6-MB single-stride record (the fast path's pinned DMA), all against the oracle."""
    import torch
    from iggy_amd.codec import raw_messages
    n, pl = 65_536, 1024
    total = 256 + n * (48 + pl)
    g = torch.Generator().manual_seed(77)
    t_ids = torch.randint(1, 2**62, (2 * n,), dtype=torch.int64, generator=g).pin_memory()
    t_ots = (1_700_000_000_000_000 + torch.arange(n, dtype=torch.int64)).pin_memory()
    t_pay = torch.randint(0, 256, (n * pl,), dtype=torch.uint8, generator=g).pin_memory()
    t_pls = torch.full((n,), pl, dtype=torch.int32).pin_memory()
    raw = raw_messages(t_ids.numpy().view(np.uint64), t_ots.numpy().view(np.uint64), t_pay.numpy(),
                       t_pls.numpy().view(np.uint32))
    wires = [torch.zeros(total, dtype=torch.uint8).pin_memory() for _ in range(2)]
    poss = [torch.zeros(n, dtype=torch.int64).pin_memory() for _ in range(2)]
    small = O.synth_batch(6000, 1000, seed=78)  # 6.3 MB: fast path, pinned DMA
    t_small = torch.from_numpy(small.copy()).pin_memory()
    p_small = torch.zeros(6000, dtype=torch.int64).pin_memory()
    # the encode checked against the oracle once
    c = cx.wait(cx.encode_submit(raw, 1, wires[0].numpy()))
    assert c.error.kind == 0 and c.bytes == total
    rc, e, want = O.encode_batch(raw, 1)
    assert rc == 0 and np.array_equal(wires[0].numpy(), np.frombuffer(want, dtype=np.uint8))

    def three():
        return [cx.encode_submit(raw, 1, wires[1].numpy()),
                cx.decode_submit(wires[0].numpy(), abi.INTEGRITY_VERIFY, poss[1].numpy().view(np.uint64)),
                cx.decode_submit(t_small.numpy(), abi.INTEGRITY_VERIFY, p_small.numpy().view(np.uint64))]

    for t in three():  # warm-up: the three slots' buffers, streams and scratch sized
        assert cx.wait(t).error.kind == 0
    s0 = cx.host_stats()
    tks = three()
    s1 = cx.host_stats()
    done = [cx.wait(t) for t in tks]
    for k in ("staged_bytes", "settle_events", "host_waits", "device_allocs", "pinned_allocs"):
        assert s1[k] == s0[k], (k, s0, s1)
    assert s1["pinned_h2d_bytes"] - s0["pinned_h2d_bytes"] == 28 * n + n * pl + total + small.size
    assert done[0].error.kind == 0 and np.array_equal(wires[1].numpy(), wires[0].numpy())
    assert done[1].error.kind == 0 and done[1].frame_count == n
    assert np.array_equal(poss[1].numpy(), np.arange(n, dtype=np.int64) * (48 + pl))
    orc, oe, oh, of = O.decode_batch_slice_with(small, 0)
    assert done[2].error.kind == 0 == orc and np.array_equal(p_small.numpy().view(np.uint64), np.asarray(of, dtype=np.uint64))


def test_registrations_may_not_share_a_page(cx):
    """iggy_codec_host_register refuses a range whose pages meet a live registration's
    (the runtime pins whole pages: two objects over one page leave a dead mapping when
    either is undone); page-aligned neighbours register side by side, and
    the refused range registers once its neighbour is gone."""
    from iggy_amd.codec import CodecError, host_buffer
    raw = host_buffer(3 * 4096)
    a, b = raw[:5000], raw[5000:9000]   # b starts inside a's second page
    cx.host_register(a)
    try:
        with pytest.raises(CodecError) as ei:
            cx.host_register(b)
        assert ei.value.rc == abi.ERR_INVALID_ARGUMENT
        c, d = host_buffer(5000), host_buffer(100)
        cx.host_register(c)
        cx.host_register(d)
        cx.host_unregister(d)
        cx.host_unregister(c)
    finally:
        cx.host_unregister(a)
    cx.host_register(b)
    cx.host_unregister(b)

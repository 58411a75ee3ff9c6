"""GPU parity at the exact shapes of every BASELINE config, and the concurrency
cases the parity suite does not reach:

  C1  10 batches x 1 000 x 256 B: encode -> decode through the asynchronous slots,
      wire bytes and frame positions against the oracle;
  C4  262 144 x 1 KiB batches streamed back to back through encode_submit ->
      decode_submit on registered (pinned) host buffers, two batches in flight,
      wire bytes and positions byte-exact against the oracle;
  mixed co-residency: a C2-shape uniform decode (160 KiB of LDS per CU) on context A
      beside a C3-shape general decode on context B, both exact, no timeout;
  the general kernel on grids of fewer than 8 workgroups (the two-level barrier's
      ngrp = nwg branch);
  the producer's flush when every slot of the context is held by the caller
      (IGGY_ERR_BUSY, nothing lost, a retry after the slots drain is exact).
C2 and C3 at full size are in test_parity_gpu.py. Integer byte work: all exact."""
import ctypes
import threading

import numpy as np
import pytest

from iggy_amd import abi
from iggy_amd.torch_io import to_device, to_host
from iggy_amd.codec import raw_messages
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cx():
    from iggy_amd.codec import Codec
    c = Codec(0)
    yield c
    c.close()


def _soa(n, lo, hi, seed):
    """BASELINE.md input spec: ids two draws (non-zero), origin_ts = 1.7e15 + i, random payloads."""
    rng = np.random.default_rng(seed)
    pls = rng.integers(lo, hi + 1, size=n).astype(np.uint32)
    ids = rng.integers(1, 2**63, size=2 * n, dtype=np.uint64)
    ots = (1_700_000_000_000_000 + np.arange(n)).astype(np.uint64)
    pay = rng.integers(0, 256, size=int(pls.sum()), dtype=np.uint8)
    return dict(ids=ids, ots=ots, pay=pay, pls=pls)


def _raw(m):
    return raw_messages(m["ids"], m["ots"], m["pay"], m["pls"])


def _stream_encode_decode(cx, batches, in_flight):
    """Encode each SoA batch (encode_submit) into a registered wire buffer, then decode
    the wire bytes (decode_submit) into registered position buffers, `in_flight`
    batches deep; -> [(wire bytes, completion of the decode, positions)]."""
    from iggy_amd.codec import host_buffer
    outs = []
    for m in batches:
        n = len(m["pls"])
        need = 256 + 48 * n + int(m["pls"].sum())
        wire = host_buffer(need)  # (registrations may not share a page)
        pos = host_buffer(n, np.uint64)
        outs.append((wire, pos))
    for wire, pos in outs:
        cx.host_register(wire)
        cx.host_register(pos)
    try:
        raws = [_raw(m) for m in batches]
        enc = {}
        dec = {}
        results = [None] * len(batches)
        k_enc = k_dec = 0
        # encode k runs while decode k-1 runs; at most `in_flight` of each are queued
        while k_dec < len(batches):
            while k_enc < len(batches) and k_enc - k_dec < in_flight:
                enc[k_enc] = cx.encode_submit(raws[k_enc], 0, outs[k_enc][0])
                k_enc += 1
            c = cx.wait(enc.pop(k_dec))
            assert c.op == abi.OP_ENCODE and c.error.kind == 0, c.error
            assert c.bytes == outs[k_dec][0].size
            dec[k_dec] = cx.decode_submit(outs[k_dec][0], abi.INTEGRITY_VERIFY, outs[k_dec][1])
            if k_dec >= 1:
                results[k_dec - 1] = cx.wait(dec.pop(k_dec - 1))
            k_dec += 1
        results[-1] = cx.wait(dec.pop(len(batches) - 1))
        return [(outs[k][0].tobytes(), results[k], outs[k][1]) for k in range(len(batches))]
    finally:
        for wire, pos in outs:
            cx.host_unregister(wire)
            cx.host_unregister(pos)


def _check_stream(batches, got):
    for m, (wire, c, pos) in zip(batches, got):
        orc, oe, owire = O.encode_batch(_raw(m))
        assert orc == 0, oe
        assert wire == owire
        drc, de, dh, dframes = O.decode_batch_slice_with(np.frombuffer(owire, dtype=np.uint8), 0)
        assert drc == 0, de
        assert c.op == abi.OP_DECODE and c.error.kind == 0, c.error
        assert c.header.astuple() == dh.astuple() and c.frame_count == len(dframes)
        assert np.array_equal(pos, dframes)


def test_c1_ten_batches_encode_decode(cx):
    """C1 (core/bench producer batches, defaults.rs:33): 10 x 1 000 x 256 B."""
    batches = [_soa(1000, 256, 256, seed=0x16619E3779B97F4A ^ k) for k in range(10)]
    _check_stream(batches, _stream_encode_decode(cx, batches, in_flight=2))


def test_c4_exact_streamed_batches(cx):
    """C4: 262 144 x 1 KiB per batch, K = 4 batches back to back through the
    asynchronous slots (registered host buffers, encode of batch k beside the
    decode of batch k - 1), wire bytes and positions exact."""
    batches = [_soa(262_144, 1024, 1024, seed=0x16619E3779B97F4A ^ (0xC4 + k)) for k in range(4)]
    _check_stream(batches, _stream_encode_decode(cx, batches, in_flight=2))


def _torch():
    import torch
    return torch


def _res(t):
    return abi.DecodeResult.from_buffer_copy(to_host(t).tobytes())


def test_uniform_beside_general_two_contexts():
    """A C2-shape uniform decode (persistent grid, 160 KiB LDS per CU) on context A
    and a C3-shape general decode (grid barriers, 20-us membership close) on context
    B, on two streams from two host threads, several times over: the general
    kernel's barriers count only the workgroups that joined, the uniform grid never
    waits for residency, so both finish exact and neither times out."""
    torch = _torch()
    from iggy_amd.codec import Codec
    recs = [O.synth_batch(262_144, 1024, 1024, seed=51), O.synth_batch(120_000, 64, 4096, seed=52)]
    expect = [O.decode_batch_slice_with(r, 0) for r in recs]
    ctxs = [Codec(0), Codec(0)]
    errors = []
    paths = [1, 2]

    def run(k):
        try:
            s = torch.cuda.Stream()
            d = to_device(recs[k], "cuda:0")
            n = int(expect[k][2].message_count)
            pos = torch.zeros(n, dtype=torch.int64, device="cuda:0")
            res = [torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device="cuda:0")
                   for _ in range(8)]
            torch.cuda.synchronize()
            for it in range(8):
                assert ctxs[k].decode_device(d.data_ptr(), recs[k].size, 0, pos.data_ptr(), n, res[it].data_ptr(),
                                             s.cuda_stream) == 0
            s.synchronize()
            for it in range(8):
                got = _res(res[it])
                assert got.error.kind == 0, (k, it, got.error.kind)
                assert got.path == paths[k]
                assert got.computed_checksum == expect[k][2].batch_checksum
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


@pytest.mark.parametrize("n,lo,hi", [(40, 1000, 2500), (60, 1000, 3000), (100, 1500, 3000), (220, 1000, 2500),
                                     (400, 1500, 2000)])
def test_general_walk_small_grids(cx, n, lo, hi):
    """Variable frames in records of 70-700 KB: the general grid is one WG per 64 KiB
    (+2), so 3..12 workgroups: below and above the two-level barrier's 8 counters."""
    rec = O.synth_batch(n, lo, hi, seed=0x5A11 ^ n)
    for integ in (0, 1):
        rc, e, h, frames = cx.decode_batch_slice_with(rec, integ)
        orc, oe, oh, of = O.decode_batch_slice_with(rec, integ)
        assert rc == orc and e.astuple() == oe.astuple()
        assert rc == 0 and np.array_equal(frames, of)
    bad = rec.copy()
    bad[256 + rec.size // 2] ^= 0x40
    rc, e, _, _ = cx.decode_batch_slice_with(bad, 0)
    orc, oe, _, _ = O.decode_batch_slice_with(bad, 0)
    assert rc == orc and e.astuple() == oe.astuple()


def test_producer_flush_busy_keeps_buffer(cx):
    """Every asynchronous slot of the context held by the caller's own decode submits:
    the producer's flush returns IGGY_ERR_BUSY with no request written and the buffer
    intact; after the submits are retired the same flush is exact."""
    from iggy_amd.codec import Producer
    from oracle import sdk_ref as S
    rec = O.synth_batch(20_000, 1024, 1024, seed=61)
    tickets = [cx.decode_submit(rec, abi.INTEGRITY_VERIFY) for _ in range(8)]
    p = Producer(cx, batch_length=0, batch_size=0, direct=False)
    m = _soa(500, 0, 300, seed=62)
    st = (S.ID_NUMERIC, (1).to_bytes(4, "little"))
    tp = (S.ID_NUMERIC, (2).to_bytes(4, "little"))
    pt = (S.PART_BALANCED, b"")
    p.append(abi.Identifier.raw(*st), abi.Identifier.raw(*tp), abi.Partitioning.raw(*pt), _raw(m))
    before = p.pending()
    cap = 4096 + 48 * 500 + int(m["pls"].sum())
    rc, e, out, reqs = p.flush(cap=cap)
    assert rc == abi.ERR_BUSY and reqs == []
    assert p.pending() == before
    for t in tickets:
        assert cx.wait(t).error.kind == 0
    rc, e, out, reqs = p.flush(cap=cap)
    assert rc == 0 and len(reqs) == 1 and reqs[0].sent == 1 and reqs[0].error.kind == 0
    orc, oe, batch = O.encode_batch(_raw(m))
    assert orc == 0
    r = reqs[0]
    assert out.tobytes()[r.offset:r.offset + r.length] == S.send_messages_body(st, tp, pt, batch, 500)
    assert p.pending()[:2] == (0, 0)
    p.close()


def test_producer_flush_reused_reqs_after_busy(cx):
    """A caller reusing one request array across flushes: a flush that
    writes two requests, then one that hits BUSY on its first submit, must report no
    request and leave no stale `sent` flag in the array; the buffer stays intact and the
    retried flush is exact."""
    from iggy_amd.abi import ProducerRequest
    from iggy_amd.codec import Producer
    from oracle import sdk_ref as S
    p = Producer(cx, batch_length=0, batch_size=0, direct=False)
    st = (S.ID_NUMERIC, (1).to_bytes(4, "little"))
    tps = [(S.ID_NUMERIC, (k).to_bytes(4, "little")) for k in (2, 3)]
    pt = (S.PART_BALANCED, b"")
    reqs = (ProducerRequest * 16)()
    ms = [_soa(300, 0, 200, seed=70 + k) for k in range(2)]
    for tp, m in zip(tps, ms):
        p.append(abi.Identifier.raw(*st), abi.Identifier.raw(*tp), abi.Partitioning.raw(*pt), _raw(m))
    cap = 8192 + sum(48 * 300 + int(m["pls"].sum()) for m in ms)
    rc, e, out, got = p.flush(cap=cap, max_reqs=16, reqs=reqs)
    assert rc == 0 and len(got) == 2 and all(r.sent == 1 for r in got)
    ms2 = [_soa(200, 0, 100, seed=80 + k) for k in range(2)]
    for tp, m in zip(tps, ms2):
        p.append(abi.Identifier.raw(*st), abi.Identifier.raw(*tp), abi.Partitioning.raw(*pt), _raw(m))
    before = p.pending()
    rec = O.synth_batch(20_000, 1024, 1024, seed=61)
    tickets = [cx.decode_submit(rec, abi.INTEGRITY_VERIFY) for _ in range(8)]
    rc, e, out, got = p.flush(cap=cap, max_reqs=16, reqs=reqs)
    assert rc == abi.ERR_BUSY and got == []
    assert reqs[0].sent == 0 and reqs[1].sent == 0
    assert p.pending() == before
    for t in tickets:
        assert cx.wait(t).error.kind == 0
    rc, e, out, got = p.flush(cap=cap, max_reqs=16, reqs=reqs)
    assert rc == 0 and len(got) == 2
    for r, tp, m in zip(got, tps, ms2):
        orc, oe, batch = O.encode_batch(_raw(m))
        assert r.sent == 1 and r.error.kind == 0
        assert out.tobytes()[r.offset:r.offset + r.length] == S.send_messages_body(st, tp, pt, batch, 200)
    p.close()

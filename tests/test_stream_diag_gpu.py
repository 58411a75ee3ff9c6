"""GPU parity of the streamed variable-size decode (decode_stream.hip, the
diagnostic build's dbg bit 0x200000: a next-round candidate, not the product
path) against the oracle: the record shapes and corruptions of
tests/test_stream_model_cpu.py (which checks the same algorithm on the CPU), a
full C3 record, frames longer than the LDS window's overhang (one-lane global
hashing), tiny and empty walks, stride breaks. Run explicitly:
    python -m pytest tests/test_stream_diag_gpu.py -m gpu_diag
Byte work: all exact."""
import os
import struct

import numpy as np
import pytest

from iggy_amd import abi
from oracle import oracle as O

pytestmark = [pytest.mark.gpu_diag,
              pytest.mark.skipif(not __import__("torch").cuda.is_available(), reason="needs a GPU")]


@pytest.fixture(scope="module")
def dx():
    from iggy_amd.codec import DIAG_LIB_PATH, Codec, load
    os.environ["IGGY_CODEC_DBG"] = str(0x200000)
    try:
        c = Codec(0, library=load(DIAG_LIB_PATH))
    finally:
        del os.environ["IGGY_CODEC_DBG"]
    yield c
    c.close()


def _same(dx, rec):
    for integ in (abi.INTEGRITY_VERIFY, abi.INTEGRITY_LAYOUT_ONLY):
        rc, e, h, frames = dx.decode_batch_slice_with(rec, integ)
        orc, oe, oh, of = O.decode_batch_slice_with(rec, integ)
        assert rc == orc and e.astuple() == oe.astuple(), (e.astuple(), oe.astuple())
        if rc == 0:
            assert h.astuple() == oh.astuple() and np.array_equal(frames, of)


@pytest.mark.parametrize("n,lo,hi,seed", [(300, 64, 4096, 1), (20000, 64, 512, 2), (6000, 1000, 3000, 3),
                                          (400, 5000, 20000, 4), (30, 0, 200, 5), (25, 0, 0, 6), (3, 10, 90, 7)])
def test_shapes(dx, n, lo, hi, seed):
    _same(dx, O.synth_batch(n, lo, hi, seed=seed))


def test_c3_record(dx):
    _same(dx, O.synth_batch(1 << 20, 64, 4096, seed=0xC3))


@pytest.mark.parametrize("seed", range(4))
def test_corruptions(dx, seed):
    rec = O.synth_batch(8000, 64, 2048, seed=40 + seed)
    ok, e0, h0, frames = O.decode_batch_slice_with(rec, 0)
    assert ok == 0
    st = [int(x) for x in frames]
    rng = np.random.default_rng(seed)
    cases = []
    b = rec.copy(); b[256 + st[5000] + 100] ^= 4; cases.append(b)
    b = rec.copy(); b[256 + st[3] + 2] ^= 1; cases.append(b)
    b = rec.copy(); b[40] ^= 0x10; cases.append(b)
    b = rec.copy(); b[256 + st[4000] + 41] = 7; cases.append(b)
    b = rec.copy(); struct.pack_into("<I", b, 48, 7999); cases.append(b)
    b = rec.copy(); struct.pack_into("<I", b, 256 + st[2500] + 36, struct.unpack_from("<I", b, 256 + st[2500] + 36)[0] + 8)
    cases.append(b)
    b = rec.copy(); b[256 + st[7000] + 100] ^= 2; b[256 + st[1000] + 44] = 1; cases.append(b)
    k = int(rng.integers(10, 7990))
    b = rec.copy(); b[256 + st[k] + 60] ^= 0x80; cases.append(b)
    b = rec.copy(); b[256 + st[-1] + 60] ^= 0x80; cases.append(b)  # the last frame
    for c in cases:
        _same(dx, c)


def test_fake_headers_in_payloads(dx):
    rng = np.random.default_rng(9)
    n = 4000
    pls = rng.integers(100, 1500, size=n).astype(np.uint32)
    ids = rng.integers(1, 2**63, size=2 * n, dtype=np.uint64)
    ots = (1_700_000_000_000_000 + np.arange(n)).astype(np.uint64)
    pay = np.zeros(int(pls.sum()), dtype=np.uint8)
    for p in range(0, pay.size - 48, 97):
        struct.pack_into("<II", pay, p + 32, int(rng.integers(0, 60)), 0)
    from iggy_amd.codec import raw_messages
    rc, e, out = O.encode_batch(raw_messages(ids, ots, pay, pls), 1)
    assert rc == 0
    _same(dx, np.frombuffer(out, dtype=np.uint8).copy())


def test_stride_break_goes_general(dx):
    pls = [1024] * 5000
    pls[2500] -= 8
    pls[2501] += 8
    rng = np.random.default_rng(3)
    n = len(pls)
    ids = rng.integers(1, 2**63, size=2 * n, dtype=np.uint64)
    ots = (1_700_000_000_000_000 + np.arange(n)).astype(np.uint64)
    pay = rng.integers(0, 256, size=sum(pls), dtype=np.uint8)
    from iggy_amd.codec import raw_messages
    rc, e, out = O.encode_batch(raw_messages(ids, ots, pay, np.asarray(pls, dtype=np.uint32)), 1)
    assert rc == 0
    _same(dx, np.frombuffer(out, dtype=np.uint8).copy())

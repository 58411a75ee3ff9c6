"""CPU check of the streamed variable-size decode's algorithm (scripts/stream_model.py,
the design model of the next general-decode kernel) against the oracle: tiles in
any order with speculative entries (some deliberately wrong), group summaries by
the last finisher, the link fed partial ready prefixes, deferred scatter and
batch-checksum words counted per block in any order, the chain over full blocks
only, the finisher's partial block and last stripe. Same verdicts, positions and
error payloads as decode_batch_slice_with (batch.rs:391-527) on clean records and
on every kind of corruption. No GPU, no product code."""
import os
import struct
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
import stream_model as SM  # noqa: E402
from oracle import oracle as O  # noqa: E402


def _check(body, verify=True, **kw):
    integ = 0 if verify else 1
    rc, e, h, frames = O.decode_batch_slice_with(body, integ)
    kind, reason, fpos, computed, abc = SM.decode(bytes(body), verify=verify, **kw)
    assert (kind, reason) == (e.kind, e.reason), (kind, reason, e.astuple())
    if kind == SM.OK:
        assert [int(x) for x in frames] == fpos
        if verify:
            assert computed == h.batch_checksum
    elif kind in (SM.MSG_CS, SM.BATCH_CS):
        assert abc == (e.a, e.b, e.c)


SHAPES = [(300, 64, 4096, 1), (2000, 64, 512, 2), (600, 1000, 3000, 3), (40, 5000, 9000, 4), (30, 0, 200, 5),
          (1200, 200, 200, 6)]


@pytest.mark.parametrize("n,lo,hi,seed", SHAPES)
@pytest.mark.parametrize("T", [512, 4096])
def test_clean_records(n, lo, hi, seed, T):
    rec = O.synth_batch(n, lo, hi, seed=seed)
    for verify in (True, False):
        _check(rec, verify, T=T, seed=seed)
    _check(rec, True, T=T, seed=seed + 100, adversarial_picks=True, starve=True)


@pytest.mark.parametrize("seed", range(6))
def test_corruptions(seed):
    rng = np.random.default_rng(seed)
    rec = O.synth_batch(800, 64, 2048, seed=40 + seed)
    bl = int(struct.unpack_from("<Q", rec, 32)[0])
    ok, e0, h0, frames = O.decode_batch_slice_with(rec, 0)
    assert ok == 0
    starts = [int(x) for x in frames]
    cases = []
    b = rec.copy(); b[256 + starts[500] + 100] ^= 4; cases.append(b)                      # payload: message checksum
    b = rec.copy(); b[256 + starts[3] + 2] ^= 1; cases.append(b)                          # a stored checksum
    b = rec.copy(); b[40] ^= 0x10; cases.append(b)                                        # the batch checksum field
    b = rec.copy(); b[256 + starts[400] + 41] = 7; cases.append(b)                        # frame reserved: walk stops
    b = rec.copy(); struct.pack_into("<I", b, 48, 799); cases.append(b)                   # count off by one
    b = rec.copy(); struct.pack_into("<I", b, 256 + starts[250] + 36,
                                     struct.unpack_from("<I", b, 256 + starts[250] + 36)[0] + 8)
    cases.append(b)                                                                       # a length: the walk re-tiles
    b = rec.copy(); b[256 + starts[700] + 100] ^= 2; b[256 + starts[100] + 44] = 1; cases.append(b)  # two breaks
    k = int(rng.integers(10, 790))
    b = rec.copy(); b[256 + starts[k] + 60] ^= 0x80; cases.append(b)
    for i, c in enumerate(cases):
        for verify in (True, False):
            _check(c, verify, T=1024, seed=seed * 10 + i, adversarial_picks=(i % 2 == 0), starve=(i % 3 == 0))
    assert bl == rec.size


def test_fake_headers_in_payloads():
    """payloads full of zero runs and header-like bytes: many false candidates, the
    picks go wrong and the link repairs tiles"""
    rng = np.random.default_rng(9)
    n = 400
    pls = rng.integers(100, 1500, size=n).astype(np.uint32)
    ids = rng.integers(1, 2**63, size=2 * n, dtype=np.uint64)
    ots = (1_700_000_000_000_000 + np.arange(n)).astype(np.uint64)
    pay = np.zeros(int(pls.sum()), dtype=np.uint8)
    # fake 48-B headers with small plausible lengths every ~97 bytes
    for p in range(0, pay.size - 48, 97):
        struct.pack_into("<II", pay, p + 32, int(rng.integers(0, 60)), 0)
    from iggy_amd.codec import raw_messages
    rc, e, out = O.encode_batch(raw_messages(ids, ots, pay, pls), 1)
    assert rc == 0
    rec = np.frombuffer(out, dtype=np.uint8).copy()
    for T in (256, 2048):
        _check(rec, True, T=T, seed=T)
        _check(rec, True, T=T, seed=T + 1, adversarial_picks=True, starve=True)
        _check(rec, False, T=T, seed=T + 2)

"""GPU parity of the poll reply body (iggy_codec_build_polled_body,
build_polled_messages_body, core/server/src/responses.rs:1666-1714) against
oracle/sdk_ref.build_polled_messages_body: a disk chunk's walk fragments (whole
records and rewritten-header slices) served plain, encrypted records decrypted on the
GPU (decrypt_batch_record, server_common/src/send_messages.rs:364-415), and every
error the reference raises in its record order. Byte work: exact."""
import struct

import numpy as np
import pytest

from crypt_util import key_for, nonces_for, raw_record
from golden_util import reference_vectors
from iggy_amd import abi
from oracle import oracle as O
from oracle import sdk_ref as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cx():
    from iggy_amd.codec import Codec
    c = Codec(0)
    yield c
    c.close()


def _same(cx, pid, off, frags, key=None, cap=None):
    rc, e, body = cx.build_polled_body(pid, off, frags, key, cap)
    orc, oe, obody = S.build_polled_messages_body(pid, off, frags, key)
    assert rc == orc, (e, oe)
    if rc == 0:
        assert body == obody
    else:
        assert (e.kind, e.a, e.b) == (oe[0], oe[2], oe[3]) or e.kind == oe[0] == abi.ERR_INVALID_COMMAND
    return rc, body


def _chunk(shapes, base_offset=1000, seed=5):
    recs, off = [], base_offset
    for k, (n, lo, hi) in enumerate(shapes):
        r = O.synth_batch(n, lo, hi, 0, seed=seed * 100 + k)
        rc, e, h, out = O.stamp_batch(r, off, 5000 + 10 * k)
        recs.append(np.frombuffer(out, dtype=np.uint8).copy())
        off += n
    return np.concatenate(recs)


def _fragments(chunk, frags, headers):
    out = []
    for f, h in zip(frags, headers):
        if f.full_body:
            out.append(chunk[f.body_start: f.body_end].tobytes())
        else:
            out.append(h)
            out.append(chunk[f.body_start: f.body_end].tobytes())
    return out


def test_golden_poll_body(cx):
    body = bytes.fromhex(reference_vectors()["poll_body_hex"])
    pid, off, _ = struct.unpack_from("<IQI", body, 0)
    rc, got = _same(cx, pid, off, [body[16:300], body[300:]])
    assert rc == 0 and got == body


@pytest.mark.parametrize("q", [(abi.LOOKUP_OFFSET, 1000, 10**6), (abi.LOOKUP_OFFSET, 1030, 2000),
                               (abi.LOOKUP_OFFSET, 3500, 100), (abi.LOOKUP_TIMESTAMP, 5010, 500)])
def test_chunk_walk_fragments_plain(cx, q):
    chunk = _chunk([(40, 10, 900), (3000, 1024, 1024), (1, 5, 5), (700, 0, 3000)])
    kind, value, count = q
    rc, w, frags, hdrs = O.walk_disk_chunk(chunk, kind, value, count)
    assert rc == 0 and frags
    _same(cx, 3, 9999, _fragments(chunk, frags, hdrs))


def _sealed(n, lo, hi, uh, seed):
    raw = raw_record(n, lo, hi, seed=seed, uh_max=uh)
    rc, e, enc = O.encrypt_batch(key_for(seed), raw, nonces_for(n, seed))
    assert rc == 0
    return raw, enc


def test_encrypted_records_decrypted(cx):
    key = key_for(31)
    recs, plain = [], []
    for k, (n, lo, hi, uh) in enumerate([(5, 0, 17, 0), (300, 10, 2000, 40), (1, 3000, 3000, 0), (2000, 64, 4096, 20)]):
        raw = raw_record(n, lo, hi, seed=200 + k, uh_max=uh)
        rc, e, enc = O.encrypt_batch(key, raw, nonces_for(n, 300 + k))
        recs.append(enc)
        plain.append(raw.tobytes())
    rc, body = _same(cx, 1, 77, recs, key)
    assert rc == 0 and body[16:] == b"".join(plain)
    # fragments that split records anywhere
    stream = b"".join(recs)
    cuts = [0, 100, 255, 256, 9000, len(stream) - 7, len(stream)]
    _same(cx, 1, 77, [stream[a:b] for a, b in zip(cuts, cuts[1:])], key)


def test_errors_in_record_order(cx):
    key = key_for(41)
    recs = []
    for k in range(3):
        raw = raw_record(50, 10, 500, seed=400 + k, uh_max=30)
        rc, e, enc = O.encrypt_batch(key, raw, nonces_for(50, 500 + k))
        recs.append(bytearray(enc))
    # wrong key: the first record's first section
    _same(cx, 1, 2, [bytes(r) for r in recs], key_for(42))
    # a flipped ciphertext byte in record 1 and a bad header in record 2: the decrypt
    # error of record 1 comes first
    bad1 = bytearray(recs[1]); bad1[256 + 48 + 20] ^= 1
    bad2 = bytearray(recs[2]); bad2[60] = 9
    rc, _ = _same(cx, 1, 2, [bytes(recs[0]), bytes(bad1), bytes(bad2)], key)
    assert rc == abi.ERR_CANNOT_DECRYPT_DATA
    rc, _ = _same(cx, 1, 2, [bytes(recs[0]), bytes(recs[1]), bytes(bad2)], key)
    assert rc == abi.ERR_INVALID_COMMAND
    # truncated last record, plain and decrypting
    for k in (None, key):
        rc, _ = _same(cx, 1, 2, [bytes(recs[0]), bytes(recs[1][:-3])], k)
        assert rc == abi.ERR_INVALID_COMMAND
    # a record whose frames do not tile (layout-only decode inside the decrypt)
    bad = bytearray(recs[0]); struct.pack_into("<I", bad, 48, 49)
    rc, _ = _same(cx, 1, 2, [bytes(bad)], key)
    assert rc == abi.ERR_INVALID_COMMAND
    # count overflow: served plain (headers only), then with the decrypt in front of it
    big = bytearray(_chunk([(3, 10, 10)])); struct.pack_into("<I", big, 48, 0xFFFFFFFE)
    rc, _ = _same(cx, 1, 2, [bytes(big), _chunk([(3, 10, 10)]).tobytes()])
    assert rc == abi.ERR_INVALID_COMMAND


def test_empty_and_capacity(cx):
    rc, body = _same(cx, 9, 123, [])
    assert rc == 0 and body == struct.pack("<IQI", 9, 123, 0)
    chunk = _chunk([(10, 100, 100)])
    rc, e, body = cx.build_polled_body(1, 1, [chunk], None, cap=16 + chunk.size - 1)
    assert rc == abi.ERR_CAPACITY and e.a == 16 + chunk.size

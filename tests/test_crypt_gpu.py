"""GPU parity of the at-rest encryption re-encode (iggy_codec_encrypt_batch_device /
iggy_codec_decrypt_batch_device; encrypt_batch_request / decrypt_batch_record,
core/server_common/src/send_messages.rs:293-415) against the CPU oracle: byte-exact
records (AES-256-GCM sections, restamped lengths, per-message and batch checksums),
the error precedence, and a full C2-shaped round trip. Integer/byte work: bit-exact."""
import ctypes

import numpy as np
import pytest

from crypt_util import frame_sections, key_for, nonces_for, raw_record
from iggy_amd import abi
from iggy_amd.torch_io import to_host
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cx():
    from iggy_amd.codec import Codec
    c = Codec(0)
    yield c
    c.close()


def _dev(a):
    """A plain pageable torch copy, on purpose: the module where round 5's fault surfaced
    runs the runtime's pageable path again, now that the suite's registrations no longer
    share pages; the other modules copy through pinned staging."""
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


def _run(cx, enc: bool, key, rec, nonces=None, cap=None, length=None):
    import torch
    d_rec = _dev(rec)
    n = rec.size // 48 + 1
    cap = cap if cap is not None else rec.size + 56 * n + 256
    d_out = torch.zeros(max(cap, 1), dtype=torch.uint8, device="cuda")
    d_res = torch.zeros(ctypes.sizeof(abi.CryptResult), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()
    ln = rec.size if length is None else length
    if enc:
        d_non = _dev(nonces)
        rc = cx.encrypt_batch_device(key, d_rec.data_ptr(), ln, d_non.data_ptr(), d_out.data_ptr(), cap,
                                     d_res.data_ptr(), s)
    else:
        rc = cx.decrypt_batch_device(key, d_rec.data_ptr(), ln, d_out.data_ptr(), cap, d_res.data_ptr(), s)
    assert rc == 0
    torch.cuda.synchronize()
    r = abi.CryptResult.from_buffer_copy(to_host(d_res).tobytes())
    out = to_host(d_out)[: r.out_len].tobytes() if r.error.kind == 0 else b""
    return r, out


CASES = [(1, 0, 0, 0), (5, 0, 17, 0), (33, 1, 300, 60), (300, 900, 1100, 0), (130, 4000, 4096, 100),
         (2000, 64, 4096, 20), (1000, 1024, 1024, 0)]


@pytest.mark.parametrize("n,lo,hi,uh", CASES)
def test_encrypt_matches_oracle(cx, n, lo, hi, uh):
    rec = raw_record(n, lo, hi, seed=7 * n + hi, uh_max=uh)
    key, nonces = key_for(n + 1), nonces_for(n, n + 2)
    rc, e, want = O.encrypt_batch(key, rec, nonces)
    assert rc == 0, e.astuple()
    r, got = _run(cx, True, key, rec, nonces)
    assert r.error.kind == 0, r.error.astuple()
    assert r.out_len == len(want) and r.frame_count == n
    assert got == want
    assert r.batch_checksum == int(np.frombuffer(want[40:48], dtype=np.uint64)[0])


@pytest.mark.parametrize("n,lo,hi,uh", CASES)
def test_decrypt_matches_oracle(cx, n, lo, hi, uh):
    rec = raw_record(n, lo, hi, seed=11 * n + lo, uh_max=uh)
    key, nonces = key_for(n + 3), nonces_for(n, n + 4)
    rc, e, enc = O.encrypt_batch(key, rec, nonces)
    assert rc == 0
    encb = np.frombuffer(enc, dtype=np.uint8).copy()
    r, got = _run(cx, False, key, encb)
    assert r.error.kind == 0, r.error.astuple()
    assert got == rec.tobytes()


def test_key_change_between_calls(cx):
    rec = raw_record(40, 10, 500, seed=3, uh_max=30)
    nonces = nonces_for(40, 3)
    for k in (key_for(1), key_for(2), key_for(1)):
        rc, e, want = O.encrypt_batch(k, rec, nonces)
        r, got = _run(cx, True, k, rec, nonces)
        assert got == want


def test_decrypt_errors_match_oracle(cx):
    rec = raw_record(300, 10, 2000, seed=21, uh_max=80)
    key, nonces = key_for(21), nonces_for(300, 21)
    rc, e, enc = O.encrypt_batch(key, rec, nonces)
    encb = np.frombuffer(enc, dtype=np.uint8).copy()
    secs = frame_sections(encb)
    cases = []
    for fr, sec in ((250, 0), (17, 1), (299, 0)):
        bad = encb.copy()
        off, ln = (secs[fr][0], secs[fr][1]) if sec == 0 else (secs[fr][2], secs[fr][3])
        if ln == 0:
            continue
        bad[off + ln - 5] ^= 0x10
        cases.append(bad)
    # two bad frames: the first one wins
    two = encb.copy()
    two[secs[200][0] + 20] ^= 1
    two[secs[40][0] + 13] ^= 1
    cases.append(two)
    for bad in cases:
        rc, e, _ = O.decrypt_batch(key, bad)
        r, _ = _run(cx, False, key, bad)
        assert (r.error.kind, r.error.a, r.error.b) == (rc, e.a, e.b)
    # wrong key, trailing bytes, plaintext input, capacity
    rc, e, _ = O.decrypt_batch(bytes(32), encb)
    r, _ = _run(cx, False, bytes(32), encb)
    assert (r.error.kind, r.error.a) == (rc, e.a) == (abi.ERR_CANNOT_DECRYPT_DATA, 0)
    longer = np.concatenate([encb, np.zeros(16, dtype=np.uint8)])
    r, _ = _run(cx, False, key, longer)
    assert r.error.kind == abi.ERR_INVALID_COMMAND
    r, _ = _run(cx, False, key, rec)
    rc, e, _ = O.decrypt_batch(key, rec)
    assert (r.error.kind, r.error.a) == (rc, e.a)
    r, _ = _run(cx, False, key, encb, cap=len(rec) - 1)
    assert r.error.kind == abi.ERR_CAPACITY and r.error.a == len(rec)


def test_encrypt_errors(cx):
    rec = raw_record(100, 100, 300, seed=4)
    bad = rec.copy()
    bad[256 + 48 + 5] ^= 1
    rc, e, _ = O.encrypt_batch(key_for(4), bad, nonces_for(100, 4))
    r, _ = _run(cx, True, key_for(4), bad, nonces_for(100, 4))
    assert rc == abi.ERR_INVALID_MESSAGE_CHECKSUM
    assert r.error.astuple() == e.astuple()
    need = len(rec) + 28 * 100
    r, _ = _run(cx, True, key_for(4), rec, nonces_for(100, 4), cap=need - 1)
    assert r.error.kind == abi.ERR_CAPACITY and r.error.a == need
    r, out = _run(cx, True, key_for(4), rec, nonces_for(100, 4), cap=need)
    assert r.error.kind == 0 and len(out) == need


def test_full_size_c2_round_trip(cx):
    """1 M x 1 KiB (C2 shape): decrypt(encrypt(x)) == x on the device, the encrypted
    record Verify-decodes, and sampled sections equal the oracle's."""
    import torch
    n = 1 << 20
    rec = O.synth_batch(n, 1024, 1024, seed=0x16619E3779B97F4A)
    key = key_for(77)
    nonces = nonces_for(n, 77)
    d_rec = _dev(rec)
    d_non = _dev(nonces)
    cap = rec.size + 28 * n + 256
    d_enc = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    d_res = torch.zeros(ctypes.sizeof(abi.CryptResult), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()
    assert cx.encrypt_batch_device(key, d_rec.data_ptr(), rec.size, d_non.data_ptr(), d_enc.data_ptr(), cap,
                                   d_res.data_ptr(), s) == 0
    torch.cuda.synchronize()
    r = abi.CryptResult.from_buffer_copy(to_host(d_res).tobytes())
    assert r.error.kind == 0 and r.out_len == rec.size + 28 * n and r.frame_count == n
    d_pos = torch.zeros(n, dtype=torch.int64, device="cuda")
    d_dres = torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device="cuda")
    assert cx.decode_device(d_enc.data_ptr(), r.out_len, abi.INTEGRITY_VERIFY, d_pos.data_ptr(), n,
                            d_dres.data_ptr(), s) == 0
    torch.cuda.synchronize()
    dr = abi.DecodeResult.from_buffer_copy(to_host(d_dres).tobytes())
    assert dr.error.kind == 0 and dr.frame_count == n
    enc = to_host(d_enc[: r.out_len])
    for i in (0, 1, 4095, 524287, n - 1):  # frames: 1100 B encrypted, 1072 B plain
        f_in, f_out = 256 + 1072 * i, 256 + 1100 * i
        assert enc[f_out + 48: f_out + 48 + 1052].tobytes() == O.gcm_seal(
            key, nonces[24 * i: 24 * i + 12].tobytes(), rec[f_in + 48: f_in + 48 + 1024].tobytes())
    d_dec = torch.zeros(rec.size, dtype=torch.uint8, device="cuda")
    assert cx.decrypt_batch_device(key, d_enc.data_ptr(), r.out_len, d_dec.data_ptr(), rec.size,
                                   d_res.data_ptr(), s) == 0
    torch.cuda.synchronize()
    r2 = abi.CryptResult.from_buffer_copy(to_host(d_res).tobytes())
    assert r2.error.kind == 0 and r2.out_len == rec.size
    assert torch.equal(d_dec, d_rec)

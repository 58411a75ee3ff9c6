"""CPU tests of the at-rest encryption oracle (oracle/crypt_ref.c): AES-256-GCM
against the GCM spec's AES-256 test cases and the OpenSSL-generated fixtures
(tests/golden/crypt_gcm.json), then the batch re-encodes
encrypt_batch_request / decrypt_batch_record
(core/server_common/src/send_messages.rs:293-415): round trips, frame layout and
the error cases (crypto.rs:80-90 CannotDecryptData, the exact-length check)."""
import json
import os

import numpy as np
import pytest

from crypt_util import frame_sections, key_for, nonces_for, raw_record
from iggy_amd import abi
from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))


def test_gcm_spec_test_cases_13_14():
    # McGrew & Viega, "The Galois/Counter Mode of Operation", AES-256 test cases 13 and 14
    assert O.gcm_seal(bytes(32), bytes(12), b"").hex() == "00" * 12 + "530f8afbc74536b9a963b4f1c4cb738b"
    assert O.gcm_seal(bytes(32), bytes(12), bytes(16)).hex() == (
        "00" * 12 + "cea7403d4d606b6e074ec5d3baf39d18" + "d0d1c8a799996bf0265b98b5d48ab919")


def test_gcm_matches_openssl_fixtures():
    cases = json.load(open(os.path.join(HERE, "golden", "crypt_gcm.json")))["cases"]
    assert len(cases) >= 20
    for c in cases:
        key, nonce, pt = bytes.fromhex(c["key"]), bytes.fromhex(c["nonce"]), bytes.fromhex(c["plaintext"])
        sealed = O.gcm_seal(key, nonce, pt)
        assert sealed.hex() == c["sealed"], len(pt)
        assert O.gcm_open(key, sealed) == pt
        bad = bytearray(sealed)
        bad[len(bad) // 2] ^= 0x40
        assert O.gcm_open(key, bytes(bad)) is None
    assert O.gcm_open(bytes(32), bytes(27)) is None  # shorter than nonce + tag


@pytest.mark.parametrize("n,lo,hi,uh", [(1, 0, 0, 0), (7, 0, 40, 0), (50, 1, 300, 60), (200, 900, 1100, 0),
                                        (64, 4000, 4096, 30)])
def test_encrypt_decrypt_round_trip(n, lo, hi, uh):
    rec = raw_record(n, lo, hi, seed=n * 31 + hi, uh_max=uh)
    key, nonces = key_for(n), nonces_for(n, n)
    rc, e, enc = O.encrypt_batch(key, rec, nonces)
    assert rc == 0, e.astuple()
    encb = np.frombuffer(enc, dtype=np.uint8)
    # the encrypted record is a valid record: Verify decode passes
    rc2, e2, h2, _ = O.decode_batch_slice_with(encb, abi.INTEGRITY_VERIFY)
    assert rc2 == 0, e2.astuple()
    rc0, _, h0, _ = O.decode_batch_slice_with(rec, abi.INTEGRITY_VERIFY)
    assert (h2.partition_id, h2.base_offset, h2.base_timestamp, h2.origin_timestamp, h2.message_count) == (
        h0.partition_id, h0.base_offset, h0.base_timestamp, h0.origin_timestamp, h0.message_count)
    # every section is nonce || AES-256-GCM || tag under its own nonce
    src, dst = frame_sections(rec), frame_sections(encb)
    for i, ((sp, spl, su, suh), (dp, dpl, du, duh)) in enumerate(zip(src, dst)):
        assert dpl == spl + 28 and duh == (suh + 28 if suh else 0)
        assert enc[dp: dp + dpl] == O.gcm_seal(key, nonces[24 * i: 24 * i + 12].tobytes(), rec[sp: sp + spl].tobytes())
        if suh:
            assert enc[du: du + duh] == O.gcm_seal(key, nonces[24 * i + 12: 24 * i + 24].tobytes(),
                                                  rec[su: su + suh].tobytes())
    rc3, e3, dec = O.decrypt_batch(key, encb)
    assert rc3 == 0, e3.astuple()
    assert dec == rec.tobytes()  # decrypt(encrypt(x)) == x, header and checksums included


def test_decrypt_errors():
    rec = raw_record(20, 10, 200, seed=5, uh_max=50)
    key, nonces = key_for(5), nonces_for(20, 5)
    rc, e, enc = O.encrypt_batch(key, rec, nonces)
    assert rc == 0
    encb = np.frombuffer(enc, dtype=np.uint8).copy()
    secs = frame_sections(encb)
    # a tampered tag in frame 13's payload -> CannotDecryptData at frame 13
    bad = encb.copy()
    bad[secs[13][0] + secs[13][1] - 1] ^= 1
    rc, e, _ = O.decrypt_batch(key, bad)
    assert rc == abi.ERR_CANNOT_DECRYPT_DATA and (e.a, e.b) == (13, 0)
    # the wrong key fails on frame 0
    rc, e, _ = O.decrypt_batch(bytes(32), encb)
    assert rc == abi.ERR_CANNOT_DECRYPT_DATA and e.a == 0
    # trailing bytes: decrypt_batch_record needs record.len() == total_size()
    longer = np.concatenate([encb, np.zeros(8, dtype=np.uint8)])
    rc, e, _ = O.decrypt_batch(key, longer)
    assert rc == abi.ERR_INVALID_COMMAND
    # a plaintext record (sections shorter than nonce + tag exist) fails to decrypt
    tiny = raw_record(3, 0, 5, seed=9)
    rc, e, _ = O.decrypt_batch(key, tiny)
    assert rc == abi.ERR_CANNOT_DECRYPT_DATA and e.a == 0


def test_encrypt_verifies_input():
    rec = raw_record(10, 100, 200, seed=8)
    bad = rec.copy()
    bad[256 + 60] ^= 1  # a payload byte of frame 0: message checksum mismatch
    rc, e, _ = O.encrypt_batch(key_for(1), bad, nonces_for(10, 1))
    assert rc == abi.ERR_INVALID_MESSAGE_CHECKSUM

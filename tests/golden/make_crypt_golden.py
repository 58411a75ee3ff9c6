"""Generate tests/golden/crypt_gcm.json: AES-256-GCM sections sealed by the system
OpenSSL (libcrypto EVP_aes_256_gcm, 96-bit IV, empty AAD, 16-B tag) in the
Aes256GcmEncryptor layout nonce || ciphertext || tag
(core/common/src/utils/crypto.rs:70-78). The reference's `aes-gcm` crate is not in
/root/reference; OpenSSL implements the same NIST SP 800-38D algorithm. Run once
here; the JSON is the committed fixture (the GPU box needs no libcrypto).

usage: python tests/golden/make_crypt_golden.py
"""
import ctypes
import json
import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))


def ossl_seal(L, key: bytes, iv: bytes, pt: bytes) -> bytes:
    c = L.EVP_CIPHER_CTX_new()
    assert L.EVP_EncryptInit_ex(ctypes.c_void_p(c), ctypes.c_void_p(L.EVP_aes_256_gcm()), None, key, iv) == 1
    out = ctypes.create_string_buffer(len(pt) + 16)
    ol = ctypes.c_int(0)
    if pt:
        assert L.EVP_EncryptUpdate(ctypes.c_void_p(c), out, ctypes.byref(ol), pt, len(pt)) == 1
    fl = ctypes.c_int(0)
    assert L.EVP_EncryptFinal_ex(ctypes.c_void_p(c), ctypes.byref(out, ol.value), ctypes.byref(fl)) == 1
    tag = ctypes.create_string_buffer(16)
    assert L.EVP_CIPHER_CTX_ctrl(ctypes.c_void_p(c), 0x10, 16, tag) == 1  # EVP_CTRL_GCM_GET_TAG
    L.EVP_CIPHER_CTX_free(ctypes.c_void_p(c))
    return iv + out.raw[: len(pt)] + tag.raw


def main():
    L = ctypes.CDLL("libcrypto.so.3")
    L.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
    L.EVP_aes_256_gcm.restype = ctypes.c_void_p
    r = random.Random(0x1661)
    cases = []
    for n in [0, 1, 12, 15, 16, 17, 31, 32, 33, 63, 64, 65, 100, 255, 256, 1000, 1023, 1024, 1025, 1040, 4096, 4111]:
        key = bytes(r.randrange(256) for _ in range(32))
        iv = bytes(r.randrange(256) for _ in range(12))
        pt = bytes(r.randrange(256) for _ in range(n))
        cases.append({"key": key.hex(), "nonce": iv.hex(), "plaintext": pt.hex(), "sealed": ossl_seal(L, key, iv, pt).hex()})
    with open(os.path.join(HERE, "crypt_gcm.json"), "w") as f:
        json.dump({"source": "OpenSSL libcrypto.so.3 EVP_aes_256_gcm (make_crypt_golden.py)", "cases": cases}, f,
                  indent=0)
    print(f"{len(cases)} cases")


if __name__ == "__main__":
    main()

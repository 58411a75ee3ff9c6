"""Shared builders for the at-rest encryption tests (test_crypt_oracle.py on CPU,
test_crypt_gpu.py on the GPU): records with mixed payload sizes (partial AES blocks,
empty payloads) and optional user headers, built by the oracle encoder."""
import numpy as np

from iggy_amd import abi
from oracle import oracle as O


def raw_record(n: int, lo: int, hi: int, seed: int, uh_max: int = 0, partition_id: int = 3):
    """Encoded record (numpy u8) of n messages, payloads U[lo, hi], user headers
    U[0, uh_max] (0 = none)."""
    rng = np.random.default_rng(seed)
    pls = rng.integers(lo, hi + 1, size=n).astype(np.uint32)
    ids = rng.integers(1, 2**63, size=2 * n, dtype=np.uint64)
    ots = (1_700_000_000_000_000 + np.arange(n, dtype=np.uint64) * 7).astype(np.uint64)
    pay = rng.integers(0, 256, size=max(int(pls.sum()), 1), dtype=np.uint8)
    uhl = rng.integers(0, uh_max + 1, size=n).astype(np.uint32) if uh_max else None
    uhb = rng.integers(0, 256, size=max(int(uhl.sum()), 1), dtype=np.uint8) if uh_max else None
    raw = abi.RawMessages(n, ids.ctypes.data, ots.ctypes.data, pay.ctypes.data, pls.ctypes.data,
                          uhb.ctypes.data if uh_max else None, uhl.ctypes.data if uh_max else None)
    rc, e, out = O.encode_batch(raw, partition_id)
    assert rc == 0, e.astuple()
    return np.frombuffer(out, dtype=np.uint8).copy()


def nonces_for(n: int, seed: int) -> np.ndarray:
    return np.random.default_rng(seed ^ 0x5EED).integers(0, 256, size=24 * max(n, 1), dtype=np.uint8)


def key_for(seed: int) -> bytes:
    return np.random.default_rng(seed ^ 0xC0FFEE).integers(0, 256, size=32, dtype=np.uint8).tobytes()


def frame_sections(record: np.ndarray):
    """[(offset of payload, payload length, offset of user headers, their length)] per frame."""
    rc, e, h, pos = O.decode_batch_slice_with(record, abi.INTEGRITY_LAYOUT_ONLY)
    assert rc == 0, e.astuple()
    out = []
    for p in pos:
        f = 256 + int(p)
        uh = int(record[f + 32: f + 36].view(np.uint32)[0])
        pl = int(record[f + 36: f + 40].view(np.uint32)[0])
        out.append((f + 48, pl, f + 48 + pl, uh))
    return out

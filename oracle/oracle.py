"""ctypes loader for the CPU oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module; it is the checker, never the thing measured or shipped. See
oracle/oracle.h for what it restates and how it is pinned.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

from iggy_amd.abi import (  # shared ABI struct definitions (types only)
    BatchHeader,
    PolledMessage,
    RawMessages,
    SliceQuery,
    SliceResult,
    WireError,
)

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

u64 = ctypes.c_uint64
u32 = ctypes.c_uint32
vp = ctypes.c_void_p


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_xxh3_64.restype = u64
        L.oracle_xxh3_64.argtypes = [vp, ctypes.c_size_t]
        L.oracle_xxh3_64_fast.restype = u64
        L.oracle_xxh3_64_fast.argtypes = [vp, ctypes.c_size_t]
        L.oracle_batch_header_decode.argtypes = [vp, u64, vp, vp]
        L.oracle_decode_batch_slice_with.argtypes = [vp, u64, ctypes.c_int, vp, vp, u64, vp, vp]
        L.oracle_verify_and_recompute.argtypes = [vp, vp, u64, vp, vp, u64, vp, vp]
        L.oracle_calculate_batch_checksum.restype = u64
        L.oracle_calculate_batch_checksum.argtypes = [vp, vp, u64]
        L.oracle_encoded_batch_size.restype = u64
        L.oracle_encoded_batch_size.argtypes = [vp]
        L.oracle_encode_batch.argtypes = [vp, u64, vp, u64, vp, vp]
        L.oracle_poll_decode.argtypes = [vp, u64, ctypes.c_int, vp, u64, vp, vp]
        L.oracle_stamp_batch.argtypes = [vp, u64, u64, u64, vp, vp]
        L.oracle_synth_batch.restype = u64
        L.oracle_synth_batch.argtypes = [vp, u64, u64, u32, u32, u32, u64, u64]
        L.oracle_synth_batch_size.restype = u64
        L.oracle_synth_batch_size.argtypes = [u64, u32, u32, u32, u64]
        L.oracle_cpu_decode_bench.restype = ctypes.c_double
        L.oracle_cpu_decode_bench.argtypes = [vp, u64, ctypes.c_int, ctypes.c_int, vp]
        L.oracle_cpu_decode_bench_integrity.restype = ctypes.c_double
        L.oracle_cpu_decode_bench_integrity.argtypes = [vp, u64, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp]
        L.oracle_has_avx2.restype = ctypes.c_int
        L.oracle_cpu_encode_bench.restype = ctypes.c_double
        L.oracle_cpu_encode_bench.argtypes = [vp, u64, ctypes.c_int, ctypes.c_int, vp]
        L.oracle_select_batch_slice.argtypes = [vp, u64, vp, vp, vp]
        L.oracle_decode_prepare.argtypes = [vp, u64, ctypes.c_int, vp, vp]
        L.oracle_admit_batch.argtypes = [vp, u64, u32, u64, ctypes.c_int, vp, u64, vp, vp]
        L.oracle_recover_segment.argtypes = [vp, u64, u64, vp]
        L.oracle_walk_disk_chunk.argtypes = [vp, u64, vp, ctypes.c_int, vp, vp, u64, vp]
        L.oracle_walk_segment_payload.argtypes = [vp, u64, u64, vp, u64, vp]
        L.oracle_aes256_block.argtypes = [vp, vp, vp]
        L.oracle_gcm_seal.argtypes = [vp, vp, vp, u64, vp]
        L.oracle_gcm_open.argtypes = [vp, vp, u64, vp]
        L.oracle_encrypt_batch.argtypes = [vp, vp, u64, vp, vp, u64, vp, vp]
        L.oracle_decrypt_batch.argtypes = [vp, vp, u64, vp, u64, vp, vp]
        L.oracle_cpu_gcm_bench.restype = ctypes.c_double
        L.oracle_cpu_gcm_bench.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.oracle_cpu_gcm_bench_timed.restype = ctypes.c_double
        L.oracle_cpu_gcm_bench_timed.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_int]
        _lib = L
    return _lib


def _ptr(buf) -> int:
    """Address of a bytes/bytearray/numpy buffer (bytes are copied)."""
    import numpy as np

    if isinstance(buf, np.ndarray):
        return buf.ctypes.data
    if isinstance(buf, bytearray):
        return ctypes.addressof((ctypes.c_char * len(buf)).from_buffer(buf)) if len(buf) else 0
    raise TypeError("pass bytearray or numpy array")


def _as_np(buf):
    import numpy as np

    if isinstance(buf, np.ndarray):
        return buf
    return np.frombuffer(bytes(buf), dtype=np.uint8).copy()


def xxh3_64(data: bytes) -> int:
    a = _as_np(data)
    return lib().oracle_xxh3_64(a.ctypes.data if a.size else None, a.size)


def xxh3_64_fast(data: bytes) -> int:
    a = _as_np(data)
    return lib().oracle_xxh3_64_fast(a.ctypes.data if a.size else None, a.size)


def decode_batch_slice_with(body, integrity: int = 0, want_frames: bool = True):
    """-> (rc, WireError, BatchHeader, frame_positions list)"""
    import numpy as np

    a = _as_np(body)
    h = BatchHeader()
    e = WireError()
    cap = a.size // 48 + 1 if want_frames else 0
    pos = np.zeros(max(cap, 1), dtype=np.uint64)
    n = u64(0)
    rc = lib().oracle_decode_batch_slice_with(
        a.ctypes.data, a.size, integrity, ctypes.byref(h), pos.ctypes.data if cap else None,
        cap, ctypes.byref(n), ctypes.byref(e))
    frames = pos[: n.value].copy() if (rc == 0 and want_frames) else None
    return rc, e, h, frames


def calculate_batch_checksum(h: BatchHeader, blob) -> int:
    a = _as_np(blob)
    return lib().oracle_calculate_batch_checksum(ctypes.byref(h), a.ctypes.data if a.size else None, a.size)


def encode_batch(raw: "RawMessages", partition_id: int = 0):
    """raw: iggy_amd.abi.RawMessages bound to host arrays. -> (rc, err, bytes)."""
    import numpy as np

    need = lib().oracle_encoded_batch_size(ctypes.byref(raw)) if raw.count else 256
    out = np.zeros(need, dtype=np.uint8)
    n = u64(0)
    e = WireError()
    rc = lib().oracle_encode_batch(ctypes.byref(raw), partition_id, out.ctypes.data, need,
                                   ctypes.byref(n), ctypes.byref(e))
    return rc, e, out[: n.value].tobytes() if rc == 0 else b""


def poll_decode(records, mode: int = 0, cap: int | None = None):
    a = _as_np(records)
    if cap is None:
        cap = a.size // 48 + 1
    out = (PolledMessage * max(cap, 1))()
    n = u64(0)
    e = WireError()
    rc = lib().oracle_poll_decode(a.ctypes.data if a.size else None, a.size, mode, out, cap,
                                  ctypes.byref(n), ctypes.byref(e))
    return rc, e, [out[i] for i in range(n.value)]


def stamp_batch(batch, base_offset: int, base_timestamp: int):
    a = _as_np(batch)
    h = BatchHeader()
    e = WireError()
    rc = lib().oracle_stamp_batch(a.ctypes.data, a.size, base_offset, base_timestamp,
                                  ctypes.byref(h), ctypes.byref(e))
    return rc, e, h, a.tobytes()


def decode_prepare(frame, validate: bool = True):
    """decode_prepare_slice / _trusted -> (rc, WireError, BatchHeader)"""
    a = _as_np(frame)
    h = BatchHeader()
    e = WireError()
    rc = lib().oracle_decode_prepare(a.ctypes.data if a.size else None, a.size, 1 if validate else 0,
                                     ctypes.byref(h), ctypes.byref(e))
    return rc, e, h


def admit_batch(batch, metadata_messages_count: int, partition_id: int, checksum_mode: int = 0):
    """admit_wire_request's batch half -> (rc, WireError, BatchHeader, admitted bytes or None)"""
    import numpy as np

    a = _as_np(batch)
    out = np.zeros(max(a.size, 1), dtype=np.uint8)
    h = BatchHeader()
    e = WireError()
    rc = lib().oracle_admit_batch(a.ctypes.data if a.size else None, a.size, metadata_messages_count,
                                  partition_id, checksum_mode, out.ctypes.data, out.size, ctypes.byref(h),
                                  ctypes.byref(e))
    return rc, e, h, (out[:a.size].tobytes() if rc == 0 else None)


def recover_segment(messages, start_offset: int):
    """recover_segment_bounds' index-less walk -> (rc, SegmentRecovery)"""
    from iggy_amd.abi import SegmentRecovery

    a = _as_np(messages)
    out = SegmentRecovery()
    rc = lib().oracle_recover_segment(a.ctypes.data if a.size else None, a.size, start_offset, ctypes.byref(out))
    return rc, out


def select_slice(record, kind: int, value: int, count: int, ceiling: int = 2**64 - 1, already_matched: int = 0):
    """-> (rc, SliceResult, header bytes or None)"""
    import numpy as np

    a = _as_np(record)
    q = SliceQuery(kind, count, value, ceiling, already_matched, 0)
    out = SliceResult()
    hdr = np.zeros(256, dtype=np.uint8)
    rc = lib().oracle_select_batch_slice(a.ctypes.data if a.size else None, a.size, ctypes.byref(q),
                                         ctypes.byref(out), hdr.ctypes.data)
    return rc, out, (hdr.tobytes() if rc == 0 and out.selected else None)


def synth_batch(n: int, pl_min: int, pl_max: int | None = None, uh_len: int = 0,
                seed: int = 0x16619E3779B97F4A, partition_id: int = 1, out=None):
    """Seeded synthetic stamped record (BASELINE.md input spec) as numpy u8."""
    import numpy as np

    if pl_max is None:
        pl_max = pl_min
    size = lib().oracle_synth_batch_size(n, pl_min, pl_max, uh_len, seed)
    if out is None:
        out = np.empty(size, dtype=np.uint8)
    got = lib().oracle_synth_batch(out.ctypes.data, out.size, n, pl_min, pl_max, uh_len, seed,
                                   partition_id)
    assert got == size
    return out[:size]


def cpu_decode_bench(body, threads: int, reps: int, integrity: int = 0):
    """Seconds for `threads` threads to each walk `reps` copies (integrity 0 = Verify,
    1 = LayoutOnly), and the batch checksum (Verify; 0 on any error or LayoutOnly)."""
    a = _as_np(body)
    c = u64(0)
    secs = lib().oracle_cpu_decode_bench_integrity(a.ctypes.data, a.size, threads, reps, integrity, ctypes.byref(c))
    return secs, c.value


def cpu_encode_bench(raw: "RawMessages", partition_id: int, threads: int, reps: int):
    b = u64(0)
    secs = lib().oracle_cpu_encode_bench(ctypes.byref(raw), partition_id, threads, reps, ctypes.byref(b))
    return secs, b.value


def walk_disk_chunk(chunk, kind: int, value: int, count: int, ceiling: int = 2**64 - 1, already_matched: int = 0,
                    integrity: int = 0, cap: int = 64):
    """walk_disk_chunk (poll_plan.rs:950-1011) -> (rc, ChunkWalk, [ChunkFragment], [header bytes])"""
    import numpy as np
    from iggy_amd.abi import ChunkFragment, ChunkWalk

    a = _as_np(chunk)
    q = SliceQuery(kind, count, value, ceiling, already_matched, 0)
    frags = (ChunkFragment * max(cap, 1))()
    hdrs = np.zeros(256 * max(cap, 1), dtype=np.uint8)
    w = ChunkWalk()
    rc = lib().oracle_walk_disk_chunk(a.ctypes.data if a.size else None, a.size, ctypes.byref(q), integrity, frags,
                                      hdrs.ctypes.data, cap, ctypes.byref(w))
    n = min(w.fragments, cap)
    return rc, w, [frags[i] for i in range(n)], [hdrs[256 * i: 256 * i + 256].tobytes() for i in range(n)]


def walk_segment_payload(payload, base_offset: int, index_cap: int = 4096):
    """walk_segment_payload (state_transfer.rs:715-833) -> (rc, SegmentWalk, index bytes)"""
    import numpy as np
    from iggy_amd.abi import SegmentWalk

    a = _as_np(payload)
    idx = np.zeros(24 * max(index_cap, 1), dtype=np.uint8)
    w = SegmentWalk()
    rc = lib().oracle_walk_segment_payload(a.ctypes.data if a.size else None, a.size, base_offset, idx.ctypes.data,
                                           index_cap, ctypes.byref(w))
    n = min(w.index_entries, index_cap)
    return rc, w, idx[: 24 * n].tobytes()


# ------------------------------------------------------------ at-rest encryption
def aes256_block(key: bytes, block: bytes) -> bytes:
    import numpy as np

    k = np.frombuffer(bytes(key), dtype=np.uint8).copy()
    b = np.frombuffer(bytes(block), dtype=np.uint8).copy()
    out = np.zeros(16, dtype=np.uint8)
    lib().oracle_aes256_block(k.ctypes.data, b.ctypes.data, out.ctypes.data)
    return out.tobytes()


def gcm_seal(key: bytes, nonce: bytes, pt: bytes) -> bytes:
    """Aes256GcmEncryptor::encrypt with the given nonce -> nonce || ct || tag"""
    import numpy as np

    k = np.frombuffer(bytes(key), dtype=np.uint8).copy()
    nn = np.frombuffer(bytes(nonce), dtype=np.uint8).copy()
    p = _as_np(pt)
    out = np.zeros(len(pt) + 28, dtype=np.uint8)
    lib().oracle_gcm_seal(k.ctypes.data, nn.ctypes.data, p.ctypes.data if p.size else None, p.size, out.ctypes.data)
    return out.tobytes()


def gcm_open(key: bytes, data: bytes):
    """Aes256GcmEncryptor::decrypt -> plaintext bytes, or None (CannotDecryptData)"""
    import numpy as np

    k = np.frombuffer(bytes(key), dtype=np.uint8).copy()
    d = _as_np(data)
    out = np.zeros(max(len(data) - 28, 1), dtype=np.uint8)
    rc = lib().oracle_gcm_open(k.ctypes.data, d.ctypes.data if d.size else None, d.size, out.ctypes.data)
    return None if rc else out[: max(len(data) - 28, 0)].tobytes()


def encrypt_batch(key: bytes, record, nonces):
    """encrypt_batch_request's batch transform -> (rc, WireError, bytes)"""
    import numpy as np

    k = np.frombuffer(bytes(key), dtype=np.uint8).copy()
    a = _as_np(record)
    nn = _as_np(nonces)
    cap = a.size + 56 * (a.size // 48 + 1) + 256
    out = np.zeros(cap, dtype=np.uint8)
    n = u64(0)
    e = WireError()
    rc = lib().oracle_encrypt_batch(k.ctypes.data, a.ctypes.data, a.size, nn.ctypes.data if nn.size else None,
                                    out.ctypes.data, cap, ctypes.byref(n), ctypes.byref(e))
    return rc, e, out[: n.value].tobytes() if rc == 0 else b""


def decrypt_batch(key: bytes, record):
    """decrypt_batch_record -> (rc, WireError, bytes)"""
    import numpy as np

    k = np.frombuffer(bytes(key), dtype=np.uint8).copy()
    a = _as_np(record)
    out = np.zeros(max(a.size, 256), dtype=np.uint8)
    n = u64(0)
    e = WireError()
    rc = lib().oracle_decrypt_batch(k.ctypes.data, a.ctypes.data, a.size, out.ctypes.data, out.size,
                                    ctypes.byref(n), ctypes.byref(e))
    return rc, e, out[: n.value].tobytes() if rc == 0 else b""


def cpu_gcm_bench(threads: int, nsec: int, secsize: int) -> float:
    """seconds for threads x nsec AES-256-GCM seals of secsize bytes (OpenSSL); -1 if unavailable"""
    return lib().oracle_cpu_gcm_bench(threads, nsec, secsize)


def cpu_gcm_gib_s(threads: int, seconds: float, secsize: int = 1024) -> float:
    """Aggregate OpenSSL AES-256-GCM seal rate of `threads` workers started together and
    stopped by one deadline (thread start-up outside the window); -1 if unavailable."""
    n = lib().oracle_cpu_gcm_bench_timed(threads, seconds, secsize)
    return -1.0 if n < 0 else n * secsize / seconds / 2**30

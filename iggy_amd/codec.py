"""Python host binding of the MI355X codec (ctypes over include/iggy_codec.h).

Mirrors the reference interface of the path (names and error behaviour of
core/binary_protocol/src/batch.rs, requests/messages/send_messages.rs,
common/src/types/message/polled_messages.rs): every method returns the same
outcome the Rust function would, with `WireError` fields mirrored by
iggy_amd.abi.WireError. The library is the product path; there is no CPU
fallback — constructing a Codec without a gfx950 device raises.
"""
from __future__ import annotations

import ctypes
import os
import re

import numpy as np

from . import abi
from .abi import (BatchHeader, Completion, DecodeResult, EncodeResult, Identifier, Partitioning, PolledMessage,
                  PolledPrefix, ProducerConfig, ProducerRequest, RawMessages, SendMessagesHeader, SliceQuery,
                  SliceResult, WireError)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libiggy_codec.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "iggy_codec.h")

u64 = ctypes.c_uint64
u32 = ctypes.c_uint32
vp = ctypes.c_void_p
ci = ctypes.c_int
_lib = None


class CodecError(RuntimeError):
    def __init__(self, rc: int, err: WireError | None = None, what: str = ""):
        self.rc = rc
        self.err = err
        super().__init__(f"{what}: rc={rc} {err!r}")


def exported_symbols() -> list[str]:
    """Every function the C ABI header declares."""
    with open(HEADER_PATH) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w\s\*]*?\b(iggy_\w+)\s*\(", text, flags=re.M)
    return sorted(set(names))


def use_library(path: str) -> None:
    """Diagnostics only: bind this module to another build of the library (the
    ablation build libiggy_codec_diag.so) before the first lib() call."""
    global LIB_PATH, _lib
    if _lib is not None:
        raise RuntimeError("the codec library is already loaded")
    LIB_PATH = path


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        _lib = load(LIB_PATH)
    return _lib


DIAG_LIB_PATH = os.path.join(_HERE, "libiggy_codec_diag.so")


def load(path: str) -> ctypes.CDLL:
    """Load one build of the library and declare its C ABI (lib() is the product build)."""
    if not os.path.exists(path):
        raise FileNotFoundError(
            f"{path} missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    # PyTorch-ROCm ships its own libamdhip64.so.7 / libhsa-runtime64.so.1 under the
    # same sonames as /opt/rocm's. Whichever loads first serves the whole process;
    # load torch's first (when torch is installed) so that torch and the codec share
    # one HIP runtime and torch's lazy GPU init never runs beside another runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(path)
    L.iggy_codec_abi_version.restype = u32
    L.iggy_codec_create.argtypes = [ci, ctypes.POINTER(vp)]
    L.iggy_codec_destroy.argtypes = [vp]
    L.iggy_codec_destroy.restype = None
    L.iggy_codec_reserve.argtypes = [vp, u64, u64]
    L.iggy_codec_stream.argtypes = [vp]
    L.iggy_codec_stream.restype = vp
    L.iggy_codec_synchronize.argtypes = [vp]
    L.iggy_batch_header_decode.argtypes = [vp, u64, vp, vp]
    L.iggy_batch_header_encode.argtypes = [vp, vp]
    L.iggy_batch_header_encode.restype = None
    L.iggy_encoded_batch_size.argtypes = [vp]
    L.iggy_encoded_batch_size.restype = u64
    L.iggy_codec_xxh3_64.argtypes = [vp, vp, u64, vp]
    L.iggy_codec_decode_batch.argtypes = [vp, vp, u64, ci, vp, vp, u64, vp, vp]
    L.iggy_codec_verify_and_recompute_batch_checksum.argtypes = [vp, vp, vp, u64, vp, vp]
    L.iggy_codec_calculate_batch_checksum.argtypes = [vp, vp, vp, u64, vp]
    L.iggy_codec_encode_batch.argtypes = [vp, vp, u64, vp, u64, vp, vp]
    L.iggy_codec_poll_decode.argtypes = [vp, vp, u64, ci, vp, u64, vp, vp]
    L.iggy_codec_decode_records.argtypes = [vp, vp, u64, vp, u64, ci, vp]
    L.iggy_frame_read.argtypes = [ci, vp, u64, u64, vp, vp]
    L.iggy_frame_read_rest.argtypes = [ci, vp, u64, vp]
    L.iggy_codec_convert_request.argtypes = [vp, vp, u64, u64, ci, vp, u64, vp, vp, vp]
    L.iggy_codec_stamp_batch.argtypes = [vp, vp, u64, u64, u64, vp, vp]
    L.iggy_codec_decode_batch_device.argtypes = [vp, vp, u64, ci, vp, u64, vp, vp]
    L.iggy_codec_encode_batch_device.argtypes = [vp, vp, u64, vp, u64, vp, vp]
    L.iggy_codec_batch_checksum_device.argtypes = [vp, vp, vp, vp, u64, vp, vp]
    L.iggy_codec_xxh3_64_ranges_device.argtypes = [vp, vp, vp, vp, u64, vp, vp]
    L.iggy_codec_select_slice.argtypes = [vp, vp, u64, vp, vp, vp, vp]
    L.iggy_codec_select_slice_device.argtypes = [vp, vp, vp, u64, vp, vp, vp, vp]
    L.iggy_codec_stamp_batch_device.argtypes = [vp, vp, vp, u64, u64, u64, vp, vp]
    L.iggy_codec_decode_prepare.argtypes = [vp, vp, u64, ci, vp, vp]
    L.iggy_codec_admit_batch.argtypes = [vp, vp, u64, u32, u64, ci, vp, u64, vp, vp]
    L.iggy_codec_recover_segment.argtypes = [vp, vp, u64, u64, vp]
    L.iggy_codec_walk_disk_chunk.argtypes = [vp, vp, u64, vp, ci, vp, vp, u64, vp]
    L.iggy_codec_walk_segment_payload.argtypes = [vp, vp, u64, u64, vp, u64, vp]
    L.iggy_codec_segment_write_device.argtypes = [vp, ci, u64, vp, u64, ci, ctypes.POINTER(u64)]
    L.iggy_codec_encrypt_batch_device.argtypes = [vp, vp, vp, u64, vp, vp, u64, vp, vp]
    L.iggy_codec_decrypt_batch_device.argtypes = [vp, vp, vp, u64, vp, u64, vp, vp]
    L.iggy_codec_build_polled_body.argtypes = [vp, u32, u64, vp, u64, vp, vp, u64, ctypes.POINTER(u64), vp]
    L.iggy_codec_profile_enable.argtypes = [vp, ci]
    L.iggy_codec_profile_read.argtypes = [vp, ci, vp, vp]
    L.iggy_codec_host_stats.argtypes = [vp, vp]
    L.iggy_codec_service_start.argtypes = [vp]
    L.iggy_codec_service_stop.argtypes = [vp]
    L.iggy_codec_host_register.argtypes = [vp, vp, u64]
    L.iggy_codec_host_unregister.argtypes = [vp, vp]
    L.iggy_codec_host_pinned.argtypes = [vp, u64]
    L.iggy_codec_decode_submit.argtypes = [vp, vp, u64, ci, vp, u64, ctypes.POINTER(u64)]
    L.iggy_codec_encode_submit.argtypes = [vp, vp, u64, vp, u64, ctypes.POINTER(u64)]
    L.iggy_codec_poll.argtypes = [vp, u64, vp]
    L.iggy_codec_wait.argtypes = [vp, u64, vp]
    L.iggy_codec_error_string.argtypes = [u32, u32]
    L.iggy_codec_error_string.restype = ctypes.c_char_p
    L.iggy_codec_debug_set.argtypes = [vp, u32]
    L.iggy_send_messages_header_encode.argtypes = [vp, vp, u64, ctypes.POINTER(u64)]
    L.iggy_send_messages_header_decode.argtypes = [vp, u64, vp, ctypes.POINTER(u64), vp]
    L.iggy_send_messages_encoded_size.argtypes = [vp, vp]
    L.iggy_send_messages_encoded_size.restype = u64
    L.iggy_codec_send_messages_encode.argtypes = [vp, vp, vp, vp, u64, ctypes.POINTER(u64), vp]
    L.iggy_codec_polled_messages_from_bytes.argtypes = [vp, vp, u64, vp, vp, u64, ctypes.POINTER(u64), vp]
    L.iggy_producer_create.argtypes = [vp, vp, ctypes.POINTER(vp)]
    L.iggy_producer_destroy.argtypes = [vp]
    L.iggy_producer_destroy.restype = None
    L.iggy_producer_append.argtypes = [vp, vp, vp, vp, vp, ctypes.POINTER(ci)]
    L.iggy_producer_pending.argtypes = [vp, ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(u64)]
    L.iggy_producer_flush.argtypes = [vp, vp, u64, vp, u64, ctypes.POINTER(u64), vp]
    return L


def _np(buf) -> np.ndarray:
    if isinstance(buf, np.ndarray):
        return np.ascontiguousarray(buf).view(np.uint8).reshape(-1)
    return np.frombuffer(bytes(buf), dtype=np.uint8).copy()


def _addr(a: np.ndarray):
    return a.ctypes.data if a.size else None


def frame_read(fd: int, cap: int, max_message_size: int = 64 << 20, grow: bool = False):
    """read_message (message_bus/src/framing.rs:107-164) + Message::<GenericHeader>::
    try_from on a blocking socket fd -> (rc, WireError, frame bytes as a numpy view of a
    4096-aligned buffer). grow: a frame larger than cap continues in a larger buffer
    (iggy_frame_read_rest) instead of returning IGGY_ERR_CAPACITY."""
    raw = np.zeros(cap + 4096, dtype=np.uint8)
    off = (-raw.ctypes.data) % 4096
    buf = raw[off: off + cap]
    n = u64(0)
    e = WireError()
    rc = lib().iggy_frame_read(fd, buf.ctypes.data if cap else None, cap, max_message_size, ctypes.byref(n),
                               ctypes.byref(e))
    if rc == abi.ERR_CAPACITY and grow and n.value:
        # the reference grows its buffer in place (framing.rs:150-160): a larger aligned
        # buffer takes the header and the rest of the frame is read into it
        big = np.zeros(n.value + 4096, dtype=np.uint8)
        off = (-big.ctypes.data) % 4096
        nb = big[off: off + n.value]
        nb[:256] = buf[:256]
        rc = lib().iggy_frame_read_rest(fd, nb.ctypes.data, n.value, ctypes.byref(e))
        return rc, e, nb if rc == 0 else nb[:0]
    return rc, e, buf[: n.value] if rc == 0 else buf[:0]


def send_messages_header_encode(h: SendMessagesHeader) -> bytes:
    """SendMessagesHeader WireEncode (send_messages.rs:209-220): metadata fields, no length prefix."""
    n = u64(0)
    out = np.zeros(1024, dtype=np.uint8)
    rc = lib().iggy_send_messages_header_encode(ctypes.byref(h), out.ctypes.data, out.size, ctypes.byref(n))
    if rc:
        raise CodecError(rc, None, "send_messages_header_encode")
    return out[: n.value].tobytes()


def send_messages_header_decode(buf):
    """SendMessagesHeader::decode (send_messages.rs:222-241) -> (rc, WireError, header, consumed)."""
    a = _np(buf)
    h = SendMessagesHeader()
    n = u64(0)
    e = WireError()
    rc = lib().iggy_send_messages_header_decode(_addr(a), a.size, ctypes.byref(h), ctypes.byref(n), ctypes.byref(e))
    return rc, e, h, n.value


class Codec:
    """One codec context bound to one HIP device (thread-per-core shards each own one)."""

    def __init__(self, device: int = 0, library: ctypes.CDLL | None = None):
        self._L = library if library is not None else lib()
        h = vp()
        rc = self._L.iggy_codec_create(device, ctypes.byref(h))
        if rc != 0:
            raise CodecError(rc, None, f"iggy_codec_create(device={device})")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.iggy_codec_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def stream(self) -> int:
        return self._L.iggy_codec_stream(self._h) or 0

    def reserve(self, max_batch_bytes: int, max_frames: int = 0):
        rc = self._L.iggy_codec_reserve(self._h, max_batch_bytes, max_frames)
        if rc:
            raise CodecError(rc, None, "reserve")

    # ----------------------------------------------------------- host buffers
    def xxh3_64(self, data) -> int:
        a = _np(data)
        out = u64(0)
        rc = self._L.iggy_codec_xxh3_64(self._h, _addr(a), a.size, ctypes.byref(out))
        if rc:
            raise CodecError(rc, None, "xxh3_64")
        return out.value

    def decode_batch_slice_with(self, body, integrity: int = abi.INTEGRITY_VERIFY,
                                want_frames: bool = True):
        """decode_batch_slice_with (batch.rs:391) -> (rc, WireError, BatchHeader, frames)."""
        a = _np(body)
        h = BatchHeader()
        e = WireError()
        cap = a.size // 48 + 1 if want_frames else 0
        pos = np.zeros(max(cap, 1), dtype=np.uint64)
        n = u64(0)
        rc = self._L.iggy_codec_decode_batch(self._h, _addr(a), a.size, integrity, ctypes.byref(h),
                                             pos.ctypes.data if cap else None, cap, ctypes.byref(n),
                                             ctypes.byref(e))
        frames = pos[: n.value].copy() if (rc == 0 and want_frames) else None
        return rc, e, h, frames

    def decode_batch_into(self, body: np.ndarray, integrity: int, pos: np.ndarray | None,
                          h: BatchHeader | None = None, e: WireError | None = None) -> tuple[int, int]:
        """decode_batch_slice_with into caller arrays (no allocation: latency
        measurements, registered buffers) -> (rc, frame count)."""
        h = h if h is not None else BatchHeader()
        e = e if e is not None else WireError()
        n = u64(0)
        rc = self._L.iggy_codec_decode_batch(self._h, body.ctypes.data, body.nbytes, integrity, ctypes.byref(h),
                                             pos.ctypes.data if pos is not None else None,
                                             pos.size if pos is not None else 0, ctypes.byref(n), ctypes.byref(e))
        return rc, n.value

    def verify_and_recompute_batch_checksum(self, h: BatchHeader, blob):
        a = _np(blob)
        out = u64(0)
        e = WireError()
        rc = self._L.iggy_codec_verify_and_recompute_batch_checksum(
            self._h, ctypes.byref(h), _addr(a), a.size, ctypes.byref(out), ctypes.byref(e))
        return rc, e, out.value

    def calculate_batch_checksum(self, h: BatchHeader, blob) -> int:
        a = _np(blob)
        out = u64(0)
        rc = self._L.iggy_codec_calculate_batch_checksum(self._h, ctypes.byref(h), _addr(a), a.size,
                                                         ctypes.byref(out))
        if rc:
            raise CodecError(rc, None, "calculate_batch_checksum")
        return out.value

    def encode_batch(self, raw: RawMessages, partition_id: int = 0):
        """SendMessagesEncoder::encode batch section -> (rc, WireError, bytes)."""
        need = self._L.iggy_encoded_batch_size(ctypes.byref(raw)) if raw.count else 256
        out = np.zeros(need, dtype=np.uint8)
        n = u64(0)
        e = WireError()
        rc = self._L.iggy_codec_encode_batch(self._h, ctypes.byref(raw), partition_id, out.ctypes.data,
                                             need, ctypes.byref(n), ctypes.byref(e))
        return rc, e, (out[: n.value].tobytes() if rc == 0 else b"")

    def poll_decode(self, records, mode: int = abi.POLL_MODE_SDK, cap: int | None = None):
        a = _np(records)
        if cap is None:
            cap = a.size // 48 + 1
        out = (PolledMessage * max(cap, 1))()
        n = u64(0)
        e = WireError()
        rc = self._L.iggy_codec_poll_decode(self._h, _addr(a), a.size, mode, out, cap,
                                            ctypes.byref(n), ctypes.byref(e))
        return rc, e, [out[i] for i in range(n.value)]

    def stamp_batch(self, batch, base_offset: int, base_timestamp: int):
        a = _np(batch).copy()
        h = BatchHeader()
        e = WireError()
        rc = self._L.iggy_codec_stamp_batch(self._h, a.ctypes.data, a.size, base_offset,
                                            base_timestamp, ctypes.byref(h), ctypes.byref(e))
        return rc, e, h, a.tobytes()

    def select_slice(self, record, kind: int, value: int, count: int, ceiling: int = 2**64 - 1,
                     already_matched: int = 0):
        """select_batch_slice + served header (journal.rs:1025-1137) ->
        (rc, WireError, SliceResult, header bytes or None)."""
        a = _np(record)
        q = SliceQuery(kind, count, value, ceiling, already_matched, 0)
        out = SliceResult()
        hdr = np.zeros(256, dtype=np.uint8)
        e = WireError()
        rc = self._L.iggy_codec_select_slice(self._h, _addr(a), a.size, ctypes.byref(q), ctypes.byref(out),
                                             hdr.ctypes.data, ctypes.byref(e))
        return rc, e, out, (hdr.tobytes() if rc == 0 and out.selected else None)

    def decode_prepare(self, frame, validate: bool = True):
        """decode_prepare_slice / _trusted (server_common/src/send_messages.rs:542-622)
        -> (rc, WireError, BatchHeader)."""
        a = _np(frame)
        h = BatchHeader()
        e = WireError()
        rc = self._L.iggy_codec_decode_prepare(self._h, _addr(a), a.size, 1 if validate else 0,
                                               ctypes.byref(h), ctypes.byref(e))
        return rc, e, h

    def admit_batch(self, batch, metadata_messages_count: int, partition_id: int,
                    checksum_mode: int = abi.CHECKSUM_COMPUTE):
        """admit_wire_request's batch half (server_common/src/send_messages.rs:480-540)
        -> (rc, WireError, BatchHeader, admitted bytes or None)."""
        a = _np(batch)
        out = np.zeros(max(a.size, 1), dtype=np.uint8)
        h = BatchHeader()
        e = WireError()
        rc = self._L.iggy_codec_admit_batch(self._h, _addr(a), a.size, metadata_messages_count, partition_id,
                                            checksum_mode, out.ctypes.data, out.size, ctypes.byref(h),
                                            ctypes.byref(e))
        return rc, e, h, (out[:a.size].tobytes() if rc == 0 else None)

    def decode_records(self, buf, offsets, integrity: int = abi.INTEGRITY_VERIFY):
        """decode_batch_slice_with of record k = buf[offsets[k]:] for every k, one launch
        for the single-stride records -> (rc, [DecodeResult])."""
        a = _np(buf)
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        out = (abi.DecodeResult * max(offs.size, 1))()
        rc = self._L.iggy_codec_decode_records(self._h, _addr(a), a.size, offs.ctypes.data if offs.size else None,
                                               offs.size, integrity, out)
        return rc, [out[i] for i in range(offs.size)]

    def convert_request(self, frame, partition_id: int, checksum_mode: int = 0, cap: int | None = None):
        """convert_request_message + admit_wire_request (server_common/src/send_messages.rs:459-540)
        on one [RoutedRequestHeader][body] frame -> (rc, WireError, BatchHeader, output bytes)."""
        a = _np(frame)
        cap = a.size + 256 if cap is None else cap
        out = np.zeros(max(cap, 1), dtype=np.uint8)
        n = u64(0)
        h = BatchHeader()
        e = WireError()
        rc = self._L.iggy_codec_convert_request(self._h, _addr(a), a.size, partition_id, checksum_mode,
                                                out.ctypes.data, cap, ctypes.byref(n), ctypes.byref(h),
                                                ctypes.byref(e))
        return rc, e, h, out[: n.value].tobytes()

    def recover_segment(self, messages, start_offset: int):
        """recover_segment_bounds' index-less walk (segment_recovery.rs:425-530)
        -> (rc, SegmentRecovery)."""
        a = _np(messages)
        out = abi.SegmentRecovery()
        rc = self._L.iggy_codec_recover_segment(self._h, _addr(a), a.size, start_offset, ctypes.byref(out))
        return rc, out

    def walk_disk_chunk(self, chunk, kind: int, value: int, count: int, ceiling: int = 2**64 - 1,
                        already_matched: int = 0, integrity: int = abi.INTEGRITY_VERIFY, cap: int = 64):
        """walk_disk_chunk (poll_plan.rs:950-1011) -> (rc, ChunkWalk, [ChunkFragment], [header bytes])."""
        a = _np(chunk)
        q = SliceQuery(kind, count, value, ceiling, already_matched, 0)
        frags = (abi.ChunkFragment * max(cap, 1))()
        hdrs = np.zeros(256 * max(cap, 1), dtype=np.uint8)
        w = abi.ChunkWalk()
        rc = self._L.iggy_codec_walk_disk_chunk(self._h, _addr(a), a.size, ctypes.byref(q), integrity, frags,
                                                hdrs.ctypes.data, cap, ctypes.byref(w))
        n = min(w.fragments, cap)
        return rc, w, [frags[i] for i in range(n)], [hdrs[256 * i: 256 * i + 256].tobytes() for i in range(n)]

    def walk_segment_payload(self, payload, base_offset: int, index_cap: int = 4096):
        """walk_segment_payload (state_transfer.rs:715-833) -> (rc, SegmentWalk, index bytes)."""
        a = _np(payload)
        idx = np.zeros(24 * max(index_cap, 1), dtype=np.uint8)
        w = abi.SegmentWalk()
        rc = self._L.iggy_codec_walk_segment_payload(self._h, _addr(a), a.size, base_offset, idx.ctypes.data,
                                                     index_cap, ctypes.byref(w))
        n = min(w.index_entries, index_cap)
        return rc, w, idx[: 24 * n].tobytes()

    def segment_write_device(self, fd: int, position: int, d_bytes: int, length: int, fsync: bool = False) -> int:
        """MessagesWriter::save_frozen_batches for device-resident batches -> bytes written."""
        w = u64(0)
        rc = self._L.iggy_codec_segment_write_device(self._h, fd, position, d_bytes, length, 1 if fsync else 0,
                                                     ctypes.byref(w))
        if rc:
            raise CodecError(rc, None, "segment_write_device")
        return w.value

    def encrypt_batch_device(self, key: bytes, d_record: int, length: int, d_nonces: int, d_out: int, cap: int,
                             d_result: int, stream: int | None = None) -> int:
        """encrypt_batch_request's batch re-encode (send_messages.rs:293-355) on device buffers;
        d_nonces: 24 B per message (payload nonce, user-headers nonce). Result: abi.CryptResult."""
        if len(key) != 32:
            raise ValueError("AES-256 key must be 32 bytes")
        k = ctypes.create_string_buffer(bytes(key), 32)
        return self._L.iggy_codec_encrypt_batch_device(self._h, k, d_record, length, d_nonces, d_out, cap,
                                                       d_result, stream)

    def decrypt_batch_device(self, key: bytes, d_record: int, length: int, d_out: int, cap: int, d_result: int,
                             stream: int | None = None) -> int:
        """decrypt_batch_record (send_messages.rs:357-415) on device buffers. Result: abi.CryptResult."""
        if len(key) != 32:
            raise ValueError("AES-256 key must be 32 bytes")
        k = ctypes.create_string_buffer(bytes(key), 32)
        return self._L.iggy_codec_decrypt_batch_device(self._h, k, d_record, length, d_out, cap, d_result, stream)

    def build_polled_body(self, partition_id: int, current_offset: int, fragments, key: bytes | None = None,
                          cap: int | None = None):
        """build_polled_messages_body (core/server/src/responses.rs:1666-1714) over host
        fragments (bytes / numpy) -> (rc, WireError, body bytes)."""
        arrs = [_np(f) for f in fragments]
        spans = (abi.PollFragment * max(len(arrs), 1))()
        for k, a in enumerate(arrs):
            spans[k].data = a.ctypes.data if a.size else None
            spans[k].len = a.size
        total = sum(a.size for a in arrs)
        cap = 16 + total if cap is None else cap
        out = np.zeros(max(cap, 1), dtype=np.uint8)
        n = u64(0)
        e = WireError()
        if key is not None and len(key) != 32:
            raise ValueError("AES-256 key must be 32 bytes")
        k = np.frombuffer(bytes(key), dtype=np.uint8).copy() if key is not None else None
        rc = self._L.iggy_codec_build_polled_body(self._h, partition_id, current_offset, spans, len(arrs),
                                                  k.ctypes.data if k is not None else None, out.ctypes.data, cap,
                                                  ctypes.byref(n), ctypes.byref(e))
        return rc, e, out[: n.value].tobytes()

    def select_slice_device(self, d_record: int, d_frame_pos: int, nframes: int, query: SliceQuery,
                            d_out: int, d_header: int | None = None, stream: int | None = None) -> int:
        return self._L.iggy_codec_select_slice_device(self._h, d_record, d_frame_pos, nframes, ctypes.byref(query),
                                                      d_out, d_header, stream)

    def stamp_device(self, d_record: int, d_frame_pos: int, nframes: int, base_offset: int, base_timestamp: int,
                     d_header: int | None = None, stream: int | None = None) -> int:
        return self._L.iggy_codec_stamp_batch_device(self._h, d_record, d_frame_pos, nframes, base_offset,
                                                     base_timestamp, d_header, stream)

    # --------------------------------------------------------- device buffers
    def decode_device(self, d_body: int, length: int, integrity: int, d_frame_pos: int | None,
                      cap: int, d_result: int, stream: int | None = None) -> int:
        return self._L.iggy_codec_decode_batch_device(self._h, d_body, length, integrity,
                                                      d_frame_pos, cap, d_result, stream)

    def encode_device(self, raw_dev: RawMessages, partition_id: int, d_out: int, cap: int,
                      d_result: int, stream: int | None = None) -> int:
        return self._L.iggy_codec_encode_batch_device(self._h, ctypes.byref(raw_dev), partition_id,
                                                      d_out, cap, d_result, stream)

    def xxh3_ranges_device(self, d_data, d_offsets, d_lengths, n, d_out, stream=None) -> int:
        return self._L.iggy_codec_xxh3_64_ranges_device(self._h, d_data, d_offsets, d_lengths, n,
                                                        d_out, stream)

    # ------------------------------------------- asynchronous host buffers
    def host_register(self, arr: np.ndarray):
        rc = self._L.iggy_codec_host_register(self._h, arr.ctypes.data, arr.nbytes)
        if rc:
            raise CodecError(rc, None, "host_register")

    def host_unregister(self, arr: np.ndarray):
        rc = self._L.iggy_codec_host_unregister(self._h, arr.ctypes.data)
        if rc:
            raise CodecError(rc, None, "host_unregister")

    def host_pinned(self, ptr: int, length: int) -> bool:
        """Whether the codec copies [ptr, ptr + length) by DMA directly (pinned memory)."""
        return bool(self._L.iggy_codec_host_pinned(ptr, length))

    def decode_submit(self, body: np.ndarray, integrity: int, frame_pos: np.ndarray | None = None) -> int:
        """-> ticket. `body` (and `frame_pos`) must stay alive until the ticket completes."""
        t = u64(0)
        cap = frame_pos.size if frame_pos is not None else 0
        rc = self._L.iggy_codec_decode_submit(self._h, _addr(body), body.size, integrity,
                                              frame_pos.ctypes.data if frame_pos is not None else None, cap,
                                              ctypes.byref(t))
        if rc:
            raise CodecError(rc, None, "decode_submit")
        return t.value

    def encode_submit(self, raw: RawMessages, partition_id: int, out: np.ndarray) -> int:
        t = u64(0)
        rc = self._L.iggy_codec_encode_submit(self._h, ctypes.byref(raw), partition_id, out.ctypes.data, out.size,
                                              ctypes.byref(t))
        if rc:
            raise CodecError(rc, None, "encode_submit")
        return t.value

    def poll(self, ticket: int):
        """-> Completion, or None while the operation is in flight (never blocks)."""
        c = Completion()
        rc = self._L.iggy_codec_poll(self._h, ticket, ctypes.byref(c))
        if rc == abi.ERR_PENDING:
            return None
        if rc:
            raise CodecError(rc, None, "poll")
        return c

    def wait(self, ticket: int) -> Completion:
        c = Completion()
        rc = self._L.iggy_codec_wait(self._h, ticket, ctypes.byref(c))
        if rc:
            raise CodecError(rc, None, "wait")
        return c

    def profile_enable(self, on: bool = True):
        self._L.iggy_codec_profile_enable(self._h, 1 if on else 0)

    def profile_read(self, which: int = 0):
        n = u64(0)
        ms = ctypes.c_double(0)
        self._L.iggy_codec_profile_read(self._h, which, ctypes.byref(n), ctypes.byref(ms))
        return n.value, ms.value

    def service_start(self):
        """iggy_codec_service_start: small synchronous host decodes go to resident workgroups."""
        rc = self._L.iggy_codec_service_start(self._h)
        if rc:
            raise CodecError(rc, None, "service_start")

    def service_stop(self):
        rc = self._L.iggy_codec_service_stop(self._h)
        if rc:
            raise CodecError(rc, None, "service_stop")

    def host_stats(self) -> dict:
        """iggy_codec_host_stats: cumulative copy / wait / allocation counters."""
        st = abi.HostStats()
        rc = self._L.iggy_codec_host_stats(self._h, ctypes.byref(st))
        if rc:
            raise CodecError(rc, None, "host_stats")
        return st.as_dict()


PAGE = 4096


def host_buffer(shape, dtype=np.uint8) -> np.ndarray:
    """A zeroed numpy array that starts on a page boundary and owns every page it
    touches (its byte size rounded up to whole pages inside one allocation): a buffer
    iggy_codec_host_register accepts beside any other such buffer (registrations may
    not share a page, include/iggy_codec.h)."""
    dt = np.dtype(dtype)
    n = int(np.prod(shape)) * dt.itemsize
    span = max(PAGE, (n + PAGE - 1) // PAGE * PAGE)
    raw = np.zeros(span + PAGE, dtype=np.uint8)
    off = (-raw.ctypes.data) % PAGE
    return raw[off:off + n].view(dt).reshape(shape)


def page_aligned(a: np.ndarray) -> np.ndarray:
    """A host_buffer copy of `a` (same dtype, shape and bytes)."""
    out = host_buffer(a.shape, a.dtype)
    out[...] = a
    return out


def raw_messages(ids: np.ndarray, origin_timestamps: np.ndarray, payloads: np.ndarray,
                 payload_lengths: np.ndarray, user_headers: np.ndarray | None = None,
                 user_headers_lengths: np.ndarray | None = None) -> RawMessages:
    """Build the SoA `&[RawMessage]` view over host numpy arrays (kept alive by the caller)."""
    n = len(payload_lengths)
    return RawMessages(n, ids.ctypes.data, origin_timestamps.ctypes.data,
                       payloads.ctypes.data if payloads.size else None, payload_lengths.ctypes.data,
                       user_headers.ctypes.data if user_headers is not None and user_headers.size else None,
                       user_headers_lengths.ctypes.data if user_headers_lengths is not None else None)


class Producer:
    """The SDK producer's buffer in front of the GPU encoder (producer_sharding.rs:136-247,
    producer.rs:406-470): append() per send call, flush() -> SendMessages request bodies."""

    def __init__(self, codec: Codec, batch_length: int = 0, batch_size: int = 0, direct: bool = False):
        self._L = codec._L
        self._codec = codec
        cfg = ProducerConfig(batch_length, batch_size, 1 if direct else 0, 0, 0)
        h = vp()
        rc = self._L.iggy_producer_create(codec.handle, ctypes.byref(cfg), ctypes.byref(h))
        if rc:
            raise CodecError(rc, None, "iggy_producer_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.iggy_producer_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def append(self, stream: Identifier, topic: Identifier, part: Partitioning, raw: RawMessages) -> bool:
        due = ci(0)
        rc = self._L.iggy_producer_append(self._h, ctypes.byref(stream), ctypes.byref(topic), ctypes.byref(part),
                                          ctypes.byref(raw), ctypes.byref(due))
        if rc:
            raise CodecError(rc, None, "iggy_producer_append")
        return bool(due.value)

    def pending(self):
        e, b, m = u64(0), u64(0), u64(0)
        self._L.iggy_producer_pending(self._h, ctypes.byref(e), ctypes.byref(b), ctypes.byref(m))
        return e.value, b.value, m.value

    def flush(self, cap: int, max_reqs: int = 4096, out: np.ndarray | None = None, reqs=None):
        """-> (rc, WireError, out bytes, [ProducerRequest]). `reqs`: a caller-owned
        (ProducerRequest * max_reqs) array reused across flushes (the C caller's form)."""
        if out is None:
            out = np.zeros(max(cap, 1), dtype=np.uint8)
        if reqs is None:
            reqs = (ProducerRequest * max(max_reqs, 1))()
        n = u64(0)
        e = WireError()
        rc = self._L.iggy_producer_flush(self._h, out.ctypes.data, cap, reqs, max_reqs, ctypes.byref(n),
                                         ctypes.byref(e))
        return rc, e, out, [reqs[i] for i in range(n.value)]


"""Generate the committed golden fixtures under tests/golden/.

Run in the build container:  python tests/golden/make_golden.py

Two independent sources, neither of them our own C oracle:

1. reference_vectors.json — the Rust-generated golden vectors that the
   reference's own SDK tests hold (copied as data, with their source lines):
   foreign/node/src/wire/message/message-batch.test.ts:47-75 and
   foreign/go/binary_serialization/vsr_response_deserializer_test.go:294.
2. xxh3_vectors.bin/.json and batches/*.bin + cases.json — XXH3-64 values from
   libxxhash 0.8.2 (python `xxhash` 3.8.1, spec-identical to twox-hash 2.1.3's
   XXH3) and batch records assembled by the small pure-Python builder below
   (a second restatement of batch.rs / send_messages.rs, written separately
   from oracle/codec_ref.c), with the outcome the reference semantics dictate
   for each corruption case.
"""
from __future__ import annotations

import json
import os
import struct

import xxhash

HERE = os.path.dirname(os.path.abspath(__file__))
H = 256
F = 48


def det_bytes(n: int, seed: int) -> bytes:
    """splitmix64 byte stream (deterministic, full 0-255 range)."""
    out = bytearray()
    s = seed & 0xFFFFFFFFFFFFFFFF
    while len(out) < n:
        s = (s + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        z ^= z >> 31
        out += struct.pack("<Q", z)
    return bytes(out[:n])


def xxh3(b: bytes) -> int:
    return xxhash.xxh3_64_intdigest(b)


# ---------------------------------------------------------------- builder
def frame(id_: int, offset_delta: int, ts_delta: int, payload: bytes, user_headers: bytes = b"") -> bytes:
    """batch.rs:550-560 / send_messages.rs:148-163."""
    hdr = bytearray(F)
    hdr[8:24] = id_.to_bytes(16, "little")
    struct.pack_into("<IIII", hdr, 24, offset_delta, ts_delta, len(user_headers), len(payload))
    body = bytes(hdr) + payload + user_headers
    cs = xxh3(body[8:])
    return struct.pack("<Q", cs) + body[8:]


def batch_checksum(partition_id, base_offset, base_ts, origin_ts, batch_length, count, frames) -> int:
    """batch.rs:439-459: 44 header bytes || each frame's stored checksum."""
    buf = struct.pack("<QQQQQI", partition_id, base_offset, base_ts, origin_ts, batch_length, count)
    for f in frames:
        buf += f[:8]
    return xxh3(buf)


def record(frames, partition_id=7, base_offset=0, base_ts=0, origin_ts=1_000, count=None,
           checksum=None) -> bytes:
    blob = b"".join(frames)
    n = len(frames) if count is None else count
    bl = H + len(blob)
    cs = batch_checksum(partition_id, base_offset, base_ts, origin_ts, bl, n, frames) if checksum is None else checksum
    hdr = bytearray(H)
    struct.pack_into("<QQQQQQI", hdr, 0, partition_id, base_offset, base_ts, origin_ts, bl, cs, n)
    return bytes(hdr) + blob


def encode_send(messages, partition_id=0):
    """SendMessagesEncoder::encode batch section (send_messages.rs:89-181)."""
    origin = min(m[1] for m in messages)
    frames = []
    for i, (id_, ots, payload, uh) in enumerate(messages):
        frames.append(frame(id_, i, ots - origin, payload, uh))
    return record(frames, partition_id=partition_id, origin_ts=origin)


def main():
    # 1. reference golden vectors (data, with provenance)
    ref = {
        "source_produce": "foreign/node/src/wire/message/message-batch.test.ts:47-60",
        "source_poll": "foreign/node/src/wire/message/message-batch.test.ts:62-75; "
                       "foreign/go/binary_serialization/vsr_response_deserializer_test.go:294",
        "produce_batch_hex": (
            "000000000000000000000000000000000000000000000000e803000000000000"
            "8c01000000000000a91f38c86307267c02000000000000000000000000000000"
            + "00" * 32 * 6 +
            "bfd2b9205a759675070000000000000000000000000000000000000000000000"
            "000000000d000000000000000000000066697273742d7061796c6f6164d66b7e"
            "1c758eb7c0080000000000000000000000000000000100000032000000110000"
            "000e00000000000000000000007365636f6e642d7061796c6f6164757365722d"
            "6865616465722d6279746573"),
        "poll_body_hex": (
            "0300000065000000000000000200000003000000000000006400000000000000"
            "8813000000000000e8030000000000008c01000000000000c96826b38a8feed2"
            "0200000000000000000000000000000000000000000000000000000000000000"
            + "00" * 32 * 5 +
            "00000000000000000000000000000000bfd2b9205a7596750700000000000000"
            "00000000000000000000000000000000000000000d0000000000000000000000"
            "66697273742d7061796c6f6164d66b7e1c758eb7c00800000000000000000000"
            "00000000000100000032000000110000000e0000000000000000000000736563"
            "6f6e642d7061796c6f6164757365722d6865616465722d6279746573"),
        "messages": [
            {"id": 7, "origin_timestamp": 1000, "payload": "first-payload", "user_headers": "",
             "checksum": 0x7596755a20b9d2bf, "offset": 100, "timestamp": 5000},
            {"id": 8, "origin_timestamp": 1050, "payload": "second-payload",
             "user_headers": "user-header-bytes", "checksum": 0xc0b78e751c7e6bd6,
             "offset": 101, "timestamp": 5000},
        ],
        "produce_batch_checksum": 0x7c260763c8381fa9,
        "poll_record_checksum": 0xd2ee8f8ab32668c9,
        "poll_prefix": {"partition_id": 3, "current_offset": 101, "count": 2},
    }
    # self-check the builder against the Rust bytes before trusting it
    msgs = [(m["id"], m["origin_timestamp"], m["payload"].encode(), m["user_headers"].encode())
            for m in ref["messages"]]
    produced = encode_send(msgs)
    assert produced.hex() == ref["produce_batch_hex"], "python builder disagrees with Rust golden"
    with open(os.path.join(HERE, "reference_vectors.json"), "w") as f:
        json.dump(ref, f, indent=1)

    # 2a. XXH3 vectors, every length class the path uses
    lengths = sorted(set(list(range(0, 260)) + [296, 300, 511, 512, 513, 1000, 1023, 1024, 1025,
                                                  1064, 1071, 1088, 1089, 2047, 2048, 2049,
                                                  4136, 8191, 8192, 8193, 65536, 100003]))
    data = det_bytes(max(lengths) + 64, 0x16619E3779B97F4A)
    vecs = []
    blob = bytearray()
    for n in lengths:
        off = len(blob)
        blob += data[n % 7: n % 7 + n]
        vecs.append({"offset": off, "length": n, "xxh3": xxh3(bytes(blob[off:off + n]))})
    with open(os.path.join(HERE, "xxh3_vectors.bin"), "wb") as f:
        f.write(blob)
    with open(os.path.join(HERE, "xxh3_vectors.json"), "w") as f:
        json.dump({"generator": "libxxhash 0.8.2 via python xxhash 3.8.1", "vectors": vecs}, f)

    # 2b. batch records + expected outcome per reference semantics
    os.makedirs(os.path.join(HERE, "batches"), exist_ok=True)
    cases = []

    def add(name, rec: bytes, integrity: int, expect, note, frames=None):
        fn = f"batches/{name}.bin"
        with open(os.path.join(HERE, fn), "wb") as f:
            f.write(rec)
        cases.append({"name": name, "file": fn, "integrity": integrity, "expect": expect,
                      "frames": frames, "note": note})

    def frames_of(fs):
        pos, out = 0, []
        for fr in fs:
            out.append(pos)
            pos += len(fr)
        return out

    ok = {"kind": 0}
    # batch.rs tests, as data
    fs = [frame(1, 0, 0, b"first"), frame(2, 1, 5, b"second")]
    add("two_frames", record(fs), 0, ok, "batch.rs:591-599 decode_verifies_checksums", frames_of(fs))
    fs1 = [frame(1, 0, 0, b"payload")]
    r = bytearray(record(fs1)); r[-1] ^= 0xFF
    stored = struct.unpack_from("<Q", r, H)[0]
    computed = xxh3(bytes(r[H + 8:]))
    add("flipped_body_byte", bytes(r), 0,
        {"kind": 4, "a": stored, "b": computed, "c": 0}, "batch.rs:602-610")
    r = bytearray(record(fs1)); r[40] ^= 0xFF
    stored_b = struct.unpack_from("<Q", r, 40)[0]
    computed_b = batch_checksum(7, 0, 0, 1000, len(r), 1, fs1)
    add("flipped_batch_checksum", bytes(r), 0,
        {"kind": 3, "a": stored_b, "b": computed_b, "c": 0}, "batch.rs:613-620")
    r = bytearray(record(fs1)); r[40:48] = b"\0" * 8
    add("layout_only_zero_checksum", bytes(r), 1, ok, "batch.rs:623-628", frames_of(fs1))
    r = bytearray(record(fs1)); struct.pack_into("<I", r, 48, 2)
    add("miscounted_layout", bytes(r), 1, {"kind": 2, "reason": 3}, "batch.rs:631-636")
    add("miscounted_verify", bytes(record(fs1, count=2)), 0, {"kind": 2, "reason": 3},
        "count error after a clean walk (batch.rs:500-503)")
    rec = record(fs1)
    add("truncated", rec[:-1], 0, {"kind": 1, "a": 0, "b": len(rec), "c": len(rec) - 1},
        "batch.rs:639-642")
    r = bytearray(record(fs1)); r[H + 40] = 1
    add("frame_reserved_nonzero", bytes(r), 1, {"kind": 2, "reason": 3}, "batch.rs:645-649")
    r = bytearray(record(fs1)); r[52] = 1
    add("header_reserved_first", bytes(r), 0, {"kind": 2, "reason": 2}, "batch.rs:653-658")
    r = bytearray(record(fs1)); r[255] = 1
    add("header_reserved_last", bytes(r), 0, {"kind": 2, "reason": 2}, "batch.rs:660-661")
    r = bytearray(record(fs1)); struct.pack_into("<Q", r, 32, 255); r[52] = 1
    add("batch_length_short_before_reserved", bytes(r), 0, {"kind": 2, "reason": 1},
        "batch_length < 256 is checked before reserved (batch.rs:107-123)")
    add("short_header", bytes(100), 0, {"kind": 1, "a": 0, "b": 256, "c": 100}, "batch.rs:99-105")
    add("empty_blob", record([]), 0, ok, "zero frames, count 0", [])
    add("empty_blob_count1", record([], count=1), 0, {"kind": 2, "reason": 3}, "count 1, no frames")
    # trailing bytes past batch_length are allowed (batch.rs:367-372)
    fs = [frame(i + 1, i, i, det_bytes(100, i)) for i in range(5)]
    add("trailing_bytes", record(fs) + b"\x55" * 33, 0, ok, "readers step by batch_length",
        frames_of(fs))
    # precedence: checksum mismatch at frame i beats a layout break at j > i
    fs = [frame(i + 1, i, 0, det_bytes(300, 100 + i)) for i in range(6)]
    r = bytearray(record(fs))
    pos = H + sum(len(f) for f in fs[:2]) + 60
    r[pos] ^= 1  # corrupt frame 2 body
    pos5 = H + sum(len(f) for f in fs[:5]) + 40
    r[pos5] = 9  # frame 5 reserved nonzero -> walk stops there
    f2 = bytes(r[H + sum(len(f) for f in fs[:2]): H + sum(len(f) for f in fs[:3])])
    add("mismatch_beats_layout", bytes(r), 0,
        {"kind": 4, "a": struct.unpack_from("<Q", f2)[0], "b": xxh3(f2[8:]), "c": 2},
        "first mismatch in walk order wins (batch.rs:480-503)")
    # frames beyond message_count are still hashed before the count error
    fs = [frame(i + 1, i, 0, det_bytes(64, 200 + i)) for i in range(4)]
    r = bytearray(record(fs, count=2))
    p3 = H + sum(len(f) for f in fs[:3])
    r[p3 + 50] ^= 0x80
    f3 = bytes(r[p3:p3 + len(fs[3])])
    add("hash_beyond_count", bytes(r), 0,
        {"kind": 4, "a": struct.unpack_from("<Q", f3)[0], "b": xxh3(f3[8:]), "c": 3},
        "frame 3 > count 2 hashed first")
    # message-checksum offset saturates: base_offset near u64::MAX
    fs = [frame(9, 0xFFFFFFFF, 0, b"sat")]
    r = bytearray(record(fs, base_offset=0xFFFFFFFFFFFFFFF0)); r[-1] ^= 1
    fx = bytes(r[H:])
    add("offset_saturates", bytes(r), 0,
        {"kind": 4, "a": struct.unpack_from("<Q", fx)[0], "b": xxh3(fx[8:]),
         "c": 0xFFFFFFFFFFFFFFFF}, "saturating_add (batch.rs:490-493)")
    # every XXH3 length class in one batch (hashed len = 40 + pl + uh)
    pls = [0, 1, 8, 16, 24, 25, 56, 57, 88, 89, 120, 200, 201, 216, 984, 985, 1024, 2008, 2009,
           4096]
    fs = [frame(1000 + i, i, 3 * i, det_bytes(pl, 300 + i), det_bytes(i % 3 * 5, 700 + i))
          for i, pl in enumerate(pls)]
    add("length_classes", record(fs, base_offset=10, base_ts=20), 0, ok,
        "hashed 40..4146 B: 17-128, 129-240 and long paths", frames_of(fs))
    # uniform 1 KiB frames (C2 shape, small N) — exercises the uniform-stride kernel
    fs = [frame(i + 1, i, i, det_bytes(1024, 900 + i)) for i in range(300)]
    add("uniform_1k_300", record(fs, partition_id=1, base_ts=1_700_000_000_001_000,
                                 origin_ts=1_700_000_000_000_000), 0, ok,
        "C2 shape at N=300", frames_of(fs))
    # uniform stride but one frame with a different size in the middle (fast path must bail)
    fs = [frame(i + 1, i, i, det_bytes(256 if i != 77 else 200, 1900 + i)) for i in range(150)]
    add("stride_break", record(fs), 0, ok, "non-uniform frame mid-batch", frames_of(fs))
    # C1 shape: 1000 x 256 B
    fs = [frame(i + 1, i, i, det_bytes(256, 3000 + i)) for i in range(1000)]
    add("c1_1000x256", record(fs), 0, ok, "BASELINE C1 batch shape", frames_of(fs))

    with open(os.path.join(HERE, "cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (xxhash 3.8.1 / libxxhash 0.8.2)",
                   "cases": cases}, f, indent=1)
    print(f"wrote {len(vecs)} xxh3 vectors and {len(cases)} batch cases")


if __name__ == "__main__":
    main()

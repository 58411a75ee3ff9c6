"""GPU parity of the fused admission of a framed request: iggy_frame_read
(message_bus/src/framing.rs:107-164) off a socket straight into an aligned,
registered buffer, then iggy_codec_convert_request (server_common/src/
send_messages.rs:459-540: canonical-batch probe, SendMessagesHeader decode,
admit_wire_request on the GPU), against oracle/sdk_ref.convert_request (the C
restatement's decode and admit under it). Byte work: every output is exact."""
import socket
import struct
import threading

import numpy as np
import pytest

from iggy_amd import abi
from iggy_amd.codec import frame_read, page_aligned, raw_messages
from oracle import oracle as O
from oracle import sdk_ref as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cx():
    from iggy_amd.codec import Codec
    c = Codec(0)
    yield c
    c.close()


def _batch(n, lo, hi, seed, partition_id=0):
    rng = np.random.default_rng(seed)
    pls = rng.integers(lo, hi + 1, size=n).astype(np.uint32)
    ids = rng.integers(1, 2**63, size=2 * n, dtype=np.uint64)
    ots = (1_700_000_000_000_000 + np.arange(n)).astype(np.uint64)
    pay = rng.integers(0, 256, size=int(pls.sum()), dtype=np.uint8)
    rc, e, out = O.encode_batch(raw_messages(ids, ots, pay, pls), partition_id)
    assert rc == 0, e
    return out


def _frame(body: bytes, fill=3) -> bytes:
    hdr = bytearray([fill]) * 256
    struct.pack_into("<I", hdr, 48, 256 + len(body))
    return bytes(hdr) + body


NUM1 = (S.ID_NUMERIC, (1).to_bytes(4, "little"))
NUM2 = (S.ID_NUMERIC, (2).to_bytes(4, "little"))


def _cases():
    wire = [S.send_messages_body(NUM1, NUM2, (S.PART_BALANCED, b""), _batch(n, lo, hi, n), n)
            for n, lo, hi in [(1, 0, 0), (1000, 256, 256), (3000, 1024, 1024), (500, 0, 3000)]]
    out = [("wire", _frame(b)) for b in wire]
    good = wire[1]
    # count mismatch, empty metadata, trailing bytes, a flipped payload byte
    bad = bytearray(good); struct.pack_into("<I", bad, 4 + 18 - 4, 999); out.append(("count", _frame(bytes(bad))))
    out.append(("short", _frame(b"\x01\x00")))
    out.append(("trailing", _frame(good + b"\x00" * 9)))
    bad = bytearray(good); bad[-100] ^= 1; out.append(("msgcs", _frame(bytes(bad))))
    bad = bytearray(good); bad[0] = 200; out.append(("metalen", _frame(bytes(bad))))
    # canonical batches (the encrypt ingest path re-entering): matching / other partition / empty
    canon = _batch(700, 100, 900, 7, partition_id=5)
    out.append(("canon", _frame(canon)))
    out.append(("canon_other_partition", _frame(_batch(700, 100, 900, 7, partition_id=6))))
    bad = bytearray(canon); bad[300] ^= 4; out.append(("canon_corrupt", _frame(bytes(bad))))
    return out


@pytest.mark.parametrize("mode", [0, 1])  # ChecksumMode::{Compute, Skip}
def test_convert_request_matches_oracle(cx, mode):
    for name, frame in _cases():
        rc, e, h, out = cx.convert_request(np.frombuffer(frame, dtype=np.uint8), 5, mode)
        orc, oe, oout = S.convert_request(frame, 5, mode)
        assert rc == orc, (name, e.astuple(), oe)
        assert tuple(e.astuple()) == tuple(oe), name
        assert out == oout, name


def test_socket_frame_to_admitted_batch(cx):
    """A producer's framed request arrives over a stream socket in pieces: read into a
    registered aligned buffer, admitted on the GPU, exact."""
    frames = [f for name, f in _cases() if name in ("wire", "canon")]
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_STREAM)
    try:
        def send():
            data = b"".join(frames)
            for i in range(0, len(data), 65_000):
                a.sendall(data[i:i + 65_000])
        t = threading.Thread(target=send)
        t.start()
        for f in frames:
            rc, e, buf = frame_read(b.fileno(), 8 << 20)
            assert rc == 0 and buf.tobytes() == f
            buf = page_aligned(buf)  # (registrations may not share a page)
            cx.host_register(buf)
            try:
                rc, e, h, out = cx.convert_request(buf, 5, 0)
            finally:
                cx.host_unregister(buf)
            orc, oe, oout = S.convert_request(f, 5, 0)
            assert rc == orc == 0 and out == oout
        t.join()
    finally:
        a.close()
        b.close()

"""The server socket side: read_message
(core/message_bus/src/framing.rs:107-171) through the C ABI on a socketpair, no
GPU. The reference's own framing tests (framing.rs `mod tests`) exercise the same
cases: a body frame, a header-only frame, sizes outside [256, max], EOF inside the
header or the body, several frames back to back on one stream."""
import socket
import struct
import threading

import numpy as np
import pytest

from iggy_amd import abi
from iggy_amd.codec import frame_read


def _frame(body: bytes, size=None, fill=7) -> bytes:
    hdr = bytearray([fill]) * 256
    struct.pack_into("<I", hdr, 48, 256 + len(body) if size is None else size)
    return bytes(hdr) + body


def _send(sock, data: bytes, close=True, chunk=997):
    def run():
        for i in range(0, len(data), chunk):  # arrives in pieces, as on a real stream
            sock.sendall(data[i:i + chunk])
        if close:
            sock.shutdown(socket.SHUT_WR)
    t = threading.Thread(target=run)
    t.start()
    return t


@pytest.fixture
def pair():
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_STREAM)
    yield a, b
    a.close()
    b.close()


def test_body_and_header_only_frames_back_to_back(pair):
    a, b = pair
    rng = np.random.default_rng(1)
    bodies = [rng.integers(0, 256, 70_000, dtype=np.uint8).tobytes(), b"", b"x" * 3]
    t = _send(a, b"".join(_frame(x, fill=k + 1) for k, x in enumerate(bodies)))
    for k, body in enumerate(bodies):
        rc, e, buf = frame_read(b.fileno(), 1 << 17)
        assert rc == 0, e.astuple()
        assert buf.ctypes.data % 4096 == 0  # the body lands in the same aligned buffer as the header
        assert buf.tobytes() == _frame(body, fill=k + 1)
    t.join()
    rc, e, buf = frame_read(b.fileno(), 1 << 17)  # the peer closed: no next frame
    assert rc == abi.ERR_CONNECTION_CLOSED


@pytest.mark.parametrize("size", [0, 255, (64 << 20) + 1])
def test_size_outside_bounds_is_invalid_command(pair, size):
    a, b = pair
    t = _send(a, _frame(b"", size=size))
    rc, e, _ = frame_read(b.fileno(), 1 << 16)
    assert rc == abi.ERR_INVALID_COMMAND and e.kind == abi.ERR_INVALID_COMMAND
    t.join()


def test_max_message_size_is_the_callers(pair):
    a, b = pair
    t = _send(a, _frame(b"y" * 1000))
    rc, e, _ = frame_read(b.fileno(), 1 << 16, max_message_size=1255)
    assert rc == abi.ERR_INVALID_COMMAND
    t.join()


@pytest.mark.parametrize("cut", [0, 100, 255, 256, 300])
def test_eof_inside_the_frame_is_connection_closed(pair, cut):
    a, b = pair
    t = _send(a, _frame(b"z" * 500)[:cut])
    rc, e, _ = frame_read(b.fileno(), 1 << 16)
    assert rc == abi.ERR_CONNECTION_CLOSED
    t.join()


def test_frame_larger_than_the_buffer(pair):
    a, b = pair
    t = _send(a, _frame(b"w" * 5000))
    rc, e, _ = frame_read(b.fileno(), 4096)
    assert rc == abi.ERR_CAPACITY and e.a == 5256
    t.join()


def test_closed_descriptor_is_tcp_error():
    a, b = socket.socketpair()
    fd = b.detach()
    import os
    os.close(fd)
    a.close()
    rc, e, _ = frame_read(fd, 4096)
    assert rc == abi.ERR_TCP_ERROR


def test_frame_larger_than_the_buffer_resumes(pair):
    """IGGY_ERR_CAPACITY leaves the body on the socket: the caller grows its buffer and
    finishes the frame (iggy_frame_read_rest); the next frame then reads normally."""
    a, b = pair
    frames = [_frame(b"w" * 5000), _frame(b"v" * 10)]
    t = _send(a, b"".join(frames))
    rc, e, buf = frame_read(b.fileno(), 4096, grow=True)
    assert rc == 0 and buf.tobytes() == frames[0] and buf.ctypes.data % 4096 == 0
    rc, e, buf = frame_read(b.fileno(), 4096)
    assert rc == 0 and buf.tobytes() == frames[1]
    t.join()


@pytest.mark.parametrize("command", [0, 5, 29, 30, 99, 255])
def test_header_bit_pattern_checked_after_the_body(pair, command):
    """Message::<GenericHeader>::try_from (consensus_message.rs:468-500): the command
    byte at offset 60 must be a Command discriminant (command.rs:90-95, <= 29); a bad one
    is InvalidCommand once the whole frame is read, so the next frame stays readable.
    Checked against the stream restatement oracle/sdk_ref.read_frames."""
    from oracle import sdk_ref as S
    a, b = pair
    bad = bytearray(_frame(b"q" * 3000)); bad[60] = command
    hdr_only = bytearray(_frame(b"")); hdr_only[60] = command
    good = _frame(b"r" * 77)
    stream = bytes(bad) + bytes(hdr_only) + good
    want = S.read_frames(stream, 1 << 16)
    t = _send(a, stream)
    for rc_want, frame_want, _ in want:
        rc, e, buf = frame_read(b.fileno(), 1 << 16)
        assert rc == rc_want and e.kind == rc_want
        assert buf.tobytes() == frame_want
    t.join()
    assert [w[0] for w in want][:3] == ([abi.ERR_INVALID_COMMAND] * 2 if command > 29 else [0, 0]) + [0]


def test_random_streams_match_the_restatement():
    """Fuzz: random frame sequences (sizes inside and outside the bounds, bad commands,
    frames above the buffer, a truncated tail) through the C reader and the restatement."""
    from oracle import sdk_ref as S
    rng = np.random.default_rng(44)
    for trial in range(60):
        parts = []
        for _ in range(int(rng.integers(1, 6))):
            body = rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()
            f = bytearray(_frame(body))
            if rng.random() < 0.2:
                f[60] = int(rng.integers(0, 256))
            if rng.random() < 0.1:
                struct.pack_into("<I", f, 48, int(rng.integers(0, 400)))
            parts.append(bytes(f))
        stream = b"".join(parts)
        if rng.random() < 0.3:
            stream = stream[: int(rng.integers(0, len(stream) + 1))]
        cap = int(rng.choice([512, 2048, 1 << 16]))
        want = S.read_frames(stream, cap, max_message_size=1 << 20)
        a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_STREAM)
        try:
            t = _send(a, stream)
            for k, (rc_want, frame_want, _) in enumerate(want):
                if rc_want == abi.ERR_CAPACITY:  # grow=True finishes that frame in the next call
                    continue
                rc, e, buf = frame_read(b.fileno(), cap, max_message_size=1 << 20, grow=True)
                assert rc == rc_want, (trial, k)
                assert buf.tobytes() == frame_want
            t.join()
        finally:
            a.close()
            b.close()

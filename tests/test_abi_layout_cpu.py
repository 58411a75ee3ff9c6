"""The ctypes mirrors in iggy_amd/abi.py against the C header itself: gcc compiles a
probe that prints sizeof and every field's offsetof for each struct of
include/iggy_codec.h, and each mirror must agree field by field (no GPU needed)."""
import ctypes
import os
import shutil
import subprocess
import tempfile

import pytest

from iggy_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "iggy_codec.h")

# ctypes mirror -> C typedef
PAIRS = {
    abi.WireError: "iggy_wire_error",
    abi.BatchHeader: "iggy_batch_header",
    abi.PolledMessage: "iggy_polled_message",
    abi.RawMessages: "iggy_raw_messages",
    abi.DecodeResult: "iggy_decode_result",
    abi.EncodeResult: "iggy_encode_result",
    abi.SliceQuery: "iggy_slice_query",
    abi.SliceResult: "iggy_slice_result",
    abi.Completion: "iggy_completion",
    abi.HostStats: "iggy_host_stats",
    abi.SegmentRecovery: "iggy_segment_recovery",
    abi.ChunkFragment: "iggy_chunk_fragment",
    abi.ChunkWalk: "iggy_chunk_walk",
    abi.SegmentWalk: "iggy_segment_walk",
    abi.CryptResult: "iggy_crypt_result",
    abi.Identifier: "iggy_identifier",
    abi.Partitioning: "iggy_partitioning",
    abi.SendMessagesHeader: "iggy_send_messages_header",
    abi.PolledPrefix: "iggy_polled_prefix",
    abi.ProducerConfig: "iggy_producer_config",
    abi.ProducerRequest: "iggy_producer_request",
    abi.PollFragment: "iggy_poll_fragment",
}


def _fields(cls):
    out = []
    for klass in reversed(cls.__mro__):
        out.extend(getattr(klass, "_fields_", []) if "_fields_" in vars(klass) else [])
    return [f[0] for f in out]


@pytest.fixture(scope="module")
def c_layout():
    cc = shutil.which("gcc")
    if not cc:
        pytest.skip("no gcc")
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for cls, cname in PAIRS.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f in _fields(cls):
            lines.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines += ["return 0;", "}"]
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "probe.c"), os.path.join(d, "probe")
        with open(src, "w") as f:
            f.write("\n".join(lines))
        subprocess.run([cc, "-std=c11", "-o", exe, src], check=True, capture_output=True)
        text = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    got = {}
    for ln in text.splitlines():
        cname, what, val = ln.split()
        got[(cname, what)] = int(val)
    return got


@pytest.mark.parametrize("cls", list(PAIRS), ids=lambda c: c.__name__)
def test_mirror_matches_header(cls, c_layout):
    cname = PAIRS[cls]
    assert ctypes.sizeof(cls) == c_layout[(cname, "size")], cname
    for f in _fields(cls):
        assert getattr(cls, f).offset == c_layout[(cname, f)], (cname, f)

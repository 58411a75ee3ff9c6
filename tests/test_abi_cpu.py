"""CPU-only checks of the C-ABI library: it loads, exports every symbol the
header declares, refuses to run without a gfx950 device, and its pure-host
header codec agrees with the oracle (no device compute here)."""
import ctypes
import os

import numpy as np
import pytest

from golden_util import batch_cases
from iggy_amd import abi, codec
from oracle import oracle as O


def test_library_exports_every_declared_symbol():
    L = codec.lib()
    names = codec.exported_symbols()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert L.iggy_codec_abi_version() == 1


def test_no_device_means_no_codec():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(codec.CodecError) as ei:
        codec.Codec(0)
    assert ei.value.rc == abi.ERR_DEVICE


@pytest.mark.parametrize("case", batch_cases(), ids=lambda c: c["name"])
def test_host_header_decode_matches_oracle(case):
    L = codec.lib()
    d = case["data"]
    h1, e1, h2, e2 = abi.BatchHeader(), abi.WireError(), abi.BatchHeader(), abi.WireError()
    r1 = L.iggy_batch_header_decode(d.ctypes.data if d.size else None, d.size, ctypes.byref(h1), ctypes.byref(e1))
    r2 = O.lib().oracle_batch_header_decode(d.ctypes.data if d.size else None, d.size, ctypes.byref(h2), ctypes.byref(e2))
    assert r1 == r2
    assert e1.astuple() == e2.astuple()
    if r1 == 0:
        assert h1.astuple() == h2.astuple()
        out = np.zeros(256, dtype=np.uint8)
        L.iggy_batch_header_encode(ctypes.byref(h1), out.ctypes.data)
        assert out.tobytes() == bytes(d[:256])


def test_error_strings():
    L = codec.lib()
    assert L.iggy_codec_error_string(abi.ERR_VALIDATION, abi.V_FRAMES_DO_NOT_TILE) == \
        b"batch frames do not tile message_count exactly"

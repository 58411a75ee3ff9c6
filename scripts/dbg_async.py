"""Diagnostic: the asynchronous single-stride fast path on a stride-breaking record."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iggy_amd import abi  # noqa: E402
from iggy_amd.codec import Codec  # noqa: E402
from oracle import oracle as O  # noqa: E402
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_hostmem_gpu import _stride_break_record  # noqa: E402

cx = Codec(0)
r = _stride_break_record()
orc, oe, oh, of = O.decode_batch_slice_with(r, 0)
print("oracle", orc, len(of))
p = np.zeros(r.size // 48 + 1, dtype=np.uint64)
print("sync", cx.decode_batch_into(r, abi.INTEGRITY_VERIFY, p))
for wp in (True, False):
    for rep in range(3):
        c = cx.wait(cx.decode_submit(r, abi.INTEGRITY_VERIFY, p if wp else None))
        print("async pos", wp, "frames", c.frame_count, "err", c.error.kind, "cs", hex(c.computed_checksum))

"""Diagnostic: stage times of the synchronous host decode of C1-shaped records
(diagnostic build, IGGY_CODEC_TIMING), pageable and registered, plus the floor of a
tiny record, on the launch path and through the resident service. Not part of the bench/tests."""
import os
import sys
import time

import numpy as np

os.environ["IGGY_CODEC_TIMING"] = "200"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iggy_amd import abi  # noqa: E402
from iggy_amd import codec as _codec  # noqa: E402
_codec.use_library(os.environ.get("IGGY_DIAG_LIB", _codec.DIAG_LIB_PATH))
from iggy_amd.codec import Codec, host_buffer, page_aligned  # noqa: E402
from oracle import oracle as O  # noqa: E402


def run(cx, rec, label, reg, svc=False):
    rec = page_aligned(rec)  # (registrations may not share a page)
    pos = host_buffer(rec.size // 48 + 1, np.uint64)
    if reg:
        cx.host_register(rec)
        cx.host_register(pos)
    if svc:
        cx.service_start()
    for _ in range(200):
        rc, nf = cx.decode_batch_into(rec, abi.INTEGRITY_VERIFY, pos)
    t = time.perf_counter()
    for _ in range(200):
        rc, nf = cx.decode_batch_into(rec, abi.INTEGRITY_VERIFY, pos)
    us = (time.perf_counter() - t) / 200 * 1e6
    if svc:
        cx.service_stop()
    print(f"{label} service={svc}: rc {rc} frames {nf} {us:.1f} us per call", flush=True)
    if reg:
        cx.host_unregister(pos)
        cx.host_unregister(rec)


def main():
    cx = Codec(0)
    c1 = O.synth_batch(1000, 256, seed=1)
    tiny = O.synth_batch(4, 256, seed=2)
    for svc in (False, True):
        for reg in (False, True):
            run(cx, c1, f"C1 registered={reg}", reg, svc)
            run(cx, tiny, f"4 msgs registered={reg}", reg, svc)


if __name__ == "__main__":
    main()

"""The resident decode service (iggy_codec_service_start) against the launch path
(diagnostic, not part of the bench): synchronous iggy_codec_decode_batch of C1 records
(1 000 x 256 B, registered and pageable) and a 4-message record, per-call wall time; then
the C2 device decode (1 M x 1 KiB) with and without the service grid resident beside it.

usage: python scripts/svc_timing.py
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from iggy_amd import abi  # noqa: E402
from iggy_amd.codec import Codec, host_buffer, page_aligned  # noqa: E402
from oracle import oracle as O  # noqa: E402  (checker)
import bench  # noqa: E402


def per_call(cx, rec, pos, reps=300):
    for _ in range(20):
        rc, nf = cx.decode_batch_into(rec, abi.INTEGRITY_VERIFY, pos)
        assert rc == 0
    t = time.perf_counter()
    for _ in range(reps):
        cx.decode_batch_into(rec, abi.INTEGRITY_VERIFY, pos)
    return (time.perf_counter() - t) / reps * 1e6


def main():
    torch.cuda.set_device(0)
    cx = Codec(0)
    out = {}
    c1 = page_aligned(O.synth_batch(1000, 256, seed=1))
    tiny = page_aligned(O.synth_batch(4, 256, seed=2))
    for name, rec in (("c1", c1), ("tiny", tiny)):
        want = O.decode_batch_slice_with(rec, 0)
        pos = host_buffer(rec.size // 48 + 1, np.uint64)
        for reg in (False, True):
            if reg:
                cx.host_register(rec)
                cx.host_register(pos)
            for svc in (False, True):
                if svc:
                    cx.service_start()
                us = per_call(cx, rec, pos)
                rc, nf = cx.decode_batch_into(rec, abi.INTEGRITY_VERIFY, pos)
                assert rc == want[0] == 0 and np.array_equal(pos[:nf], np.asarray(want[3], dtype=np.uint64))
                if svc:
                    cx.service_stop()
                out[f"{name}_{'reg' if reg else 'pag'}_{'svc' if svc else 'launch'}_us"] = round(us, 2)
            if reg:
                cx.host_unregister(pos)
                cx.host_unregister(rec)
    out["stats"] = cx.host_stats()
    # C2 device decode beside a resident service grid (another context's, kept alive)
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream()
    batch = bench.make_batch(cx, 1 << 20, 1024, 1024, 0, dev, s.cuda_stream)[0]
    L = batch.numel()
    cx.reserve(L)
    d_res = torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device=dev)
    d_pos = torch.empty(1 << 20, dtype=torch.int64, device=dev)
    other = Codec(0)

    def c2_ms(steps=10):
        for _ in range(2):
            assert cx.decode_device(batch.data_ptr(), L, 0, d_pos.data_ptr(), 1 << 20, d_res.data_ptr(), s.cuda_stream) == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(steps):
            assert cx.decode_device(batch.data_ptr(), L, 0, d_pos.data_ptr(), 1 << 20, d_res.data_ptr(), s.cuda_stream) == 0
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / steps

    out["c2_ms_alone"] = round(c2_ms(), 4)
    other.service_start()
    rc, nf = other.decode_batch_into(c1, abi.INTEGRITY_VERIFY, host_buffer(c1.size // 48 + 1, np.uint64))
    assert rc == 0
    out["c2_ms_beside_service"] = round(c2_ms(), 4)
    other.service_stop()
    out["c2_ms_after_stop"] = round(c2_ms(), 4)
    other.close()
    cx.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

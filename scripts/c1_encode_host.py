"""Diagnostic: the C1 producer side through the host API. iggy_codec_encode_submit of
C1 batches (1 000 x 256 B, SoA input in host memory, wire bytes back into host memory),
8 in flight, registered and pageable buffers, against the oracle's single-thread
encode of the same batches (the CPU leg). Every GPU output is compared byte for byte
with the oracle's. One JSON line.

usage: python scripts/c1_encode_host.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (the HIP runtime the codec shares)
from iggy_amd import codec as _codec  # noqa: E402
if os.environ.get("IGGY_LIB"):  # a library build to compare (same-box A/B)
    _codec.use_library(os.environ["IGGY_LIB"])
from iggy_amd.codec import Codec, host_buffer, page_aligned, raw_messages  # noqa: E402
from oracle import oracle as O  # noqa: E402  (the CPU leg and the check)


def main():
    nb, n, pl = 10, 1000, 256
    rng = np.random.default_rng(5)
    soas, raws, wants = [], [], []
    for b in range(nb):
        ids = rng.integers(1, 2**63, size=2 * n, dtype=np.uint64)
        ots = (1_700_000_000_000_000 + b * n + np.arange(n)).astype(np.uint64)
        pay = rng.integers(0, 256, size=n * pl, dtype=np.uint8)
        pls = np.full(n, pl, dtype=np.uint32)
        ids, ots, pay, pls = (page_aligned(a) for a in (ids, ots, pay, pls))
        soas.append((ids, ots, pay, pls))
        raws.append(raw_messages(ids, ots, pay, pls))
        rc, e, out = O.encode_batch(raws[-1], 0)
        assert rc == 0
        wants.append(np.frombuffer(out, dtype=np.uint8))
    size = wants[0].size
    outs = [host_buffer(size) for _ in range(nb)]  # (registrations may not share a page)
    cx = Codec(0)

    def run(reps):
        t = time.perf_counter()
        sub = 0.0
        for _ in range(reps):
            for lo in (0, 8):
                c0 = time.thread_time()
                tks = [cx.encode_submit(raws[b], 0, outs[b]) for b in range(lo, min(lo + 8, nb))]
                sub += time.thread_time() - c0
                for tk in tks:
                    c = cx.wait(tk)
                    assert c.error.kind == 0, c.error
        return (time.perf_counter() - t) / (reps * nb) * 1e6, sub / (reps * nb) * 1e6

    def sync(reps):
        t = time.perf_counter()
        for _ in range(reps):
            for b in range(nb):
                rc, e, o = cx.encode_batch(raws[b], 0)
                assert rc == 0, e
        return (time.perf_counter() - t) / (reps * nb) * 1e6

    line = {"batch_bytes": int(size)}
    rc, e, o = cx.encode_batch(raws[0], 0)
    assert rc == 0 and np.array_equal(np.frombuffer(o, dtype=np.uint8), wants[0])
    sync(1)
    line["sync_pageable_us_per_batch_incl_python"] = round(sync(10), 1)
    run(1)
    line["pageable_us_per_batch"], line["pageable_submit_cpu_us"] = [round(x, 1) for x in run(10)]
    assert all(np.array_equal(o, w) for o, w in zip(outs, wants))
    arrs = [a for s in soas for a in s] + outs
    for a in arrs:
        cx.host_register(a)
    try:
        run(1)
        line["registered_us_per_batch"], line["registered_submit_cpu_us"] = [round(x, 1) for x in run(10)]
        assert all(np.array_equal(o, w) for o, w in zip(outs, wants))
    finally:
        for a in arrs:
            cx.host_unregister(a)
    reps = 200
    t = time.perf_counter()
    for _ in range(reps // nb):
        for r in raws:
            O.encode_batch(r, 0)
    line["cpu_oracle_encode_us_per_batch_incl_python"] = round((time.perf_counter() - t) / reps * 1e6, 1)
    secs = sum(O.cpu_encode_bench(r, 0, 1, 20)[0] for r in raws)
    line["cpu_ref_encode_us_per_batch"] = round(secs / (20 * nb) * 1e6, 1)
    print(json.dumps(line), flush=True)
    cx.close()


if __name__ == "__main__":
    main()

"""CPU/GPU crossover of the host-buffer decode (the GPU_MIN_BYTES threshold of the
Rust dispatcher): for records of 1 KiB messages from 64 KiB to
64 MiB, the median time of iggy_codec_decode_batch (host buffer in, frame positions
out: H2D + kernels + D2H) against the CPU oracle's single-thread decode (the
reference's execution model: one shard thread walks one batch), both sides with the
same --integrity (0 = Verify, the hash walk of batch.rs:474-506; 1 = LayoutOnly,
batch.rs:508-527), which every row names. One JSON line per size, then the crossover.
Diagnostic / documentation only (oracle = the CPU leg).

usage: python scripts/crossover.py [--integrity 0|1]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from iggy_amd import codec as _codec  # noqa: E402
if os.environ.get("IGGY_LIB"):  # a library build to compare (same-box A/B)
    _codec.use_library(os.environ["IGGY_LIB"])
from iggy_amd.codec import Codec, host_buffer, page_aligned  # noqa: E402
from oracle import oracle as O  # noqa: E402  (the CPU leg)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--integrity", type=int, default=0)
    ap.add_argument("--registered", action="store_true",
                    help="register the record and the positions array first (records <= 1 MiB read in place)")
    args = ap.parse_args()
    cx = Codec(0)
    rows = []
    for kib in (64, 256, 1024, 2048, 4096, 16384, 65536):
        n = max(1, kib * 1024 // 1072)
        rec = page_aligned(O.synth_batch(n, 1024, 1024, seed=kib))  # (registrations may not share a page)
        pos = host_buffer(rec.size // 48 + 1, np.uint64)
        if args.registered:
            cx.host_register(rec)
            cx.host_register(pos)
        for _ in range(3):
            rc, nf = cx.decode_batch_into(rec, args.integrity, pos)
            assert rc == 0 and nf == n, rc
        ts = []
        for _ in range(15):
            t0 = time.perf_counter()
            cx.decode_batch_into(rec, args.integrity, pos)
            ts.append(time.perf_counter() - t0)
        gpu = float(np.median(ts))
        if args.registered:
            cx.host_unregister(pos)
            cx.host_unregister(rec)
        reps = max(1, int(0.2 / max(rec.size / 3e9, 1e-6)))
        # one thread walks `reps` copies with the GPU leg's integrity
        secs, _ = O.cpu_decode_bench(rec, 1, reps, args.integrity)
        cpu = secs / reps
        row = {"record_bytes": int(rec.size), "messages": n, "integrity_gpu": args.integrity,
               "integrity_cpu": args.integrity, "registered": args.registered,
               "gpu_host_decode_us": round(gpu * 1e6, 1), "cpu_1thread_us": round(cpu * 1e6, 1),
               "gpu_faster": gpu < cpu}
        rows.append(row)
        print(json.dumps(row), flush=True)
    cross = next((r["record_bytes"] for r in rows if r["gpu_faster"]), None)
    print(json.dumps({"crossover_record_bytes": cross, "integrity": args.integrity,
                      "registered": args.registered}), flush=True)


if __name__ == "__main__":
    main()

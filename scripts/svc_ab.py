"""Same-box A/B(/C...) of builds of the codec library on the synchronous service call
(diagnostic, not part of the bench): iggy_codec_decode_batch of a C1 record (1 000 x
256 B, registered) with the resident service started, timed from C
(scripts/_c_loop.so, the bench's sync C loop), the libraries interleaved round by round
in one process, each library's service started and stopped within its own round. Every
call's result is checked by the loop (rc, frame count); the positions once per round
against the oracle.

usage: python scripts/svc_ab.py <lib A .so> <lib B .so> [...] [--rounds 8] [--reps 300] [--gap-us G]
(--gap-us: sparse posts, G us of idle spin between calls, each call timed alone from Python)
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from iggy_amd import abi  # noqa: E402
from iggy_amd.codec import Codec, host_buffer, load, page_aligned  # noqa: E402
from oracle import oracle as O  # noqa: E402  (checker)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--reps", type=int, default=300)
    ap.add_argument("--gap-us", type=float, default=0.0)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    c_loop = ctypes.CDLL(os.path.join(ROOT, "scripts", "_c_loop.so"))
    c_loop.c_loop_decode.restype = ctypes.c_double
    c_loop.c_loop_decode.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_void_p, ctypes.c_void_p,
                                                             ctypes.c_int, ctypes.c_int, ctypes.c_int]
    src = O.synth_batch(1000, 256, seed=1)
    want = O.decode_batch_slice_with(src, 0)
    ctxs = [Codec(0, library=load(p)) for p in args.libs]
    bufs = []  # each library registers its own copy (a range registers once per process)
    for cx in ctxs:
        rec = page_aligned(src)
        pos = host_buffer(rec.size // 48 + 1, np.uint64)
        cx.host_register(rec)
        cx.host_register(pos)
        bufs.append((rec, pos))
    P = ctypes.c_void_p * 1
    U = ctypes.c_uint64 * 1
    res = {p: [] for p in args.libs}
    for r in range(args.rounds):
        order = list(zip(args.libs, ctxs, bufs))
        if r % 2:
            order.reverse()
        for p, cx, (rec, pos) in order:
            cx.service_start()
            a = (ctypes.cast(cx._L.iggy_codec_decode_batch, ctypes.c_void_p), cx._h,
                 P(rec.ctypes.data), U(rec.size), P(pos.ctypes.data), U(pos.size), U(len(want[3])), 1,
                 abi.INTEGRITY_VERIFY)
            assert c_loop.c_loop_decode(*a, 20) > 0
            if args.gap_us > 0:
                ts = []
                for _ in range(args.reps // 4):
                    t_end = time.perf_counter() + args.gap_us * 1e-6
                    while time.perf_counter() < t_end:
                        pass
                    t0 = time.perf_counter()
                    rc, nf = cx.decode_batch_into(rec, abi.INTEGRITY_VERIFY, pos)
                    ts.append(time.perf_counter() - t0)
                    assert rc == 0
                ns = statistics.median(ts) * 1e9
            else:
                ns = c_loop.c_loop_decode(*a, args.reps)
            assert ns > 0, ns
            rc, nf = cx.decode_batch_into(rec, abi.INTEGRITY_VERIFY, pos)
            assert rc == 0 and np.array_equal(pos[:nf], np.asarray(want[3], dtype=np.uint64)), p
            cx.service_stop()
            res[p].append(ns / 1e3)
    out = {os.path.basename(p): {"median_us": round(statistics.median(v), 2), "min_us": round(min(v), 2),
                                 "rounds": [round(x, 2) for x in v]} for p, v in res.items()}
    print(json.dumps(out), flush=True)
    for cx, (rec, pos) in zip(ctxs, bufs):
        cx.host_unregister(pos)
        cx.host_unregister(rec)
        cx.close()


if __name__ == "__main__":
    main()

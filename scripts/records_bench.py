"""Multi-record walks over host buffers (diagnostic / documentation; the oracle is the
CPU leg): the one-launch paths against the oracle's single-thread walks (the
reference's execution model: one shard thread walks the chunk or segment).

  chunk : walk_disk_chunk over a 1 MiB disk-poll chunk (poll_plan.rs:484) of C1
          producer batches (1 000 x 256 B), Verify, whole-chunk query
  poll  : poll_decode (SDK mode) of the same 1 MiB as a poll response body
  seg   : walk_segment_payload (state_transfer.rs:715-833) of a segment of C1 batches
  crossover: iggy_codec_decode_batch of one record of 1 KiB messages, registered
          host buffer, 64 KiB .. 16 MiB

Every GPU path takes host buffers registered once with iggy_codec_host_register
(the server's 4096-aligned pool) and is timed end to end (H2D,
kernels, D2H, sync). One JSON line per measurement.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401  (the HIP runtime the tests and bench use)
from iggy_amd import abi  # noqa: E402
from iggy_amd import codec as _codec  # noqa: E402
if os.environ.get("IGGY_LIB"):  # a library build to compare (same-box A/B)
    _codec.use_library(os.environ["IGGY_LIB"])
from iggy_amd.codec import Codec  # noqa: E402
from oracle import oracle as O  # noqa: E402  (the CPU leg)


def c1_records(nbatches, base_offset=0):
    import test_records_gpu as T
    base = T._record([256] * 1000, 7, 0, 1)
    out, off = [], base_offset
    for k in range(nbatches):
        rc, e, h, st = O.stamp_batch(base, off, 10 + k)
        out.append(np.frombuffer(st, dtype=np.uint8))
        off += 1000
    return out


def pinned_copy(a):
    """A page-aligned copy (the server's Owned<4096> buffers)."""
    raw = np.empty(a.size + 8192, dtype=np.uint8)
    off = (-raw.ctypes.data) % 4096
    b = raw[off: off + a.size]
    b[:] = a
    return b


def med(f, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    cx = Codec(0)
    what = sys.argv[1:] or ["chunk", "poll", "seg", "crossover"]
    if "chunk" in what or "poll" in what:
        recs = c1_records(3)
        tail = c1_records(1, 3000)[0][: (1 << 20) - 3 * recs[0].size]  # a torn last batch, as a chunk read ends
        chunk = pinned_copy(np.concatenate(recs + [tail]))
        cx.host_register(chunk)
        for integ in (0, 1):
            args = (abi.LOOKUP_OFFSET, 0, 10**9, 2**64 - 1, 0, integ)
            rc, w, fr, hd = cx.walk_disk_chunk(chunk, *args)
            orc, ow, ofr, ohd = O.walk_disk_chunk(chunk, *args)
            assert rc == orc and w.astuple() == ow.astuple(), (w.astuple(), ow.astuple())
            g = med(lambda: cx.walk_disk_chunk(chunk, *args), 200)
            c = med(lambda: O.walk_disk_chunk(chunk, *args), 200)
            print(json.dumps({"path": "walk_disk_chunk", "integrity": integ, "chunk_bytes": int(chunk.size),
                              "batches": int(w.batches), "gpu_us": round(g * 1e6, 1), "cpu_1thread_us": round(c * 1e6, 1),
                              "gpu_faster": g < c}), flush=True)
        body = chunk[: 3 * recs[0].size]
        rc, e, msgs = cx.poll_decode(body, 0)
        orc, oe, om = O.poll_decode(body, 0)
        assert rc == orc == 0 and len(msgs) == len(om)
        g = med(lambda: cx.poll_decode(body, 0), 100)
        c = med(lambda: O.poll_decode(body, 0), 100)
        print(json.dumps({"path": "poll_decode(SDK)", "body_bytes": int(body.size), "messages": len(msgs),
                          "gpu_us": round(g * 1e6, 1), "cpu_1thread_us": round(c * 1e6, 1), "gpu_faster": g < c}),
              flush=True)
        # the same two calls without the binding's per-call output allocation and list
        # building: preallocated descriptor arrays, the C entry points called directly
        import ctypes
        cap = body.size // 48 + 1
        gout, oout = (abi.PolledMessage * cap)(), (abi.PolledMessage * cap)()
        n1, n2, e1, e2 = abi.u64(0), abi.u64(0), abi.WireError(), abi.WireError()
        gcall = lambda: cx._L.iggy_codec_poll_decode(cx.handle, body.ctypes.data, body.size, 0, gout, cap,  # noqa: E731
                                                    ctypes.byref(n1), ctypes.byref(e1))
        ocall = lambda: O.lib().oracle_poll_decode(body.ctypes.data, body.size, 0, oout, cap,  # noqa: E731
                                                  ctypes.byref(n2), ctypes.byref(e2))
        assert gcall() == 0 and ocall() == 0 and n1.value == n2.value == len(msgs)
        g = med(gcall, 200)
        c = med(ocall, 200)
        print(json.dumps({"path": "poll_decode(SDK), C calls", "body_bytes": int(body.size), "messages": len(msgs),
                          "gpu_us": round(g * 1e6, 1), "cpu_1thread_us": round(c * 1e6, 1), "gpu_faster": g < c}),
              flush=True)
        cx.host_unregister(chunk)
    if "seg" in what:
        for nb in (4, 64, 1024):
            seg = pinned_copy(np.concatenate(c1_records(nb)))
            cx.host_register(seg)
            rc, w, idx = cx.walk_segment_payload(seg, 0)
            orc, ow, oidx = O.walk_segment_payload(seg, 0)
            assert rc == orc and w.astuple() == ow.astuple()
            reps = 20 if nb < 1024 else 5
            g = med(lambda: cx.walk_segment_payload(seg, 0), reps)
            c = med(lambda: O.walk_segment_payload(seg, 0), reps)
            print(json.dumps({"path": "walk_segment_payload", "segment_bytes": int(seg.size), "batches": nb,
                              "gpu_us": round(g * 1e6, 1), "cpu_1thread_us": round(c * 1e6, 1),
                              "gpu_gib_s": round(seg.size / g / 2**30, 2), "cpu_gib_s": round(seg.size / c / 2**30, 2),
                              "gpu_faster": g < c}), flush=True)
            cx.host_unregister(seg)
            del seg
    if "crossover" in what:
        for kib in (64, 256, 512, 1024, 4096, 16384):
            n = max(1, kib * 1024 // 1072)
            rec = pinned_copy(O.synth_batch(n, 1024, 1024, seed=kib))
            cx.host_register(rec)
            for _ in range(3):
                rc, e, h, fr = cx.decode_batch_slice_with(rec, 0)
                assert rc == 0
            g = med(lambda: cx.decode_batch_slice_with(rec, 0), 30)
            reps = max(1, int(0.2 / max(rec.size / 3e9, 1e-6)))
            secs, _ = O.cpu_decode_bench(rec, 1, reps)
            c = secs / reps
            print(json.dumps({"path": "decode_batch(host, registered)", "record_bytes": int(rec.size),
                              "gpu_us": round(g * 1e6, 1), "cpu_1thread_us": round(c * 1e6, 1), "gpu_faster": g < c}),
                  flush=True)
            cx.host_unregister(rec)
    cx.close()


if __name__ == "__main__":
    main()

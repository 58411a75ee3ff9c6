"""Same-box A/B(/C...) of builds of the codec library (diagnostic, not part of the bench):
the C2 decode (1 M x 1 KiB, Verify, device-resident) per launch, timed with HIP
events on the launch stream (iggy_codec_profile_*: the bracket the bench's roofline
uses), the two libraries interleaved round by round in one process on one record.
Each timed result is checked (no error, every frame, the batch checksum). Also the
C3-shaped variable record (general walk) with --c3.

usage: python scripts/ab_libs.py <lib A .so> <lib B .so> [<lib C .so> ...] [--rounds 6] [--steps 10]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from iggy_amd import abi  # noqa: E402
from iggy_amd.codec import Codec, load  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--messages", type=int, default=1 << 20)
    ap.add_argument("--c3", action="store_true", help="payloads U[64, 4096] (the general walk)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctxs = [Codec(0, library=load(p)) for p in args.libs]
    s = torch.cuda.Stream()
    stream = s.cuda_stream
    n = args.messages
    lo, hi = (64, 4096) if args.c3 else (1024, 1024)
    batch, keep, _ = bench.make_batch(ctxs[0], n, lo, hi, 0, dev, stream)
    L = batch.numel()
    d_pos = torch.empty(n, dtype=torch.int64, device=dev)
    d_res = torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device=dev)
    for cx in ctxs:
        cx.reserve(L)
    per = [[] for _ in ctxs]
    checksums = set()
    for rnd in range(args.rounds):
        for k, cx in enumerate(ctxs):
            for _ in range(2):
                assert cx.decode_device(batch.data_ptr(), L, 0, d_pos.data_ptr(), n, d_res.data_ptr(), stream) == 0
            torch.cuda.synchronize()
            cx.profile_enable(True)
            ev_ms = 0.0
            for _ in range(args.steps):
                d_res.zero_()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                assert cx.decode_device(batch.data_ptr(), L, 0, d_pos.data_ptr(), n, d_res.data_ptr(), stream) == 0
                e1.record(s)
                torch.cuda.synchronize()
                ev_ms += e0.elapsed_time(e1)
                r = abi.DecodeResult.from_buffer_copy(d_res.cpu().numpy().tobytes())
                assert r.error.kind == 0 and r.frame_count == n, r.error
                checksums.add(r.computed_checksum)
            launches, total_ms = cx.profile_read(0)
            cx.profile_enable(False)
            # C2: the uniform kernel's own bracket (the bench's roofline); C3: both kernels
            # (the uniform kernel hands over to the general walk), events on the stream
            per[k].append(ev_ms / args.steps if args.c3 else total_ms / max(launches, 1))
    assert len(checksums) == 1, checksums  # both builds compute the same batch checksum
    alg = L + 8 * n
    for k, p in enumerate(args.libs):
        med = statistics.median(per[k])
        print(json.dumps({"lib": p, "per_round_ms": [round(x, 4) for x in per[k]], "median_ms": round(med, 4),
                          "frac": round(alg / (med * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()

"""Diagnostic: the bench's pipelined C2 form (steps alternating over lanes, each lane
its own context, stream and 1 M x 1 KiB record) with the uniform decode's workgroup
count per context set through the diagnostic build (IGGY_CODEC_UNIFORM_GRID, read at
context creation). Two lanes of half grids run side by side on disjoint CUs instead of
overlapping one decode's tail with the next one's start.

usage: python scripts/pipe_grid.py [--steps 40] [--rounds 3]   (prints one JSON line per setting)
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from iggy_amd import abi  # noqa: E402
from iggy_amd.codec import Codec, load, DIAG_LIB_PATH  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--settings", default="", help="lanes:grid,... (default: a fixed sweep)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = load(DIAG_LIB_PATH)
    n = bench.N_MSG
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    settings = [(2, ncu - 1), (2, ncu // 2 - 1), (2, ncu // 2), (3, ncu // 3 - 1), (4, ncu // 4 - 1)]
    if args.settings:
        settings = [tuple(int(v) for v in x.split(":")) for x in args.settings.split(",")]
    made = {}
    for lanes_n, grid in settings:
        os.environ["IGGY_CODEC_UNIFORM_GRID"] = str(grid)
        lanes = []
        for li in range(lanes_n):
            cx = Codec(0, library=lib)
            s = torch.cuda.Stream(dev)
            key = li
            if key not in made:
                made[key] = bench.make_batch(cx, n, bench.PAYLOAD, bench.PAYLOAD, li, dev, s.cuda_stream)[0]
            batch = made[key]
            cx.reserve(batch.numel())
            lanes.append((cx, s, batch, torch.empty(n, dtype=torch.int64, device=dev),
                          torch.zeros(ctypes.sizeof(abi.DecodeResult), dtype=torch.uint8, device=dev)))
        L = lanes[0][2].numel()

        def step(i):
            cx, s, b, p, r = lanes[i % len(lanes)]
            assert cx.decode_device(b.data_ptr(), L, abi.INTEGRITY_VERIFY, p.data_ptr(), n, r.data_ptr(),
                                    s.cuda_stream) == 0

        for i in range(2 * len(lanes)):
            step(i)
        torch.cuda.synchronize()
        rates = []
        for _ in range(args.rounds):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(args.steps):
                step(i)
            torch.cuda.synchronize()
            rates.append(args.steps * L / (time.perf_counter() - t0) / 2**30)
        for cx, s, b, p, r in lanes:
            res = abi.DecodeResult.from_buffer_copy(r.cpu().numpy().tobytes())
            assert res.error.kind == 0 and res.frame_count == n, res.error
            cx.close()
        print(json.dumps({"lanes": lanes_n, "grid": grid, "gib_s": [round(x, 1) for x in rates],
                          "best": round(max(rates), 1)}), flush=True)


if __name__ == "__main__":
    main()

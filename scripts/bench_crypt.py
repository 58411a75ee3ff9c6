"""At-rest encryption re-encode on the C2 record (1,048,576 x 1 KiB): encrypt then
decrypt, `--steps` calls each on one stream (for rocprofv3 kernel traces; the
bench line carries the same leg as crypt_c2). Diagnostic."""
import argparse
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from iggy_amd import abi  # noqa: E402
from iggy_amd.codec import Codec  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cx = Codec(0)
    s = torch.cuda.Stream(dev)
    n = 1 << 20
    rec = bench.make_batch(cx, n, 1024, 1024, 0, dev, s.cuda_stream)[0]
    print(bench.crypt_leg(cx, dev, rec, n, args.steps, False), flush=True)


if __name__ == "__main__":
    main()

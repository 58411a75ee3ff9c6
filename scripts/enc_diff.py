"""Diagnostic: encode a segmented batch on the GPU and the oracle, list every byte range
that differs with its frame, stream position and block (not part of the bench/tests)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from iggy_amd import codec as _codec  # noqa: E402
if os.environ.get("IGGY_LIB"):
    _codec.use_library(os.environ["IGGY_LIB"])
from iggy_amd.codec import Codec, raw_messages  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    n, lo, hi = 262144, 100, 1100
    rng = np.random.default_rng(n + lo)
    pls = rng.integers(lo, hi + 1, size=n).astype(np.uint32)
    ids = rng.integers(0, 2**63, size=2 * n, dtype=np.uint64)
    ots = (1_700_000_000_000_000 + rng.integers(0, 10**6, size=n)).astype(np.uint64)
    pay = rng.integers(0, 256, size=int(pls.sum()), dtype=np.uint8)
    raw = raw_messages(ids, ots, pay, pls)
    cx = Codec(0)
    rc, e, out = cx.encode_batch(raw, 4)
    print("gpu rc", rc, e, flush=True)
    if not len(out):
        return
    orc, oe, oout = O.encode_batch(raw, 4)
    a = np.frombuffer(out, dtype=np.uint8)
    b = np.frombuffer(oout, dtype=np.uint8)
    d = np.nonzero(a != b)[0]
    print("rc", rc, orc, "len", a.size, b.size, "diff bytes", d.size, flush=True)
    sizes = 48 + pls.astype(np.int64)
    starts = 256 + np.concatenate([[0], np.cumsum(sizes)[:-1]])
    pos = np.concatenate([[0], np.cumsum(pls.astype(np.int64))[:-1]])
    runs = []
    if d.size:
        br = np.nonzero(np.diff(d) != 1)[0]
        s0 = np.concatenate([[d[0]], d[br + 1]])
        s1 = np.concatenate([d[br], [d[-1]]])
        runs = list(zip(s0, s1))
    print("runs", len(runs))
    # which frames, by segment and ordinal j inside their lane group (segments of 40/35/19/6 %)
    nb = (44 + 8 * n - 1) // 1024
    Fs = [0] + [min(n, 128 * (nb * q // 1000) - 5) for q in (400, 750, 940)] + [n]
    stride = 8 * 255 * 4
    from collections import Counter
    hist = Counter()
    badf = sorted(set(int(np.searchsorted(starts, x0, side='right') - 1) for x0, _ in runs))
    for f in badf:
        seg = max(i for i in range(4) if Fs[i] <= f)
        hist[(seg, (f - Fs[seg]) // stride)] += 1
    print("bad frames", len(badf), "by (segment, j):", sorted(hist.items()))
    # per lane group of segment 0: which ordinals are bad, and each ordinal's step index
    steps = (40 + pls.astype(np.int64) + 1023) // 1024
    bad_set = set(badf)
    shown = 0
    for vw in range(0, 1020, 7):
        for fg in range(8):
            fr = [Fs[0] + 8 * vw + fg + j * stride for j in range(20) if Fs[0] + 8 * vw + fg + j * stride < Fs[1]]
            flags = ''.join('X' if f in bad_set else '.' for f in fr)
            if 'X' in flags and shown < 25:
                st = np.concatenate([[0], np.cumsum(steps[fr])])
                print(f"vw {vw} fg {fg} frames {flags} steps-start {list(st)}")
                shown += 1
    for x0, x1 in runs[:40]:
        f = int(np.searchsorted(starts, x0, side='right') - 1)
        off = int(x0 - starts[f])
        L = 40 + int(pls[f])
        r = (int(pos[f]) - 40) % 16
        print(f"bytes [{x0}, {x1}] len {x1 - x0 + 1} frame {f} frame-off {off} stream {off - 8} L {L} r {r} "
              f"block {(off - 8) // 1024 if off >= 8 else -1} got {a[x0:x0 + 4].tobytes().hex()} want {b[x0:x0 + 4].tobytes().hex()}")


if __name__ == "__main__":
    main()

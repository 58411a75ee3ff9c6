"""Split a rocprofv3 kernel trace of scripts/diag_decode.py into its variants:
per (integrity, round, dbg variant) the decode kernels' median durations (us).
Diagnostic only."""
import sqlite3
import statistics
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    rows = [(n, d) for n, d in db.execute("select name, duration from kernels order by start")
            if "iggy::k_decode" in n]
    variants = [0, 1, 65, 32]
    order = [(0, r, v) for r in range(3) for v in variants] + [(1, r, 0) for r in range(3)]
    # each decode: Verify -> [lg, uniform, general], LayoutOnly -> [uniform, general]
    pos = 0
    for integ, rnd, v in order:
        per = 3 if integ == 0 else 2
        seq = rows[pos: pos + 12 * per]
        pos += 12 * per
        timed = seq[2 * per:]
        agg = {}
        for n, d in timed:
            key = n.split("(")[0].replace("void ", "")
            agg.setdefault(key, []).append(d / 1e3)
        txt = "  ".join(f"{k.split('::')[-1]}={statistics.median(x):.1f}" for k, x in agg.items())
        print(f"integ={integ} round={rnd} dbg={v:3d}  {txt}")


if __name__ == "__main__":
    main()

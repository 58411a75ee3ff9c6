"""Summarise a rocprofv3 rocpd database: per-kernel count / avg / min / max (us)
and, with --timeline K, the last K dispatches with start offsets (us)."""
import sqlite3
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    tl = int(sys.argv[sys.argv.index("--timeline") + 1]) if "--timeline" in sys.argv else 0
    db = sqlite3.connect(path)
    rows = list(db.execute("select name, start, end, duration, stream, queue from kernels order by start"))
    agg = defaultdict(list)
    for name, s, e, d, st, q in rows:
        agg[name].append(d)
    print(f"{'kernel':60s} {'calls':>6s} {'avg_us':>10s} {'min_us':>10s} {'max_us':>10s} {'total_ms':>10s}")
    for name, ds in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{name[:60]:60s} {len(ds):6d} {sum(ds)/len(ds)/1e3:10.2f} {min(ds)/1e3:10.2f} "
              f"{max(ds)/1e3:10.2f} {sum(ds)/1e6:10.3f}")
    if tl:
        t0 = rows[-tl][1]
        for name, s, e, d, st, q in rows[-tl:]:
            print(f"{(s - t0)/1e3:10.2f} {(e - t0)/1e3:10.2f} {d/1e3:9.2f}  {st:16s} {name[:50]}")


if __name__ == "__main__":
    main()


def per_kernel_sequence(path, name_sub):
    """Durations (us) of every dispatch whose name contains name_sub, in order."""
    db = sqlite3.connect(path)
    return [d / 1e3 for (n, d) in db.execute("select name, duration from kernels order by start")
            if name_sub in n]

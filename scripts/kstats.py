"""Per-kernel dispatch statistics from a rocprofv3 SQLite database.
usage: python scripts/kstats.py gpurun_out/<dir>/run_results.db"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute(
    "select k.display_name, count(*), avg(d.end - d.start), min(d.end - d.start), max(d.end - d.start), "
    "sum(d.end - d.start) from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol k "
    "on d.kernel_id = k.id group by k.display_name order by 6 desc").fetchall()
print(f"{'kernel':60s} {'n':>5s} {'avg_us':>10s} {'min_us':>10s} {'max_us':>10s} {'total_ms':>10s}")
for name, n, avg, mn, mx, tot in rows:
    print(f"{name[:60]:60s} {n:5d} {avg / 1e3:10.2f} {mn / 1e3:10.2f} {mx / 1e3:10.2f} {tot / 1e6:10.3f}")

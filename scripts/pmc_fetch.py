"""Turn a rocprofv3 `--pmc FETCH_SIZE` database of `bench.py` into
profiles/pmc_fetch.json: HBM bytes fetched per decode by the uniform decode's
producer grid (k_uniform_lg for C2), corrected per MI355X_MICROARCH.md (gfx950
FETCH_SIZE reports half the bytes of a wide streaming read: x2).

usage: python scripts/pmc_fetch.py <pmc_counter_collection.csv | rocpd .db> [messages] [payload]
(scripts/profile_round.sh writes gpurun_out/prof_<tag>/pmc1/pmc_counter_collection.csv)
"""
import csv
import json
import os
import sqlite3
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    db_path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    pl = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
    if db_path.endswith(".csv"):
        acc = {}
        for r in csv.DictReader(open(db_path)):
            if r["Counter_Name"] == "FETCH_SIZE":
                key = (r["Kernel_Name"], r["Dispatch_Id"])
                acc[key] = acc.get(key, 0.0) + float(r["Counter_Value"])
        rows = [(k[0], v, int(k[1])) for k, v in sorted(acc.items(), key=lambda kv: int(kv[0][1]))]
    else:
        db = sqlite3.connect(db_path)
        rows = list(db.execute(
            "select kernel_name, value, dispatch_id from counters_collection where counter_name = 'FETCH_SIZE' "
            "order by dispatch_id"))
    per_kernel = {}
    for name, kb, _ in rows:
        per_kernel.setdefault(name.split("(")[0], []).append(kb)
    target = [k for k in per_kernel if "k_decode_uniform" in k]
    if not target:
        raise SystemExit(f"no k_decode_uniform dispatches in {db_path}: {sorted(per_kernel)}")
    # decodes timed by bench.py: every k_decode_uniform dispatch (the encode-side
    # and torch kernels are separate names)
    vals = per_kernel[target[0]]
    kb = statistics.median(vals)
    hbm_bytes = kb * 1024 * 2  # gfx950 correction: FETCH_SIZE = half of the streamed bytes
    batch = 256 + n * (48 + pl)
    out = {
        "messages": n, "payload": pl, "kernel": target[0], "dispatches": len(vals),
        "fetch_size_kb_median": kb, "hbm_bytes_per_decode": int(hbm_bytes),
        "algorithmic_bytes": batch + 8 * n, "ratio_to_algorithmic": round(hbm_bytes / (batch + 8 * n), 4),
        "source": f"rocprofv3 --pmc FETCH_SIZE on bench.py at HEAD {os.environ.get('PMC_HEAD', '?')} "
                  f"({os.environ.get('PMC_PROFILE', 'profiles/')}; x2 per MI355X_MICROARCH.md gfx950 FETCH_SIZE note)",
        "all_kernels_kb_median": {k: statistics.median(v) for k, v in per_kernel.items()},
    }
    path = os.path.join(ROOT, "profiles", "pmc_fetch.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

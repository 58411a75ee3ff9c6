"""Summarise rocprofv3 --pmc counter CSVs (pmc_counter_collection.csv) for one
kernel: per-dispatch median of every counter, plus the SQ cycle split
(WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES, MI355X_MICROARCH.md)
and FETCH_SIZE as HBM bytes (x2 gfx950 correction). Diagnostic / profiles only.

usage: python scripts/pmc_summary.py <kernel substring> <csv> [<csv> ...]
"""
import csv
import json
import statistics
import sys


def main():
    want = sys.argv[1]
    per = {}
    for path in sys.argv[2:]:
        for r in csv.DictReader(open(path)):
            if want not in r["Kernel_Name"]:
                continue
            key = (path, r["Dispatch_Id"])
            per.setdefault(r["Counter_Name"], {}).setdefault(key, 0.0)
            per[r["Counter_Name"]][key] += float(r["Counter_Value"])  # summed over dimensions
    med = {k: statistics.median(v.values()) for k, v in per.items()}
    out = {"kernel": want, "dispatches": {k: len(v) for k, v in per.items()}, "median_per_dispatch": med}
    if "FETCH_SIZE" in med:
        out["hbm_bytes_per_dispatch"] = med["FETCH_SIZE"] * 1024 * 2
    wc = med.get("SQ_WAVE_CYCLES")
    if wc:
        out["sq_split_of_wave_cycles"] = {
            k: round(med[k] / wc, 4) for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                               "SQ_ACTIVE_INST_VALU") if k in med}
    if "SQ_BUSY_CYCLES" in med and "SQ_ACTIVE_INST_VALU" in med:
        out["valu_active_per_busy_cycle"] = round(med["SQ_ACTIVE_INST_VALU"] / med["SQ_BUSY_CYCLES"], 4)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()

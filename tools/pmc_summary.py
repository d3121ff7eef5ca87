"""Summarise rocprofv3 --pmc CSVs per kernel for the LAST proof in the run
(the last 24 round dispatches). Usage: pmc_summary.py dir1 [dir2 ...]"""
import csv
import sys
from collections import defaultdict


def load(d):
    rows = list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))
    return rows


def main():
    per = defaultdict(lambda: defaultdict(float))  # dispatch -> counter -> value
    meta = {}
    for d in sys.argv[1:]:
        for r in load(d):
            key = (d, int(r["Dispatch_Id"]))
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            meta[key] = (r["Kernel_Name"], int(r["Grid_Size"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for d in sys.argv[1:]:
        keys = sorted(k for k in per if k[0] == d)
        rounds = [k for k in keys if "gkr_round" in meta[k][0]][-24:]
        print(f"== {d}")
        for k in rounds:
            name, grid, ns = meta[k]
            c = per[k]
            s = " ".join(f"{n}={v:.4g}" for n, v in sorted(c.items()))
            print(f"{name[10:28]:18s} grid={grid:7d} {ns/1e3:8.1f}us {s}")


if __name__ == "__main__":
    main()

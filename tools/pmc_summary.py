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
    dirs = [a for a in sys.argv[1:] if not a.startswith("--")]
    for d in dirs:
        for r in load(d):
            key = (d, int(r["Dispatch_Id"]))
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            meta[key] = (r["Kernel_Name"], int(r["Grid_Size"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for d in dirs:
        keys = sorted(k for k in per if k[0] == d)
        if "--steps" in sys.argv:  # the matrix-core steps of the last proof (from its k_gkr_d0t)
            ks = [k for k in keys if "k_gkr_" in meta[k][0]]
            first = max((i for i, k in enumerate(ks) if "k_gkr_d0t" in meta[k][0]), default=0)
            rounds = ks[first:]
        else:
            rounds = [k for k in keys if "gkr_round" in meta[k][0]][-24:]
        print(f"== {d}")
        for k in rounds:
            name, grid, ns = meta[k]
            c = per[k]
            s = " ".join(f"{n}={v:.4g}" for n, v in sorted(c.items()))
            print(f"{name.split('(')[0].replace('void zk::', '')[:26]:26s} grid={grid:7d} {ns/1e3:8.1f}us {s}")


if __name__ == "__main__":
    main()

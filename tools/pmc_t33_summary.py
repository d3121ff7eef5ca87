"""Summarise tools/pmc_t33.sh: per-kernel SQ counters of the first k_gkr_t33
(64-octant, pipelined) against its memory-only pattern k_order<0, 2, true>
(grid 256), averaged over their dispatches, and the derived per-wave ratios.
usage: python3 tools/pmc_t33_summary.py gpurun_out/pmct33_k1 gpurun_out/pmct33_k2 gpurun_out/pmct33_m1 gpurun_out/pmct33_m2"""
import csv
import sys
from collections import defaultdict


def per_dispatch(d):
    per = defaultdict(lambda: defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        k = int(r["Dispatch_Id"])
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[k] = (r["Kernel_Name"], int(r["Grid_Size"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return per, meta


def pick(d, want):
    per, meta = per_dispatch(d)
    rows = [(per[k], meta[k][2]) for k in sorted(per) if want(meta[k][0], meta[k][1])]
    return rows


def main():
    groups = {"k_gkr_t33 (first, 64-octant pipelined)":
              (lambda n, g: "k_gkr_t33" in n and ", 64, true" in n, [a for a in sys.argv[1:] if "_k" in a]),
              "W8 pattern k_order<STRIDE, 2 ahead, stores> grid 256":
              (lambda n, g: "k_order<0, 2, true>" in n and g == 256 * 256, [a for a in sys.argv[1:] if "_m" in a])}
    for title, (want, dirs) in groups.items():
        tot, ns, cnt = defaultdict(float), [], 0
        for d in dirs:
            rows = pick(d, want)
            for c, dur in rows:
                for n, v in c.items():
                    tot[n] += v / len(rows)
                ns.append(dur)
        print(f"== {title}: {len(ns)} dispatches, mean {sum(ns) / max(len(ns), 1) / 1e3:.1f} us")
        for n in sorted(tot):
            print(f"   {n:22s} {tot[n]:.4g}")
        wc = tot.get("SQ_WAVE_CYCLES", 0)
        if wc:
            for n in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MFMA",
                      "SQ_ACTIVE_INST_ANY", "SQ_INST_CYCLES_VMEM"):
                if n in tot:
                    print(f"   {n} / SQ_WAVE_CYCLES = {tot[n] / wc:.3f}")
        if tot.get("SQ_WAVES"):
            print(f"   per wave: cycles {wc / tot['SQ_WAVES']:.4g}, VALU insts {tot.get('SQ_INSTS_VALU', 0) / tot['SQ_WAVES']:.4g}, "
                  f"VMEM rd {tot.get('SQ_INSTS_VMEM_RD', 0) / tot['SQ_WAVES']:.4g}, wr {tot.get('SQ_INSTS_VMEM_WR', 0) / tot['SQ_WAVES']:.4g}")


if __name__ == "__main__":
    main()

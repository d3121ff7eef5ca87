"""Print the kernels of the last proof in a rocprofv3 kernel trace (durations, gaps)."""
import csv, glob, sys
path = sys.argv[1] if sys.argv[1].endswith(".csv") else glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
first = ("k_gkr_round0", "k_gkr_d0")  # the first step of a proof
starts = [i for i, r in enumerate(rows) if any(f in r["Kernel_Name"] for f in first)]
rows = rows[starts[-1]:]
prev = None
tot = 0.0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void zk::", "")
    print(f"{name[:40]:40s} grid {int(r['Grid_Size_X']):8d} {(e - s) / 1e3:8.1f} us  gap {((s - prev) / 1e3 if prev else 0):6.1f}")
    tot += (e - s) / 1e3
    prev = e
print(f"sum of kernels {tot:.1f} us, span {(int(rows[-1]['End_Timestamp']) - int(rows[0]['Start_Timestamp'])) / 1e3:.1f} us")

"""HBM traffic of the dominant kernel from rocprofv3 PMC passes.

Reads gpurun_out/prof_<tag>_fetch and _write (FETCH_SIZE / WRITE_SIZE, KiB per
dispatch), takes the k_gkr_round dispatches of the LAST proof in the run, and
reports per-launch traffic = 2 * FETCH_SIZE + WRITE_SIZE bytes (the x2 is the
gfx950 correction for wide coalesced streaming reads, MI355X_MICROARCH.md
"HBM"), beside the algorithmic bytes (768 B per output pair).
Writes profiles/<tag>_traffic.json and copies the kernel-stats CSV.
usage: python tools/pmc_traffic.py <tag> <nvars>
"""
import csv
import json
import os
import shutil
import sys

KERNEL = "zk::k_gkr_round"


def dispatches(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    out = {}
    for r in rows:
        out[int(r["Dispatch_Id"])] = (r["Kernel_Name"], int(r["Grid_Size"]), float(r["Counter_Value"]))
    return [out[k] for k in sorted(out)]


def main():
    tag, nvars = sys.argv[1], int(sys.argv[2])
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    fetch = dispatches(f"{root}/gpurun_out/prof_{tag}_fetch/run_counter_collection.csv", "FETCH_SIZE")
    write = dispatches(f"{root}/gpurun_out/prof_{tag}_write/run_counter_collection.csv", "WRITE_SIZE")
    rounds = nvars - 1  # k_gkr_round(+_lanes) launches per proof
    f = [x for x in fetch if KERNEL in x[0]][-rounds:]
    w = [x for x in write if KERNEL in x[0]][-rounds:]
    assert len(f) == len(w) == rounds
    per_round = []
    for k, ((name, _, fe), (_, _, wr)) in enumerate(zip(f, w), start=1):
        pairs = 1 << (nvars - 1 - k)
        per_round.append({"round": k, "kernel": name.split("(")[0], "fetch_bytes": 2 * fe * 1024,
                          "write_bytes": wr * 1024, "alg_bytes": 768.0 * pairs})
    # the dominant kernel is the symbol k_gkr_round (large rounds); the small
    # rounds' k_gkr_round_lanes is summarised beside it
    def summary(sym):
        rs = [r for r in per_round if r["kernel"].endswith(sym)]
        t = sum(r["fetch_bytes"] + r["write_bytes"] for r in rs)
        a = sum(r["alg_bytes"] for r in rs)
        return rs, t, a

    big, tot_traffic, tot_alg = summary("k_gkr_round<zk::Bn254Fr>")
    lanes, lt, la = summary("k_gkr_round_lanes<zk::Bn254Fr>")
    res = {"kernel": "k_gkr_round", "nvars": nvars, "launches": len(big),
           "traffic_bytes_per_launch": tot_traffic / len(big), "alg_bytes_per_launch": tot_alg / len(big),
           "traffic_over_alg": tot_traffic / tot_alg,
           "lanes": {"kernel": "k_gkr_round_lanes", "launches": len(lanes),
                     "traffic_bytes_per_launch": lt / max(1, len(lanes)), "alg_bytes_per_launch": la / max(1, len(lanes)),
                     "traffic_over_alg": lt / la if la else None},
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                     "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 half-count correction)",
           "per_round": per_round}
    os.makedirs(f"{root}/profiles", exist_ok=True)
    with open(f"{root}/profiles/{tag}_traffic.json", "w") as fh:
        json.dump(res, fh, indent=1)
    shutil.copy(f"{root}/gpurun_out/prof_{tag}/run_kernel_stats.csv", f"{root}/profiles/{tag}_kernel_stats.csv")
    print(json.dumps({k: v for k, v in res.items() if k != "per_round"}, indent=1))


if __name__ == "__main__":
    main()

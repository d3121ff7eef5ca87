"""HBM traffic of the round kernels from rocprofv3 PMC passes.

Reads gpurun_out/prof_<tag>_fetch and _write (FETCH_SIZE / WRITE_SIZE, KiB per
dispatch), takes the dispatches of the LAST proof in the run (from its
k_gkr_round0), and reports per dispatch traffic = 2 * FETCH_SIZE + WRITE_SIZE
bytes (the x2 is the gfx950 correction for wide coalesced streaming reads,
MI355X_MICROARCH.md "HBM") beside the algorithmic bytes of the step schedule
(host.hpp gkr_phase): round 0 256 B per pair, a single round 768 B per output
pair, a double step 1536 B (one pending challenge) or 2560 B (two) per quad,
the persistent tail the sum of its double steps; k_gkr_d0m 128 B per input
index, k_gkr_dm 2560 B per quad, k_gkr_d0t 128 B per input index, k_gkr_t33
9216 B per octant of its output level, k_gkr_dm3 4608 B per quad.
Writes profiles/<tag>_traffic.json and copies the kernel-stats CSV.
usage: python tools/pmc_traffic.py <tag> <nvars> [dtail_max_quads]
(tools/profile_bench.sh launches steps one at a time, ZK_PRELAUNCH=0: no persistent
tail, so dtail_max_quads defaults to 0)
"""
import csv
import json
import os
import shutil
import sys


def dispatches(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    out = {}
    for r in rows:
        out[int(r["Dispatch_Id"])] = (r["Kernel_Name"].split("(")[0].replace("void ", ""), float(r["Counter_Value"]))
    return [out[k] for k in sorted(out)]


def schedule(n, dtail_max_quads=4096, d0=True, dm_min_quads=1 << 17, d0t=True):
    """(symbol prefix, algorithmic bytes) per dispatch of one proof (one GPU), as
    host.hpp gkr_phase builds it. d0t (ZK_D0T, default, n >= 11): k_gkr_d0t
    (rounds 0-2, 128 B per input index), nt k_gkr_t33 (9216 B per octant), one
    k_gkr_dm3 (4608 B per quad), then double steps with two pending challenges.
    Else d0 (ZK_D0): an even n starts with k_gkr_d0m (rounds 0 and 1). Double
    steps with >= dm_min_quads quads run as k_gkr_dm, the others as k_gkr_dround."""
    i, np_ = 0, 0
    if d0t and n >= 11:
        nt, k = -1, 0
        while 3 + 3 * k + 8 <= n:
            r = n - 3 - 3 * k
            if r % 2 == 0 and (r >= 12 or nt < 0):
                nt = k
            k += 1
        st = [("zk::k_gkr_d0t", 128.0 * (1 << n))]
        for k in range(nt):
            st.append(("zk::k_gkr_t33", 9216.0 * (1 << (n - 3 - 3 * k)) / 8))
        i = 3 + 3 * nt
        st.append(("zk::k_gkr_dm3", 4608.0 * (1 << (n - i)) / 4))
        i, np_ = i + 2, 2
    elif d0 and n >= 2 and n % 2 == 0:
        st = [("zk::k_gkr_d0m", 128.0 * (1 << n))]
        i, np_ = 2, 2
    else:
        st = [("zk::k_gkr_round0", 256.0 * (1 << (n - 1)))]
        if n >= 2:
            st.append(("zk::k_gkr_round", 768.0 * (1 << (n - 2))))
        i = 2
        if n >= 3 and (n - 2) % 2 == 1:
            st.append(("zk::k_gkr_round", 768.0 * (1 << (n - 3))))
            i = 3
        np_ = 1
    doubles = []
    while i + 1 < n:
        q = (1 << (n - i)) // 4
        doubles.append((q, np_))
        np_, i = 2, i + 2
    d0 = next((k for k, (q, _) in enumerate(doubles) if q <= dtail_max_quads), len(doubles))
    if len(doubles) - d0 < 2:
        d0 = len(doubles)
    for q, p in doubles[:d0]:
        sym = "zk::k_gkr_dm" if p == 2 and q >= dm_min_quads else f"zk::k_gkr_dround<zk::Bn254Fr, {p}>"
        st.append((sym, (1536.0 if p == 1 else 2560.0) * q))
    if d0 < len(doubles):
        st.append(("zk::k_gkr_dtail", sum((1536.0 if p == 1 else 2560.0) * q for q, p in doubles[d0:])))
    return st


def main():
    tag, nvars = sys.argv[1], int(sys.argv[2])
    dmax = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    fetch = dispatches(f"{root}/gpurun_out/prof_{tag}_fetch/run_counter_collection.csv", "FETCH_SIZE")
    write = dispatches(f"{root}/gpurun_out/prof_{tag}_write/run_counter_collection.csv", "WRITE_SIZE")
    sched = schedule(nvars, dmax)

    first = sched[0][0]

    def last_proof(ds):
        start = max(k for k, d in enumerate(ds) if d[0].startswith(first))
        return [d for d in ds[start:] if "k_gkr_" in d[0]][: len(sched)]

    f, w = last_proof(fetch), last_proof(write)
    assert len(f) == len(w) == len(sched), (len(f), len(w), len(sched))
    steps = []
    for (sym, alg), (name, fe), (_, wr) in zip(sched, f, w):
        assert name.startswith(sym.split("<")[0]), (name, sym)
        steps.append({"kernel": name, "fetch_bytes": 2 * fe * 1024, "write_bytes": wr * 1024, "alg_bytes": alg,
                      "traffic_over_alg": (2 * fe * 1024 + wr * 1024) / alg if alg else None})

    def summary(pred):
        rs = [r for r in steps if pred(r["kernel"])]
        t = sum(r["fetch_bytes"] + r["write_bytes"] for r in rs)
        a = sum(r["alg_bytes"] for r in rs)
        return {"launches": len(rs), "traffic_bytes_per_launch": t / max(1, len(rs)),
                "alg_bytes_per_launch": a / max(1, len(rs)), "traffic_over_alg": t / a if a else None}

    # the longest launch (bench.py's dominant kernel): the first k_gkr_t33 (over the inputs)
    t33 = [r for r in steps if r["kernel"].startswith("zk::k_gkr_t33")]
    if t33:
        r0 = t33[0]
        big = {"launches": 1, "traffic_bytes_per_launch": r0["fetch_bytes"] + r0["write_bytes"],
               "alg_bytes_per_launch": r0["alg_bytes"],
               "traffic_over_alg": (r0["fetch_bytes"] + r0["write_bytes"]) / r0["alg_bytes"]}
        name, kind = "k_gkr_t33 (over the input tables)", "gkr_t33"
    else:
        big, name, kind = summary(lambda k: k.startswith(first)), first[4:], "gkr_d0"
    res = {"kernel": name, "kind": kind, "nvars": nvars, **big,
           "others": {"k_gkr_d0t": summary(lambda k: "k_gkr_d0t" in k),
                      "k_gkr_t33": summary(lambda k: "k_gkr_t33" in k),
                      "k_gkr_dm3": summary(lambda k: "k_gkr_dm3" in k),
                      "k_gkr_dm": summary(lambda k: k.startswith("zk::k_gkr_dm<")),
                      "k_gkr_d0m": summary(lambda k: "k_gkr_d0m" in k),
                      "k_gkr_round0": summary(lambda k: "k_gkr_round0" in k),
                      "k_gkr_round": summary(lambda k: k.startswith("zk::k_gkr_round<")),
                      "k_gkr_dround": summary(lambda k: "k_gkr_dround" in k),
                      "k_gkr_dtail": summary(lambda k: "k_gkr_dtail" in k)},
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                     "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 half-count correction)",
           "per_step": steps}
    os.makedirs(f"{root}/profiles", exist_ok=True)
    with open(f"{root}/profiles/{tag}_traffic.json", "w") as fh:
        json.dump(res, fh, indent=1)
    shutil.copy(f"{root}/gpurun_out/prof_{tag}/run_kernel_stats.csv", f"{root}/profiles/{tag}_kernel_stats.csv")
    print(json.dumps({k: v for k, v in res.items() if k != "per_step"}, indent=1))


if __name__ == "__main__":
    main()

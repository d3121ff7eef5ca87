set -o pipefail
Q="--no-cpu-baseline --no-fold --no-e2e --no-serving --no-circuit --no-config5 --no-plain --no-config4"
mkdir -p gpurun_out/pab
for rep in 1 2; do
  for mode in plain rccl peer; do
    case $mode in plain) A="";; rccl) A="--force-rccl";; peer) A="--force-rccl --reduce peer";; esac
    timeout -k 10 240 python bench.py $Q $A > gpurun_out/pab/$mode$rep.json 2> gpurun_out/pab/$mode$rep.err || { echo "FAIL $mode"; tail -5 gpurun_out/pab/$mode$rep.err; exit 1; }
    python - "$mode" gpurun_out/pab/$mode$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
b = d["breakdown_per_step"]
print(sys.argv[1], round(d["ms_per_step"], 4), d.get("reduce"), d["proof"]["matches_oracle_fixture"], "coll/step", b["collectives"],
      [(x["kind"], x["us"]) for x in d["roofline"]["launches_of_proof"]])
PY
  done
done

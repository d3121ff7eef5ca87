# A/B of env knob sets on the 24-var proof: bench ms_per_step, interleaved rounds.
# usage: bash tools/gpu_ab.sh "ZK_X=0" "ZK_X=1" ...   (ROUNDS=3 by default)
set -o pipefail
mkdir -p gpurun_out
B="python3 bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 --no-config4 --no-events"
for r in $(seq ${ROUNDS:-3}); do
  i=0
  for cfg in "$@"; do
    env $cfg timeout -k 10 120 $B > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || { echo "FAIL $cfg"; tail -5 gpurun_out/ab_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$i.json')); print('round $r', '%-40s' % sys.argv[1], '%.4f ms' % d['ms_per_step'])" "$cfg"
    i=$((i+1))
  done
done

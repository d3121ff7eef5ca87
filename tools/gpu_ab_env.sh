# A/B of environment settings on the default 24-var bench (no events), 3 alternations.
# usage: bash tools/gpu_ab_env.sh "ZK_X=0" "ZK_X=1" ...
set -o pipefail
mkdir -p gpurun_out
B="python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 --no-config4 --no-events"
for rep in ${REPS:-1 2 3}; do
  for e in "$@"; do
    env $e timeout -k 10 120 $B > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open('gpurun_out/ab.json'));print(sys.argv[1], round(d['ms_per_step'],4))" "$e"
  done
done

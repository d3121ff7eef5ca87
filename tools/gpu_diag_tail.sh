# Per-step loop times (ZK_DEBUG_TAIL) of the 24-var proof for the default library and
# diagnostic variants in abtest/ (wrong proofs allowed: seed 7 has no fixture).
# usage: ENV="ZK_HOST_ROUNDS=6" bash tools/gpu_diag_tail.sh abtest/a.so abtest/b.so ...
set -o pipefail
mkdir -p gpurun_out
for lib in "" "$@"; do
  env $ENV ZK_LIB_PATH=$lib ZK_DEBUG_TAIL=1 timeout -k 10 120 python3 bench.py --seed 7 --steps 3 --warmup 2 --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 --no-config4 --no-plain --no-events > gpurun_out/diag.json 2> gpurun_out/diag.err || { echo "FAIL $lib"; tail -5 gpurun_out/diag.err; exit 1; }
  echo "== ${lib:-default}"
  grep "zk step [0-2] " gpurun_out/diag.err | tail -3
done

# Per-block phase stamps (ZK_DEBUG_BLOCKS=<step>) of steps 0..4 of a 24-var proof
set -o pipefail
mkdir -p gpurun_out
for s in ${STEPS:-0 1 2 3}; do
  ZK_DEBUG_TAIL=1 ZK_DEBUG_BLOCKS=$s timeout -k 10 120 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 --no-config4 --no-events > gpurun_out/blk$s.json 2> gpurun_out/blk$s.err || { tail gpurun_out/blk$s.err; exit 1; }
  grep -A6 "zk step $s " gpurun_out/blk$s.err | tail -7
done

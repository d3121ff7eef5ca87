set -o pipefail
mkdir -p gpurun_out
Q="--no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 --no-config4"
for cfg in "ZK_DM=0" "ZK_DM=1"; do env $cfg ZK_DEBUG_EVENTS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 $Q > gpurun_out/b.json 2> gpurun_out/ev_$cfg.err || exit 1; echo $cfg; grep "zk: kind" gpurun_out/ev_$cfg.err | tail -8; done

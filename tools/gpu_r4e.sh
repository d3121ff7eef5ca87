# Round 4: knob A/Bs (t33 chunk size at level 6) and the device-FS tail trace.
set -o pipefail
mkdir -p gpurun_out
REPS="1 2 3" bash tools/gpu_ab_env.sh "ZK_T33_OCT64_MIN=1" "ZK_T33_OCT64_MIN=3" || exit 1
for dfs in 0 1; do
  ZK_DEVICE_FS=$dfs ZK_DEBUG_TAIL=1 timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 --no-config4 --no-plain --no-events > gpurun_out/tt_dfs$dfs.json 2> gpurun_out/tt_dfs$dfs.err || { tail gpurun_out/tt_dfs$dfs.err; exit 1; }
  echo "ZK_DEVICE_FS=$dfs"; grep "zk dtail\|zk host rounds" gpurun_out/tt_dfs$dfs.err | tail -4
done
exit 0

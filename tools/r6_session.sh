set -o pipefail
# round 6 session 11: replicated fan-in accumulators (ZK_ACCUM_REP) parity + A/B + traces
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "baseline_workload or grid_capped or gkr" > gpurun_out/s11_tests.log 2>&1 || { tail -30 gpurun_out/s11_tests.log; exit 1; }
tail -1 gpurun_out/s11_tests.log
ZK_ACCUM_REP=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "baseline_workload or grid_capped or gkr" > gpurun_out/s11_tests8.log 2>&1 || { tail -30 gpurun_out/s11_tests8.log; exit 1; }
tail -1 gpurun_out/s11_tests8.log
REPS=6 bash tools/gpu.sh abenv=-/ZK_ACCUM_REP=8/ZK_ACCUM_REP=16 > gpurun_out/rep_ab.log 2>&1 || { tail gpurun_out/rep_ab.log; exit 1; }
cat gpurun_out/rep_ab.log
for rep in 1 8; do
  ZK_ACCUM_REP=$rep ZK_DEBUG_TAIL=1 timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 --no-plain --no-config4 --no-events > /tmp/t.json 2> /tmp/t.err || exit 1
  echo "== ZK_ACCUM_REP=$rep"; grep "zk step\|zk dtail" /tmp/t.err | tail -8
done > gpurun_out/rep_trace.log
cat gpurun_out/rep_trace.log

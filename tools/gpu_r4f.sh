# Round 4: KZG + device-FS tests, the KZG profile at 2^24 and the device-FS tail trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kzg.py tests/test_gpu_device_fs.py tests/test_gpu_gkr_circuit.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4f_tests.log 2>&1 || { tail -40 gpurun_out/r4f_tests.log; exit 1; }
tail -2 gpurun_out/r4f_tests.log
for dfs in 0 1; do
  ZK_DEVICE_FS=$dfs ZK_DEBUG_TAIL=1 timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 --no-config4 --no-plain --no-events > gpurun_out/tt_dfs$dfs.json 2> gpurun_out/tt_dfs$dfs.err || { tail gpurun_out/tt_dfs$dfs.err; exit 1; }
  echo "ZK_DEVICE_FS=$dfs"; grep "zk dtail\|zk host rounds" gpurun_out/tt_dfs$dfs.err | tail -4
done
REPS="1 2" bash tools/gpu_ab_env.sh "ZK_DEVICE_FS=0" "ZK_DEVICE_FS=1" || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kzg -o run -- python3 tools/kzg_scale.py 24 > gpurun_out/prof_kzg.out 2> gpurun_out/prof_kzg.err || { tail gpurun_out/prof_kzg.err; exit 1; }
cat gpurun_out/prof_kzg.out
head -12 gpurun_out/prof_kzg/run_kernel_stats.csv | cut -c1-160
exit 0

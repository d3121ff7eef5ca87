# Round 4: schedule tests after the posted-eq-weights change, then an A/B against abtest/*.so.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_prelaunch.py tests/test_gpu_large.py tests/test_gpu_sharded.py tests/test_gpu_device_fs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4g_tests.log 2>&1 || { tail -40 gpurun_out/r4g_tests.log; exit 1; }
tail -2 gpurun_out/r4g_tests.log
REPS="1 2 3 4" bash tools/ab_libs_ev.sh "$@" || exit 1
exit 0

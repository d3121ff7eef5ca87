# Round 4: t33 tests + A/B against abtest/*.so, the traffic passes, then gpu_r4c.sh.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_prelaunch.py tests/test_gpu_large.py -x -q --timeout 200 --timeout-method thread -k "three_round or fixture or host_rounds" > gpurun_out/r4d_tests.log 2>&1 || { tail -40 gpurun_out/r4d_tests.log; exit 1; }
tail -2 gpurun_out/r4d_tests.log
REPS="1 2 3" bash tools/ab_libs_ev.sh "$@" || exit 1
bash tools/profile_bench.sh r4 || exit 1
python3 tools/pmc_traffic.py r4 24 > gpurun_out/r4_traffic.txt 2>&1 || { tail gpurun_out/r4_traffic.txt; exit 1; }
bash tools/gpu_r4c.sh || exit 1
exit 0

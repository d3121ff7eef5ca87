# Round-4 check: the new tests first, every -m gpu test, smoke, the default
# bench, an A/B of the default library against the variants given as
# arguments (abtest/*.so), and the memory-pattern microbenchmark.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_fs.py tests/test_gpu_kzg.py -x -q --timeout 200 --timeout-method thread > gpurun_out/new_tests.log 2>&1 || { tail -40 gpurun_out/new_tests.log; exit 1; }
tail -2 gpurun_out/new_tests.log
bash tools/gpu_full.sh || exit 1
if [ $# -gt 0 ]; then REPS=${REPS:-3} bash tools/ab_libs.sh "$@" || exit 1; fi
if [ -x tools/mb_wmix ]; then timeout -k 10 180 tools/mb_wmix > gpurun_out/mb_wmix.txt 2>&1 || { tail gpurun_out/mb_wmix.txt; exit 1; }; cat gpurun_out/mb_wmix.txt; fi
exit 0

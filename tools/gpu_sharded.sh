# Sharded / collective-path GPU tests only (world 2/4/8 host-comm ranks on one card, forced-RCCL world 1).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_prelaunch.py -x -v --timeout 300 --timeout-method thread -k "sharded or world or rccl or gather or host_failure" > gpurun_out/pytest_sharded.log 2>&1 || { tail -60 gpurun_out/pytest_sharded.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_sharded.log | tail -40

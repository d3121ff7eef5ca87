set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 280 --timeout-method thread > gpurun_out/pytest_sharded.log 2>&1 || { grep -E "PASS|FAIL|Error|error" gpurun_out/pytest_sharded.log | tail -30; exit 1; }
grep -cE "PASSED" gpurun_out/pytest_sharded.log; tail -1 gpurun_out/pytest_sharded.log
bash tools/gpu_rehearsal.sh

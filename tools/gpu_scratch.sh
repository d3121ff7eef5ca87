set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py -x -q --timeout 280 --timeout-method thread > gpurun_out/ps.log 2>&1 || { tail -30 gpurun_out/ps.log; exit 1; }
tail -1 gpurun_out/ps.log
ZK_HOST_ROUNDS=6 bash tools/gpu_trace.sh | grep "host rounds" | tail -2
REPS="1 2 3 4 5" bash tools/gpu_ab_env.sh ZK_HOST_ROUNDS=4 ZK_HOST_ROUNDS=6

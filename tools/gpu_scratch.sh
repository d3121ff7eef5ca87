set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash tools/gpu_trace.sh | grep "flag -> post" | tail -9 | tr '\n' ' '; echo
bash tools/gpu_trace.sh | grep -v "flag -> post" | tail -9
REPS="1 2 3" bash tools/gpu_ab_env.sh ZK_HOST_ROUNDS=0 ZK_HOST_ROUNDS=4 ZK_HOST_ROUNDS=6

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_prelaunch.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/p.log 2>&1 || { tail -30 gpurun_out/p.log; exit 1; }
tail -1 gpurun_out/p.log
bash tools/gpu_trace.sh | grep -v "flag -> post" | tail -8
REPS="1 2 3 4 5" bash tools/gpu_ab_env.sh ZK_DTAIL3=0 ZK_DTAIL3=1

# GPU tests, the per-step trace, then an env A/B (args) of the 24-var bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash tools/gpu_trace.sh | grep -v "flag -> post" | tail -14
bash tools/gpu_ab_env.sh "$@"

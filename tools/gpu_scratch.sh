set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash tools/ab_libs.sh abtest/old.so
ZK_LIB_PATH=abtest/old.so bash tools/gpu_trace.sh | grep "zk step 1 "
bash tools/gpu_trace.sh | grep "zk step 1 "

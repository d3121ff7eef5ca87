set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_prelaunch.py -x -q --timeout 120 --timeout-method thread -k "host_rounds" > gpurun_out/p.log 2>&1 || { tail -30 gpurun_out/p.log; exit 1; }
tail -1 gpurun_out/p.log
bash tools/gpu_trace.sh | grep "host rounds\|flag -> post" | tail -12

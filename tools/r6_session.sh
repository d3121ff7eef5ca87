set -o pipefail
# round 6 session 9: ZK_MALL_ORDER 1 / 2 parity + A/B
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py -m gpu -x -q --timeout 300 --timeout-method thread -k "mall" > gpurun_out/s9_tests.log 2>&1 || { tail -30 gpurun_out/s9_tests.log; exit 1; }
tail -2 gpurun_out/s9_tests.log
REPS=6 bash tools/gpu.sh abenv=-/ZK_MALL_ORDER=1/ZK_MALL_ORDER=2 > gpurun_out/mall_ab2.log 2>&1 || { tail gpurun_out/mall_ab2.log; exit 1; }
cat gpurun_out/mall_ab2.log

# Round 4: 20-bit signed fixed-base windows for the KZG setup (default build) against the 16-bit
# windows (abtest/head.so): KZG parity incl. the full-size golden commitments, then setup timings.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kzg.py tests/test_gpu_gkr_circuit.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4s_tests.log 2>&1 || { tail -40 gpurun_out/r4s_tests.log; exit 1; }
tail -2 gpurun_out/r4s_tests.log
for lib in "" abtest/head.so "" abtest/head.so; do echo "lib=${lib:-default}"; ZK_LIB_PATH=$lib timeout -k 10 200 python3 tools/kzg_scale.py 24 24 20 || exit 1; done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kzg24t -o run -- python3 tools/kzg_scale.py 24 24 > gpurun_out/prof_kzg24t.out 2>&1 || exit 1
exit 0

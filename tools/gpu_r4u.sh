# Round 4: XYZZ accumulators in the bucket sums and the fixed-base setup (default build)
# against Jacobian madd (abtest/head.so): KZG parity incl. full-size golden, then timings + rocprof.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kzg.py tests/test_gpu_gkr_circuit.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4u_tests.log 2>&1 || { tail -40 gpurun_out/r4u_tests.log; exit 1; }
tail -2 gpurun_out/r4u_tests.log
for lib in "" abtest/head.so "" abtest/head.so; do echo "lib=${lib:-default}"; ZK_LIB_PATH=$lib timeout -k 10 200 python3 tools/kzg_scale.py 24 24 20 16 || exit 1; done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kzg24x -o run -- python3 tools/kzg_scale.py 24 24 > gpurun_out/prof_kzg24x.out 2>&1 || exit 1
exit 0

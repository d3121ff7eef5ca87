# New-knob check: the prelaunch/parity/large/sharded GPU tests with the knob's default, then
# a same-box A/B of the given settings and the per-step trace of the default.
# usage: bash tools/gpu_knob.sh "ZK_X=0" "ZK_X=1"
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_prelaunch.py tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_sharded.py -x -q --timeout 200 --timeout-method thread > gpurun_out/knob_tests.log 2>&1 || { tail -40 gpurun_out/knob_tests.log; exit 1; }
tail -n 2 gpurun_out/knob_tests.log
ROUNDS=${ROUNDS:-3} bash tools/gpu_ab.sh "$@" || exit 1
bash tools/gpu_trace.sh > gpurun_out/knob_trace.txt || exit 1
grep "zk step" gpurun_out/tt.err | tail -5

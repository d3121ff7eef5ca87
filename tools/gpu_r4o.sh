# Round 4 (record; the ZK_MSM_SORT knob and the atomic scatter were removed after this A/B):
# blocked MSM bucket sort (ZK_MSM_SORT=1) against the atomic scatter (0):
# KZG parity (incl. 2^22 / 2^24 against the golden commitments), then commit timings and a rocprof.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kzg.py tests/test_gpu_gkr_circuit.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4o_tests.log 2>&1 || { tail -40 gpurun_out/r4o_tests.log; exit 1; }
tail -2 gpurun_out/r4o_tests.log
for s in 0 1 0 1; do echo "ZK_MSM_SORT=$s"; ZK_MSM_SORT=$s timeout -k 10 200 python3 tools/kzg_scale.py 16 20 24 || exit 1; done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kzg -o run -- python3 tools/kzg_scale.py 24 > gpurun_out/prof_kzg.out 2> gpurun_out/prof_kzg.err || { tail gpurun_out/prof_kzg.err; exit 1; }
cat gpurun_out/prof_kzg.out
exit 0

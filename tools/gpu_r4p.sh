# Round 4: signed-digit MSM buckets: KZG parity (incl. 2^22 / 2^24 golden commitments), timings, rocprof.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kzg.py tests/test_gpu_gkr_circuit.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4p_tests.log 2>&1 || { tail -40 gpurun_out/r4p_tests.log; exit 1; }
tail -2 gpurun_out/r4p_tests.log
timeout -k 10 200 python3 tools/kzg_scale.py 16 20 24 24 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kzg2 -o run -- python3 tools/kzg_scale.py 24 > gpurun_out/prof_kzg2.out 2> gpurun_out/prof_kzg2.err || { tail gpurun_out/prof_kzg2.err; exit 1; }
cat gpurun_out/prof_kzg2.out
exit 0

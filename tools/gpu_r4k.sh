# Round 4: circuit prover with fold-derived layer evaluations, adaptive host rounds,
# host eq tables: parity tests, then per-layer phases and split timing.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gkr_circuit.py tests/test_gpu_prelaunch.py tests/test_gpu_parity.py tests/test_gpu_device_fs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4k_tests.log 2>&1 || { tail -40 gpurun_out/r4k_tests.log; exit 1; }
tail -2 gpurun_out/r4k_tests.log
ZK_DEBUG_CIRCUIT=1 timeout -k 10 120 python3 tools/circuit_phases.py 12 > gpurun_out/circ.out 2> gpurun_out/circ.err || { tail -30 gpurun_out/circ.err; exit 1; }
sed -n '/prove 2/,$p' gpurun_out/circ.err
timeout -k 10 300 python3 tools/circuit_time.py 12 6,8,9,10 || exit 1
exit 0

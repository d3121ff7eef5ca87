# Round 4, second check: changed tests, the t33 stray-prefetch A/B against a
# variant library, the device Fiat-Shamir and circuit host-layer A/Bs, and the
# rocprof traffic passes of the default bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gkr_circuit.py tests/test_gpu_device_fs.py tests/test_gpu_prelaunch.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4b_tests.log 2>&1 || { tail -40 gpurun_out/r4b_tests.log; exit 1; }
tail -2 gpurun_out/r4b_tests.log
REPS="1 2 3" bash tools/ab_libs_ev.sh "$@" || exit 1
REPS="1 2 3" bash tools/gpu_ab_env.sh "ZK_DEVICE_FS=0" "ZK_DEVICE_FS=1" || exit 1
for h in 8 0 6 10; do
  ZK_CIRCUIT_HOST_LGL=$h timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fold --no-e2e --no-config5 --no-config4 --no-plain --no-events > gpurun_out/circ.json 2> gpurun_out/circ.err || { tail gpurun_out/circ.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/circ.json'));print('ZK_CIRCUIT_HOST_LGL', sys.argv[1], {k: v for k, v in d['gkr_circuit'].items() if 'ms' in k})" $h
done
bash tools/profile_bench.sh r4 || exit 1
python3 tools/pmc_traffic.py r4 24 > gpurun_out/r4_traffic.txt 2>&1 || { tail gpurun_out/r4_traffic.txt; exit 1; }
tail -30 gpurun_out/r4_traffic.txt
exit 0

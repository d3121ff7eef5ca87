# New-feature GPU check: the given pytest selection, then the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_large.py tests/test_gpu_gkr_circuit.py} -x -v --timeout 300 --timeout-method thread -k "${K:-plain or kzg}" > gpurun_out/new_tests.log 2>&1 || { tail -40 gpurun_out/new_tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/new_tests.log | tail -12
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 500 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -20 gpurun_out/bench_full.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_full.json'))
print(d['ms_per_step'], d['roofline']['avg_launch_us'])
for k in ('config1_12var_prove','plain_sumcheck','cpu_baseline'): print(k, json.dumps(d.get(k))[:1500])"

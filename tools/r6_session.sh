set -o pipefail
# round 6 session 7: the whole GPU suite + smoke on this tree, the default bench line, the rocprof profile
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/r6_pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/r6_pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/r6_pytest_gpu.txt 2>&1 || { tail gpurun_out/r6_pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/r6_pytest_gpu.txt
timeout -k 10 600 python bench.py > gpurun_out/r6_bench.json 2> gpurun_out/r6_bench.err || { tail gpurun_out/r6_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r6_bench.json')); r=d['roofline']; print(d['ms_per_step'], d['value']/1e9, r['frac'], r['avg_launch_us'], [(x['kind'], x['us']) for x in r['launches_of_proof']]); k=d['config5_bls12_381']; print({x: k[x] for x in k if x.endswith('_ms')}); print(d['gkr_circuit_kzg']['ms_median'], d['gkr_circuit']['ms_median'], d['config4_26var']['ms_median'], d['cpu_baseline']['value'])"
bash tools/profile_bench.sh r6 || { tail gpurun_out/prof_r6.err; exit 1; }
echo profile ok

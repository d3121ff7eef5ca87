# Round-3 evidence on one box: every -m gpu test, smoke, rocprof kernel stats + PMC traffic
# passes, SQ counter passes, the per-step trace and the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -n 30 gpurun_out/smoke.log; exit 1; }
tail -n 1 gpurun_out/smoke.log
bash tools/profile_bench.sh r3 || { tail -n 20 gpurun_out/prof_r3.err; exit 1; }
bash tools/pmc_steps.sh || exit 1
bash tools/gpu_trace.sh > gpurun_out/r3_trace.txt || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err || { tail -n 20 gpurun_out/r3_bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/r3_bench.json'));r=d['roofline'];print(d['ms_per_step'], r['avg_launch_us'], r['frac'], [x['us'] for x in r['launches_of_proof']])"

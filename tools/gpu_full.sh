# Full GPU check: every -m gpu test, the smoke test, and the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/bench.json'));r=d['roofline'];print(d['value']/1e9, 'G field-ops/s', round(d['ms_per_step'],4),'ms', r['kernel'][:10], round(r['avg_launch_us'],1), round(r['frac'],3), {k:(round(v['ms'],4), round(v['achieved_GBs'] or 0)) for k,v in r['round_kernels'].items()}); print({k: d[k] for k in d if k.startswith('config')})"

set -o pipefail
mkdir -p gpurun_out
Q="--no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 --no-config4"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_prelaunch.py -k "first_double_step" > gpurun_out/t1.log 2>&1 || { tail -50 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
for d0 in 1 3; do ZK_D0=$d0 timeout -k 10 120 python bench.py --steps 20 --warmup 5 $Q > gpurun_out/b_d0_$d0.json 2> gpurun_out/b_d0_$d0.err || exit 1; python -c "
import json;d=json.load(open('gpurun_out/b_d0_$d0.json'));r=d['roofline'];print('ZK_D0=$d0', round(d['ms_per_step'],4), r['kernel'][:10], round(r['avg_launch_us'],1), round(r['achieved'],1), round(r['frac'],3), {k:round(v['ms'],4) for k,v in r['round_kernels'].items()})"; done

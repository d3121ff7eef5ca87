# GPU check of the matrix-core kernels: probes, parity tests, A/B bench lines
set -o pipefail
mkdir -p gpurun_out
Q="--no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 --no-config4"
timeout -k 10 60 ./tools/mb_mfma > gpurun_out/mb_mfma.txt 2>&1 || exit 1
grep -E "permlane|k_dot" gpurun_out/mb_mfma.txt
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_prelaunch.py -k "matrix_core or first_double_step" > gpurun_out/t2.log 2>&1 || { tail -40 gpurun_out/t2.log; exit 1; }
tail -2 gpurun_out/t2.log
for cfg in "ZK_DM=0" "ZK_DM=1"; do env $cfg timeout -k 10 120 python bench.py --steps 20 --warmup 5 $Q > gpurun_out/b.json 2> gpurun_out/b.err || exit 1; python -c "
import json;d=json.load(open('gpurun_out/b.json'));r=d['roofline'];print('$cfg', round(d['ms_per_step'],4), r['kernel'][:10], round(r['avg_launch_us'],1), round(r['achieved'],1), round(r['frac'],3), {k:(round(v['ms'],4), round(v['achieved_GBs'] or 0)) for k,v in r['round_kernels'].items()})"; done

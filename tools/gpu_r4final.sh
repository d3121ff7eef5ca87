# Round 4, final tree: every -m gpu test, the smoke test, the default bench line, a rocprof
# kernel trace + PMC traffic of the bench workload, and the 2-rank rehearsal.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/bench.json'));r=d['roofline'];print(round(d['value']/1e9,1), 'G field-ops/s', round(d['ms_per_step'],4),'ms', round(r['avg_launch_us'],1), round(r['frac'],3), [x['us'] for x in r['launches_of_proof']], d['gkr_circuit']['ms_median'])"
bash tools/profile_bench.sh r4f || { tail -20 gpurun_out/prof_r4f.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --comm host --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 > gpurun_out/rehearsal_2rank.json 2> gpurun_out/rehearsal_2rank.err || { tail -30 gpurun_out/rehearsal_2rank.err; exit 1; }
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --force-rccl --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 > gpurun_out/force_rccl.json 2> gpurun_out/force_rccl.err || { tail -30 gpurun_out/force_rccl.err; exit 1; }
echo done
exit 0

# Round 4, third check: the multi-rank rehearsal on one card with the SCALE
# attribution fields, the forced-RCCL world-1 path (collective events), and a
# rocprof kernel trace of the KZG setup + commit at 2^24 points.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --comm host --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 > gpurun_out/rehearsal_2rank.json 2> gpurun_out/rehearsal_2rank.err || { tail -30 gpurun_out/rehearsal_2rank.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/rehearsal_2rank.json'));print('2 ranks one card:', d['n_gpus'], round(d['ms_per_step'],3), d['config']['nvars_total'], d.get('config4_26var',{}).get('challenge0_lo')); print(json.dumps(d.get('multi_rank'), indent=1))"
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --force-rccl --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 > gpurun_out/force_rccl.json 2> gpurun_out/force_rccl.err || { tail -30 gpurun_out/force_rccl.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/force_rccl.json'));print('force rccl:', round(d['ms_per_step'],3), d['breakdown_per_step']['collectives'], d.get('config4_26var',{}).get('challenge0_lo')); print([x for x in d['roofline']['launches_of_proof']][:12]); print(d['breakdown_per_step']['kernel_ms_by_kind'])"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kzg -o run -- python3 tools/kzg_scale.py 24 > gpurun_out/prof_kzg.out 2> gpurun_out/prof_kzg.err || { tail gpurun_out/prof_kzg.err; exit 1; }
cat gpurun_out/prof_kzg.out
head -20 gpurun_out/prof_kzg/run_kernel_stats.csv
exit 0

# Multi-rank bench rehearsal on ONE card (ranks share device 0, gloo host all-reduce)
# and the world-1 RCCL data path; not scaling numbers.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --comm host --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 > gpurun_out/rehearsal_2rank.json 2> gpurun_out/rehearsal_2rank.err || { tail -30 gpurun_out/rehearsal_2rank.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/rehearsal_2rank.json'));print('2 ranks one card:', d['n_gpus'], round(d['ms_per_step'],3), d['config']['nvars_total'], d.get('config4_26var',{}).get('challenge0_lo'))"
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --force-rccl --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 > gpurun_out/force_rccl.json 2> gpurun_out/force_rccl.err || { tail -30 gpurun_out/force_rccl.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/force_rccl.json'));print('force rccl:', round(d['ms_per_step'],3), d['breakdown_per_step']['collectives'], d.get('config4_26var',{}).get('challenge0_lo'))"

# Round 4, final: the multi-rank rehearsal on one card (SCALE attribution fields, host
# communicator) and the forced-RCCL world-1 path, on the final tree.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --comm host --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 > gpurun_out/rehearsal_2rank.json 2> gpurun_out/rehearsal_2rank.err || { tail -30 gpurun_out/rehearsal_2rank.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --steps 5 --warmup 2 --comm host --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 > gpurun_out/rehearsal_4rank.json 2> gpurun_out/rehearsal_4rank.err || { tail -30 gpurun_out/rehearsal_4rank.err; exit 1; }
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --force-rccl --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 > gpurun_out/force_rccl.json 2> gpurun_out/force_rccl.err || { tail -30 gpurun_out/force_rccl.err; exit 1; }
for f in rehearsal_2rank rehearsal_4rank force_rccl; do python3 -c "
import json,sys;d=json.load(open('gpurun_out/$f.json'));print('$f', d['n_gpus'], round(d['ms_per_step'],3), d['config'].get('nvars_total'), d.get('config4_26var',{}).get('challenge0_lo'), d.get('config4_26var',{}).get('proof',{}).get('matches_oracle_fixture')); print(json.dumps(d.get('multi_rank'), indent=1)); print(json.dumps(d['breakdown_per_step']))"; done
exit 0

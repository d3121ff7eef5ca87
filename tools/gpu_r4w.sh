# Round 4: the bench's N = 8 code path rehearsed on one card (8 ranks, host communicator):
# weak-scaling headline at 27 variables in total, config 4 (26 variables over 8 ranks), the
# multi_rank attribution block. Diagnostic: 8 ranks share one GPU.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 8 --steps 3 --warmup 1 --comm host --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 > gpurun_out/rehearsal_8rank.json 2> gpurun_out/rehearsal_8rank.err || { tail -30 gpurun_out/rehearsal_8rank.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/rehearsal_8rank.json'));print(d['n_gpus'], round(d['ms_per_step'],3), d['config']['nvars_total'], d['proof'] if 'proof' in d else None); print(json.dumps(d.get('config4_26var'), indent=1)); print(json.dumps(d.get('multi_rank'), indent=1)[:3000])"
exit 0

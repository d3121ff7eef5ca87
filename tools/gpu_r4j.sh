# Round 4: per-layer phases of the circuit prover, and the 2-rank rehearsal after the
# host-communicator timing fix.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
ZK_DEBUG_CIRCUIT=1 timeout -k 10 120 python3 tools/circuit_phases.py 12 > gpurun_out/circ.out 2> gpurun_out/circ.err || { tail -30 gpurun_out/circ.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --comm host --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 > gpurun_out/rehearsal_2rank.json 2> gpurun_out/rehearsal_2rank.err || { tail -30 gpurun_out/rehearsal_2rank.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/rehearsal_2rank.json'));print(d['n_gpus'], round(d['ms_per_step'],3)); print(json.dumps(d['breakdown_per_step']))"
exit 0

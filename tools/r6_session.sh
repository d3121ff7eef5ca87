set -o pipefail
# round 6 session 10: the GPU parity files against the device bounds-check build; KZG verify timing
bash tools/gpu.sh checks > gpurun_out/r6_checks.log 2>&1 || { tail -30 gpurun_out/r6_checks.log; exit 1; }
tail -4 gpurun_out/r6_checks.log
timeout -k 10 600 python bench.py --no-cpu-baseline --no-fold --no-e2e --no-plain --no-config4 --steps 5 --warmup 2 > gpurun_out/kzg10.json 2> gpurun_out/kzg10.err || { tail gpurun_out/kzg10.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/kzg10.json')); k=d['config5_bls12_381']; print({x: k[x] for x in k if x.endswith('_ms') or 'verified' in x}); print(d.get('gkr_circuit_kzg'))"

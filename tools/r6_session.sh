set -o pipefail
# round 6 session 5: KZG host arithmetic (64-bit Fq rows, threaded Horners, batch-normalised proofs):
# the KZG tests, the parts at 2^10..2^16, config 5's leg; then the first t33's SQ counters vs its pattern
timeout -k 10 700 python -u -m pytest tests/test_gpu_kzg.py tests/test_gpu_gkr_circuit.py tests/test_pairing_cpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/s5_tests.log 2>&1 || { tail -30 gpurun_out/s5_tests.log; exit 1; }
tail -2 gpurun_out/s5_tests.log
timeout -k 10 300 python tools/kzg_parts.py > gpurun_out/kzg_parts2.log 2>&1 || { tail gpurun_out/kzg_parts2.log; exit 1; }
cat gpurun_out/kzg_parts2.log
timeout -k 10 600 python bench.py --no-cpu-baseline --no-fold --no-e2e --no-plain --no-config4 --steps 5 --warmup 2 > gpurun_out/kzg5.json 2> gpurun_out/kzg5.err || { tail gpurun_out/kzg5.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/kzg5.json')); k=d['config5_bls12_381']; print({x: k[x] for x in k if x.endswith('_ms') or 'verified' in x}); print(d.get('gkr_circuit_kzg'))"
bash tools/pmc_t33.sh || exit 1
python3 tools/pmc_t33_summary.py gpurun_out/pmct33_k1 gpurun_out/pmct33_k2 gpurun_out/pmct33_m1 gpurun_out/pmct33_m2

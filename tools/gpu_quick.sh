set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_prelaunch.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread -k "three_round or d0 or sharded or matrix" > gpurun_out/t_q.log 2>&1 || { tail -30 gpurun_out/t_q.log; exit 1; }
tail -2 gpurun_out/t_q.log
ZK_DEBUG_TAIL=1 timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 --no-config4 --no-events > gpurun_out/tt.json 2> gpurun_out/tt.err || { tail gpurun_out/tt.err; exit 1; }
grep "zk step" gpurun_out/tt.err | tail -5
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 > gpurun_out/b.json 2> gpurun_out/b.err || { tail gpurun_out/b.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/b.json'));print(d['ms_per_step'], d['roofline']['frac'], [(x['kind'],x['us']) for x in d['roofline']['launches_of_proof']], )"

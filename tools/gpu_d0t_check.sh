set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_prelaunch.py -k "three_round or first_double or matrix_core" > gpurun_out/t3.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/t3.log | head -20; tail -30 gpurun_out/t3.log; exit 1; }
tail -2 gpurun_out/t3.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_sharded.py > gpurun_out/t4.log 2>&1 || { tail -30 gpurun_out/t4.log; exit 1; }
tail -2 gpurun_out/t4.log
Q="--no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 --no-config4"
for cfg in "ZK_D0T=0" "ZK_D0T=1"; do env $cfg ZK_DEBUG_EVENTS=1 timeout -k 10 120 python bench.py --steps 10 --warmup 3 $Q > gpurun_out/b.json 2> gpurun_out/ev.err || exit 1; python -c "
import json;d=json.load(open('gpurun_out/b.json'));print('$cfg n=24', round(d['ms_per_step'],4))"; grep "zk: kind" gpurun_out/ev.err | tail -12 | tr '\n' ' '; echo; done

# ZK_D0Q (four rounds in the input pass + a fold by four): parity at oracle sizes, the
# BASELINE-size fixtures, then a same-box A/B against the default schedule.
set -o pipefail
mkdir -p gpurun_out
ZK_D0Q=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_prelaunch.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/d0q_small.log 2>&1 || { tail -40 gpurun_out/d0q_small.log; exit 1; }
tail -2 gpurun_out/d0q_small.log
ZK_D0Q=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 200 --timeout-method thread > gpurun_out/d0q_large.log 2>&1 || { tail -40 gpurun_out/d0q_large.log; exit 1; }
tail -2 gpurun_out/d0q_large.log
ROUNDS=${ROUNDS:-3} bash tools/gpu_ab.sh "ZK_D0Q=0" "ZK_D0Q=1"
ZK_D0Q=1 ZK_DEBUG_TAIL=1 timeout -k 10 120 python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 --no-config4 --no-plain --no-events > gpurun_out/tt_d0q.json 2> gpurun_out/tt_d0q.err || { tail gpurun_out/tt_d0q.err; exit 1; }
grep "zk " gpurun_out/tt_d0q.err | tail -14

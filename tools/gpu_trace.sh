set -o pipefail
mkdir -p gpurun_out
ZK_DEBUG_TAIL=1 timeout -k 10 120 python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 --no-config4 --no-events > gpurun_out/tt.json 2> gpurun_out/tt.err || { tail gpurun_out/tt.err; exit 1; }
grep "zk " gpurun_out/tt.err | tail -24

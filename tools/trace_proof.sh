# Kernel timeline of one pre-enqueued 24-var proof (rocprofv3 --kernel-trace), printed per dispatch
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 --no-config4 $*"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_pre -o run -- $B > gpurun_out/trace_pre_bench.json 2> gpurun_out/trace_pre.err || { tail gpurun_out/trace_pre.err; exit 1; }
python3 tools/trace_print.py gpurun_out/trace_pre/run_kernel_trace.csv

#!/bin/bash
# Kernel trace of the default bench workload, one launch per step (ZK_PRELAUNCH=0)
# and pre-enqueued; prints per-kernel durations and gaps of the last proof.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 --no-config4"
for pre in 0 1; do
  ZK_PRELAUNCH=$pre timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_pre$pre -o run -- $B > gpurun_out/trace_pre$pre.json 2> gpurun_out/trace_pre$pre.err || exit 1
done

#!/bin/bash
# Profile the default bench workload on the GPU box and keep the summaries.
#   1) rocprofv3 --kernel-trace --stats           -> per-kernel durations
#   2) rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE    -> HBM traffic (separate passes,
#      gfx950: FETCH_SIZE counts half of a wide streaming read; corrected in
#      tools/pmc_traffic.py)
# usage: tools/profile_bench.sh <tag>   (outputs in gpurun_out/prof_<tag>*)
set -e
TAG=${1:-r1}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-fold --no-e2e --no-serving --no-circuit --no-config5 --no-config4 --no-plain"
# Per-round launches while profiling: a pre-enqueued round kernel's duration
# includes its wait for the host-posted challenge, and the profiler slows the
# host; the kernels' work is identical either way.
export ZK_PRELAUNCH=0
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- $B > gpurun_out/prof_${TAG}_bench.json 2> gpurun_out/prof_${TAG}.err
# the product schedule itself: pre-enqueued steps, the
# persistent k_gkr_dtail and the host rounds, exactly what bench.py runs; each
# pre-enqueued kernel's duration then includes its wait for the challenge
ZK_PRELAUNCH=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_product -o run -- $B > gpurun_out/prof_${TAG}_product_bench.json 2>> gpurun_out/prof_${TAG}.err
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_${TAG}_fetch -o run -- $B > /dev/null 2>> gpurun_out/prof_${TAG}.err
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_${TAG}_write -o run -- $B > /dev/null 2>> gpurun_out/prof_${TAG}.err

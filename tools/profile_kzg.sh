#!/bin/bash
# rocprofv3 kernel trace + stats of KZG commits (setup + 2^NV-point commits, tools/kzg_scale.py)
# usage: tools/profile_kzg.sh <tag> [nv]   (outputs in gpurun_out/prof_<tag>*)
set -e
TAG=${1:-r5_kzg}
NV=${2:-24}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- python3 tools/kzg_scale.py $NV > gpurun_out/prof_${TAG}.log 2> gpurun_out/prof_${TAG}.err

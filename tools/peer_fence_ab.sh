#!/bin/bash
# The peer hand-off's system-scope release/acquire fences (kernels.hpp
# peer_release_fence / peer_acquire_fence) against the fence-free build
# (abtest/nofence.so: tools/build_variant.sh nofence -DZK_PEER_FENCE=0), on one
# card at world 1 through the collective path with peer reduction
# (--force-rccl --reduce peer: every sharded step publishes through
# peer_allreduce), alternating, REPS rounds of 30 proofs each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
SIDE="--no-cpu-baseline --no-fold --no-e2e --no-serving --no-circuit --no-config5 --no-plain --no-config4"
for rep in $(seq 1 ${REPS:-4}); do
  for lib in "" "$PWD/abtest/nofence.so"; do
    ZK_LIB_PATH=$lib timeout -k 10 180 python3 bench.py --force-rccl --reduce peer --steps 30 --warmup 5 $SIDE \
      > gpurun_out/pfab.json 2> gpurun_out/pfab.err || { tail -20 gpurun_out/pfab.err; exit 1; }
    python3 -c "
import json, sys
d = json.load(open('gpurun_out/pfab.json'))
print(sys.argv[1] or 'fenced (default)', round(d['ms_per_step'], 4), d.get('reduce'),
      [(x['kind'][4:], x['us']) for x in d['roofline']['launches_of_proof']], d['proof'].get('matches_oracle_fixture'))" \
      "$( [ -n "$lib" ] && echo 'no fences' )"
  done
done

#!/bin/bash
# Same-box A/B of whole trees (each with its own bench.py and library):
# alternates `python bench.py` (headline only) between the current tree and
# each tree given (e.g. abtest/r4tree, a git worktree of an earlier round with
# its library built), REPS rounds. Prints ms per proof with and without the
# per-launch events, and the event-timed launches.
# usage (inside gpurun, from the repo root): bash tools/ab_trees.sh abtest/r4tree [...]
# (EXTRA="--force-rccl": extra bench.py arguments for every run; NOEV=0: events only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
root=$PWD
SIDE="--no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 --no-plain --no-config4"
for rep in $(seq 1 ${REPS:-4}); do
  for tree in "." "$@"; do
    evs=("" "--no-events")
    [ "${NOEV:-1}" = "0" ] && evs=("")
    for ev in "${evs[@]}"; do
      (cd "$root/$tree" && timeout -k 10 180 python3 bench.py --steps 100 --warmup 20 $SIDE $EXTRA $ev \
        > "$root/gpurun_out/abt.json" 2> "$root/gpurun_out/abt.err") || { tail -20 gpurun_out/abt.err; exit 1; }
      python3 -c "
import json, sys
d = json.load(open('gpurun_out/abt.json'))
l = d['roofline']['launches_of_proof']
b = d.get('breakdown_per_step', {})
print(sys.argv[1], sys.argv[2] or 'events', round(d['ms_per_step'], 4), 'kern', round(sum(x['us'] for x in l), 1),
      [(x['kind'][4:], x['us']) for x in l], d['proof'].get('matches_oracle_fixture'))" "$tree" "$ev"
    done
  done
done

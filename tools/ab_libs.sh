#!/bin/bash
# A/B: default library vs variants in abtest/ (ZK_LIB_PATH), alternating, 20 proofs each
cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fold --no-e2e --no-serving --no-circuit --no-config5 --no-config4 --no-events"
for rep in ${REPS:-1 2 3 4 5}; do
  for lib in "" "$@"; do
    ZK_LIB_PATH=$lib timeout -k 10 120 $B > /tmp/o.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open('/tmp/o.json')); print(sys.argv[1] or 'default', round(d['ms_per_step'],4))" "$lib"
  done
done

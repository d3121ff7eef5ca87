#!/bin/bash
# A/B of environment knobs on the default bench workload (no events), alternating
# usage: tools/knobs.sh "ENV=.. ENV2=.." "ENV=.." ...   ("-" = defaults)
cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fold --no-e2e --no-serving --no-circuit --no-config5 --no-config4 --no-events"
for rep in 1 2; do
  for cfg in "$@"; do
    if [ "$cfg" = "-" ]; then e=""; else e="$cfg"; fi
    env $e timeout -k 10 120 $B > /tmp/o.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open('/tmp/o.json')); print(sys.argv[1], round(d['ms_per_step'],4))" "$cfg"
  done
done

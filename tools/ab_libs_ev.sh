#!/bin/bash
# A/B: default library vs variants in abtest/ (ZK_LIB_PATH), alternating; per run the
# proof time and the dominant launch's event time (bench asserts the proof digest)
cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 --no-config4"
for rep in ${REPS:-1 2 3}; do
  for lib in "" "$@"; do
    ZK_LIB_PATH=$lib timeout -k 10 120 $B > /tmp/o.json 2>/tmp/o.err || { tail -5 /tmp/o.err; exit 1; }
    python3 -c "
import json,sys; d=json.load(open('/tmp/o.json')); r=d['roofline']
print('%-24s %.4f ms  dominant %s %.1f us' % (sys.argv[1] or 'default', d['ms_per_step'], r['kernel'][:12], r['avg_launch_us']),
      [x['us'] for x in r.get('launches_of_proof', [])][:8])" "$lib"
  done
done

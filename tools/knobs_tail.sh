cd $GRAFT_REPO_ROOT
B="python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5"
for cfg in "ZK_TAIL=0" "ZK_TAIL_MAX_PAIRS=32768" "ZK_TAIL_MAX_PAIRS=8192" "ZK_TAIL_MAX_PAIRS=4096" "ZK_TAIL_MAX_PAIRS=1024" "ZK_TAIL_MAX_PAIRS=4096 ZK_LANES_MAX_PAIRS=65536"; do
  env $cfg timeout -k 10 120 $B > /tmp/o.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open('/tmp/o.json')); print(sys.argv[1], round(d['ms_per_step'],4), d['breakdown_per_step']['kernel_ms_by_kind'])" "$cfg"
done

# ms_per_step vs steps/warmup (default bench leg only), interleaved
set -o pipefail
mkdir -p gpurun_out
B="python3 bench.py --no-cpu-baseline --no-fold --no-e2e --no-circuit --no-config5 --no-config4"
for r in 1 2; do
  for sw in "10 3" "100 20" "10 3 --no-events" "100 20 --no-events"; do
    set -- $sw
    timeout -k 10 120 $B --steps $1 --warmup $2 $3 > gpurun_out/st.json 2> gpurun_out/st.err || { tail -5 gpurun_out/st.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/st.json')); print('round $r steps $1 warmup $2 $3', '%.4f ms' % d['ms_per_step'])"
  done
done

# One parametrised GPU-box runner (replaces the per-experiment gpu_r4*.sh
# launchers). Usage, from the repo root, inside gpurun:
#   bash tools/gpu.sh STEP [STEP ...]
# Steps run in order, each under its own time limit; the first failure ends the
# call (nothing else touches the GPU after a failing step). Outputs go to
# gpurun_out/<step>.{log,json,err}. Steps:
#   tests            every -m gpu test (+ smoke)
#   tests=EXPR       -m gpu tests selected by pytest -k EXPR
#   file=PATH        one GPU test file
#   smoke            __graft_entry__.smoke()
#   bench            the default bench line (what the driver runs)
#   quick            headline proof only (no side legs), 100 steps
#   c4               headline + config 4 only
#   self2            `python bench.py --gpus 2 --comm host` (self-launched ranks on one card)
#   self8            the same with 8 ranks (27-var headline, config 4 over 8 ranks)
#   rccl1            world 1 through the RCCL data path (--force-rccl)
#   trace            ZK_DEBUG_TAIL=1 per-step hand-off trace of the headline proof
#   blocks=S         ZK_DEBUG_BLOCKS per-block phases of step S (default 1)
#   profile=TAG      rocprofv3 kernel trace + stats of the headline (tools/profile_bench.sh TAG)
#   kzg              config 5 (BLS12-381 GKR + KZG commit) only
#   mb=NAME[:ARGS]   run tools/mb_NAME (a prebuilt microbenchmark) with ARGS
#   checks           the GPU parity files against the -DZK_DEVICE_CHECKS build
#                    (make -C zk-research-implementations_amd checks; ZK_LIB_PATH)
#   abenv=C1/C2/...  alternate bench configurations (each a comma-separated VAR=VAL list,
#                    "-" = defaults), REPS (default 5) rounds of 30 timed proofs each;
#                    prints ms per proof and the launch times of the event-timed proof
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
SIDE="--no-cpu-baseline --no-fold --no-e2e --no-serving --no-circuit --no-config5 --no-plain"

fail() { echo "step $1 failed (exit $2)"; tail -40 "$3"; exit 1; }

summ() {  # one-line summary of a bench JSON
  python3 - "$1" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
out = {"n": d["n_gpus"], "ms": round(d["ms_per_step"], 4), "Gops": round(d["value"] / 1e9, 1),
       "frac": round(r["frac"], 3), "top_us": round(r["avg_launch_us"], 1),
       "launches": [(x["kind"], x["us"]) for x in r["launches_of_proof"]][:8],
       "proof_ok": d["proof"].get("matches_oracle_fixture"), "comm": d.get("comm"), "launcher": d.get("launcher")}
if "config4_26var" in d:
    c = d["config4_26var"]
    out["c4_ms"] = round(c["ms_median"], 3)
    out["c4_ok"] = c["proof"].get("matches_oracle_fixture")
    if "launches_of_proof" in c:
        out["c4_launches"] = [(x["kind"], x["us"]) for x in c["launches_of_proof"]][:6]
if "cpu_baseline" in d:
    out["cpu_port_matches_fixture"] = d["cpu_baseline"].get("matches_fixture")
if "config5_bls12_381" in d:
    k = d["config5_bls12_381"]
    out["kzg_commit_ms"] = round(k["kzg_commit_ms"], 2)
    out["kzg_setup_ms"] = round(k["kzg_setup_ms"], 1)
print(json.dumps(out))
EOF
}

for step in "$@"; do
  name=${step%%=*}
  arg=${step#*=}
  [ "$arg" = "$step" ] && arg=""
  log=gpurun_out/$name.log
  echo "== $step"
  case $name in
    tests)
      if [ -n "$arg" ]; then
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$arg" > $log 2>&1 || fail $step $? $log
      else
        timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $log 2>&1 || fail $step $? $log
      fi
      tail -2 $log ;;
    file)
      timeout -k 10 900 python -u -m pytest "$arg" -m gpu -x -v --timeout 300 --timeout-method thread > $log 2>&1 || fail $step $? $log
      tail -3 $log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $log 2>&1 || fail $step $? $log
      tail -1 $log ;;
    bench)
      timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || fail $step $? gpurun_out/bench.err
      summ gpurun_out/bench.json ;;
    quick)
      timeout -k 10 300 python bench.py $SIDE --no-config4 > gpurun_out/quick.json 2> gpurun_out/quick.err || fail $step $? gpurun_out/quick.err
      summ gpurun_out/quick.json ;;
    c4)
      timeout -k 10 300 python bench.py $SIDE > gpurun_out/c4.json 2> gpurun_out/c4.err || fail $step $? gpurun_out/c4.err
      summ gpurun_out/c4.json ;;
    self2)
      env -u WORLD_SIZE -u RANK -u LOCAL_RANK timeout -k 10 600 python bench.py --gpus 2 --comm host --steps 10 --warmup 3 $SIDE > gpurun_out/self2.json 2> gpurun_out/self2.err || fail $step $? gpurun_out/self2.err
      summ gpurun_out/self2.json ;;
    self8)
      env -u WORLD_SIZE -u RANK -u LOCAL_RANK timeout -k 10 900 python bench.py --gpus 8 --comm host --steps 3 --warmup 1 $SIDE > gpurun_out/self8.json 2> gpurun_out/self8.err || fail $step $? gpurun_out/self8.err
      summ gpurun_out/self8.json ;;
    rccl1)
      timeout -k 10 300 python bench.py --force-rccl --steps 20 --warmup 5 $SIDE > gpurun_out/rccl1.json 2> gpurun_out/rccl1.err || fail $step $? gpurun_out/rccl1.err
      summ gpurun_out/rccl1.json ;;
    trace)
      ZK_DEBUG_TAIL=1 timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 $SIDE --no-config4 --no-events > gpurun_out/trace.json 2> gpurun_out/trace.err || fail $step $? gpurun_out/trace.err
      grep "zk step\|zk dtail\|zk host" gpurun_out/trace.err | tail -16 ;;
    blocks)
      s=${arg:-1}
      ZK_DEBUG_TAIL=1 ZK_DEBUG_BLOCKS=$s ZK_DEBUG_BLOCKS_FILE=gpurun_out/blocks_$s.csv timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 $SIDE --no-config4 --no-events > gpurun_out/blocks.json 2> gpurun_out/blocks_$s.err || fail $step $? gpurun_out/blocks_$s.err
      grep -A6 "zk step $s " gpurun_out/blocks_$s.err | tail -14 ;;
    profile)
      bash tools/profile_bench.sh "${arg:-r5}" || fail $step $? gpurun_out/prof_${arg:-r5}.err ;;
    kzg)
      timeout -k 10 600 python bench.py --no-cpu-baseline --no-fold --no-e2e --no-serving --no-circuit --no-plain --no-config4 --steps 5 --warmup 2 > gpurun_out/kzg.json 2> gpurun_out/kzg.err || fail $step $? gpurun_out/kzg.err
      summ gpurun_out/kzg.json ;;
    mb)
      prog=${arg%%:*}
      margs=${arg#*:}
      [ "$margs" = "$arg" ] && margs=""
      timeout -k 10 300 ./tools/mb_$prog $margs > gpurun_out/mb_$prog.log 2>&1 || fail $step $? gpurun_out/mb_$prog.log
      cat gpurun_out/mb_$prog.log | tail -40 ;;
    checks)
      export ZK_LIB_PATH=$PWD/zk-research-implementations_amd/zk_amd/_lib_checks/libzksumcheck.so
      [ -f "$ZK_LIB_PATH" ] || { echo "build the checks library first"; exit 1; }
      timeout -k 10 1100 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_prelaunch.py \
        tests/test_gpu_kzg.py tests/test_gpu_tables.py tests/test_gpu_gkr_circuit.py tests/test_gpu_device_fs.py \
        -m gpu -x -q --timeout 300 --timeout-method thread > $log 2>&1 || fail $step $? $log
      grep -c "zk device check failed" $log || true
      tail -2 $log
      unset ZK_LIB_PATH ;;
    abenv)
      IFS='/' read -ra cfgs <<< "$arg"
      for rep in $(seq 1 ${REPS:-5}); do
        for cfg in "${cfgs[@]}"; do
          envs=()
          [ "$cfg" != "-" ] && IFS=',' read -ra envs <<< "$cfg"
          env "${envs[@]}" timeout -k 10 120 python3 bench.py --steps 30 --warmup 5 $SIDE --no-config4 > gpurun_out/abenv.json 2> gpurun_out/abenv.err || fail $step $? gpurun_out/abenv.err
          python3 -c "
import json, sys
d = json.load(open('gpurun_out/abenv.json'))
print(sys.argv[1], round(d['ms_per_step'], 4), [(x['kind'], x['us']) for x in d['roofline']['launches_of_proof']][:5], d['proof']['matches_oracle_fixture'])" "$cfg"
        done
      done ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all steps ok"
exit 0

#!/usr/bin/env bash
# Round-6 GPU steps: STEPS selects a subset (in order); each GPU step has its own time limit
# and the first failure ends the script.  TESTK narrows the pytest step (-k expression),
# TESTF the test files.  VARS names lib_var/<v>/libsbr.so builds for the *vars steps.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r06}
mkdir -p "$OUT"
export TMPDIR=/tmp
( while true; do date +%T >> "$OUT/heartbeat.log"; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() { # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc" | tee -a "$OUT/steps.log"
  tail -c 1500 "$OUT/$name.out"; echo
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.err"; exit $rc; fi
}
VL=replication-social-bank-runs_amd/lib_var
NC="--no-cpu-baseline"
for s in ${STEPS:-tests smoke bench}; do
  case $s in
    tests) run tests 900 python -u -m pytest ${TESTF:-tests} -m gpu -x -v --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"} ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 300 python -u bench.py ;;
    drv) run drv 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 ;;
    drvnc) run drvnc 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 $NC ;;
    bench50) run bench50 300 python -u bench.py --steps 50 --warmup 5 $NC ;;
    single) run single 300 python -u bench.py --no-pipeline --steps 20 --warmup 2 $NC ;;
    config1) run config1 300 python -u bench.py --workload config1 --steps 50 --warmup 3 ;;
    config2) run config2 300 python -u bench.py --workload config2 --steps 20 --warmup 2 ;;
    strong) for v in ${SHARDS:-8 4 2}; do run strong${v}_k20 300 python -u bench.py --shard-of $v --steps 20 --warmup 5 $NC && run strong${v}_k50 300 python -u bench.py --shard-of $v --steps 50 --warmup 5 $NC; done ;;
    prof) run prof 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 $NC ;;
    profstrong) run profstrong 300 rocprofv3 --kernel-trace --stats -d "$OUT/profstrong" -o run --output-format csv -- python3 bench.py --shard-of 8 --steps 20 --warmup 5 $NC ;;
    hetero) run hetero 600 python -u bench.py --workload hetero --steps 20 --warmup 2 --phases ;;
    interest) run interest 600 python -u bench.py --workload interest --steps 3 --warmup 1 ;;
    social) run social 600 python -u bench.py --workload social --steps 1 --warmup 0 ;;
    dropin) run dropin 600 python -u bench.py --workload dropin --steps 30 ;;
    multihost) run multihost 300 python -u bench.py --workload multihost --steps 10 --warmup 2 ;;
    pmcall) for w in ${PMCW:-base hetero interest socbulk soclone}; do
              case $w in
                base) BA="--steps 20 --warmup 5" ;;
                hetero) BA="--workload hetero --steps 2 --warmup 1" ;;
                interest) BA="--workload interest --steps 1 --warmup 1" ;;
                socbulk) BA="--workload social --steps 1 --warmup 0 --social-max-iter 16" ;;
                soclone) BA="--workload social --steps 1 --warmup 0 --social-cols 2 --social-max-iter 16" ;;
              esac
              PMC_OUT=$OUT/pmc_$w BENCH_ARGS="$BA" bash tools/pmc.sh > "$OUT/pmc_$w.out" 2>&1; rc=$?
              echo "pmc_$w rc=$rc" | tee -a "$OUT/steps.log"; if [ $rc -ne 0 ]; then exit $rc; fi
            done ;;
    drvvars) for v in ${VARS:-}; do run drv_$v 300 env SBR_LIB=$VL/$v/libsbr.so python -u bench.py --gpus 1 --steps 20 --warmup 5 $NC --no-verify; done ;;
    bench50vars) for v in ${VARS:-}; do run bench50_$v 300 env SBR_LIB=$VL/$v/libsbr.so python -u bench.py --steps 50 --warmup 5 $NC --no-verify; done ;;
    strongvars) for v in ${VARS:-}; do run strong8_$v 300 env SBR_LIB=$VL/$v/libsbr.so python -u bench.py --shard-of 8 --steps 20 --warmup 5 $NC --no-verify; done ;;
    singlevars) for v in ${VARS:-}; do run single_$v 300 env SBR_LIB=$VL/$v/libsbr.so python -u bench.py --no-pipeline --steps 20 --warmup 2 $NC; done ;;
    config1vars) for v in ${VARS:-}; do run config1_$v 300 env SBR_LIB=$VL/$v/libsbr.so python -u bench.py --workload config1 --steps 50 --warmup 3 $NC; done ;;
    hetvars) for v in ${VARS:-}; do run hetero_$v 600 env SBR_LIB=$VL/$v/libsbr.so python -u bench.py --workload hetero --steps 10 --warmup 2 $NC; done ;;
    socialvars) for v in ${VARS:-}; do run social_$v 600 env SBR_LIB=$VL/$v/libsbr.so python -u bench.py --workload social --steps 1 --warmup 0 $NC --no-verify; done ;;
  esac
done

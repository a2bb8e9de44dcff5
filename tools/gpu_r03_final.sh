#!/usr/bin/env bash
# Round-3 evidence on one MI355X: parity suite, smoke, PMC passes (config 3 and 4 equilibrium
# kernels -> profiles/pmc_latest.json, copied back under gpurun_out), every bench line and a
# rocprofv3 kernel-trace summary of the config-3 bench.  Each GPU step has its own time limit;
# the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r03_final}
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
  tail -c 600 "$OUT/$name.out"; echo
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.err"; exit $rc; fi
}
for s in ${STEPS:-tests smoke pmc bench prof single config1 config2 hetero interest social}; do
  case $s in
    tests) run tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pmc)
      PMC_OUT=$OUT/pmc_base bash tools/pmc.sh > "$OUT/pmc_base.log" 2>&1 || { echo "pmc base failed"; tail -5 "$OUT/pmc_base.log"; exit 1; }
      python tools/pmc_summary.py "$OUT/pmc_base" "$OUT/pmc_base.txt" fig5_2048x2048 profiles/pmc_latest.json > /dev/null || exit 1
      PMC_OUT=$OUT/pmc_het BENCH_ARGS="--workload hetero" bash tools/pmc.sh > "$OUT/pmc_het.log" 2>&1 || { echo "pmc het failed"; tail -5 "$OUT/pmc_het.log"; exit 1; }
      python tools/pmc_summary.py "$OUT/pmc_het" "$OUT/pmc_het.txt" hetero_K8_1024x1024 profiles/pmc_latest.json > /dev/null || exit 1
      cp profiles/pmc_latest.json "$OUT/pmc_latest.json"
      echo "pmc rc=0" | tee -a "$OUT/steps.log" ;;
    bench) run bench 400 python -u bench.py ;;
    prof) run prof 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    single) run single 300 python -u bench.py --no-pipeline --steps 20 --warmup 2 --no-cpu-baseline ;;
    config1) run config1 300 python -u bench.py --workload config1 --steps 50 --warmup 3 ;;
    config2) run config2 300 python -u bench.py --workload config2 --steps 20 --warmup 2 ;;
    hetero) run hetero 600 python -u bench.py --workload hetero --steps 10 --warmup 2 --phases ;;
    interest) run interest 600 python -u bench.py --workload interest --steps 3 --warmup 1 ;;
    social) run social 600 python -u bench.py --workload social --steps 1 --warmup 0 ;;
  esac
done

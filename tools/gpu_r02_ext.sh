#!/usr/bin/env bash
# Round-2 GPU session: full parity suite, baseline bench (pipelined and single-sweep),
# hetero (config 4), interest and social (config 5 share, with a per-point dump) bench lines.
# STEPS selects a subset.  Each step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r02_ext}
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
  tail -c 2500 "$OUT/$name.out"; echo
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.err"; exit $rc; fi
}
for s in ${STEPS:-tests bench1 bench hetero interest social}; do
  case $s in
    tests) run tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    bench1) run bench1 300 python -u bench.py --no-pipeline --steps 20 --warmup 2 --no-cpu-baseline ;;
    bench) run bench 300 python -u bench.py ;;
    hetero) run hetero 600 python -u bench.py --workload hetero --steps 10 --warmup 2 ;;
    interest) run interest 600 python -u bench.py --workload interest --steps 3 --warmup 1 ;;
    social) run social 1000 python -u bench.py --workload social --steps 1 --warmup 0 --social-dump "$OUT/social_dump.npz" ;;
  esac
done

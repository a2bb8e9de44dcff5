#!/usr/bin/env bash
# One GPU session: parity tests, bench, kernel-trace profile.  Each GPU step has
# its own time limit; a fault/abort/timeout (rc >= 124 or signal) stops the script.
set -u
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
stop_if_fault() { # $1 = rc, $2 = step
  if [ "$1" -ge 124 ] || [ "$1" -ge 128 ]; then echo "FAULT/timeout in $2 (rc=$1): stopping" | tee -a "$OUT/steps.log"; exit "$1"; fi
}
STEPS="${STEPS:-tests bench prof}"
for s in $STEPS; do
  case "$s" in
    tests)
      timeout -k 10 "${TEST_TIMEOUT:-600}" python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
      rc=$?; echo "tests rc=$rc" | tee -a "$OUT/steps.log"; tail -5 "$OUT/pytest_gpu.log"; stop_if_fault $rc tests ;;
    bench)
      timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
      rc=$?; echo "bench rc=$rc" | tee -a "$OUT/steps.log"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"; stop_if_fault $rc bench ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/prof.log" 2>&1
      rc=$?; echo "prof rc=$rc" | tee -a "$OUT/steps.log"; tail -3 "$OUT/prof.log"; stop_if_fault $rc prof ;;
  esac
done

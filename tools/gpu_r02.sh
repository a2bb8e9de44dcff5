#!/usr/bin/env bash
# Round-2 GPU session driver: STEPS (space separated) chosen from
#   tests   full -m gpu parity suite            smoke   __graft_entry__.smoke()
#   bench   default bench line                  prof    rocprofv3 kernel-trace stats of the default bench
# Each GPU step has its own time limit; a fault/abort/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r02}
mkdir -p "$OUT"
export TMPDIR=/tmp
( while true; do date +%T >> "$OUT/heartbeat.log"; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
stop_if_bad() { if [ "$1" -ne 0 ]; then echo "step $2 failed (rc=$1): stopping" | tee -a "$OUT/steps.log"; exit "$1"; fi; }
for s in ${STEPS:-tests smoke bench}; do
  case "$s" in
    tests)
      timeout -k 10 "${TEST_TIMEOUT:-900}" python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
      rc=$?; echo "tests rc=$rc" | tee -a "$OUT/steps.log"; tail -3 "$OUT/pytest_gpu.log"; stop_if_bad $rc tests ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      rc=$?; echo "smoke rc=$rc" | tee -a "$OUT/steps.log"; tail -2 "$OUT/smoke.log"; stop_if_bad $rc smoke ;;
    bench)
      timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
      rc=$?; echo "bench rc=$rc" | tee -a "$OUT/steps.log"; cat "$OUT/bench.json"; stop_if_bad $rc bench ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/prof.log" 2>&1
      rc=$?; echo "prof rc=$rc" | tee -a "$OUT/steps.log"; stop_if_bad $rc prof ;;
    cmd)
      timeout -k 10 "${CMD_TIMEOUT:-600}" bash -c "$CMD" > "$OUT/cmd.log" 2>&1
      rc=$?; echo "cmd rc=$rc" | tee -a "$OUT/steps.log"; tail -20 "$OUT/cmd.log"; stop_if_bad $rc cmd ;;
  esac
done

#!/usr/bin/env bash
# A/B of libsbr variants on one workload (+ optional parity subset first):
#   TAG=x TESTK="hetero" VARIANTS="noxcd" BENCH_ARGS="--workload hetero --phases" bash tools/gpu_r02_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "${TESTK:-}" ]; then
  # TESTLIB=<variant>: run the parity subset against that build (bit-exactness of a candidate)
  if [ -n "${TESTLIB:-}" ]; then export SBR_LIB=replication-social-bank-runs_amd/lib_var/$TESTLIB/libsbr.so; fi
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread -k "$TESTK" > "$OUT/pytest.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
  unset SBR_LIB
fi
for v in base ${VARIANTS:-}; do
  if [ "$v" = base ]; then lib=replication-social-bank-runs_amd/lib/libsbr.so; else lib=replication-social-bank-runs_amd/lib_var/$v/libsbr.so; fi
  SBR_LIB=$lib timeout -k 10 300 python3 -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/$v.json" 2> "$OUT/$v.err"
  rc=$?
  python3 -c "import json; d=json.loads(open('$OUT/$v.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],3), {k: round(x,3) for k,x in d['kernel_ms_per_step'].items()}, d.get('eq_phase_ms'))" || true
  [ $rc -ne 0 ] && { echo "$v failed rc=$rc"; tail -5 "$OUT/$v.err"; exit $rc; }
done
exit 0

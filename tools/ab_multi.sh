#!/usr/bin/env bash
# Interleaved driver-style config-3 A/B of the tree's libsbr.so ("new") against lib_var/$BASE and
# the lib_var variants in $VARS (REPS rounds), then 50-step runs of base and new; GPU tests
# matching $TESTK first when set.
set -u
OUT=gpurun_out/${TAG:-r06_abm}
mkdir -p $OUT
VL=replication-social-bank-runs_amd/lib_var
D="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
if [ -n "${TESTK:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$TESTK" > $OUT/tests.out 2>&1 || exit 1
fi
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${BASE:-base} new ${VARS:-}; do
    L=""; NV="--no-verify"
    [ $v != new ] && L="env SBR_LIB=$VL/$v/libsbr.so"
    [ $v = new ] && [ $rep = 1 ] && NV=""
    timeout -k 10 300 $L python -u bench.py $D $NV > $OUT/drv_${v}_$rep.out 2>&1 || exit 1
  done
done
for v in ${BASE:-base} new; do
  L=""; [ $v != new ] && L="env SBR_LIB=$VL/$v/libsbr.so"
  timeout -k 10 300 $L python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-verify > $OUT/b50_$v.out 2>&1 || exit 1
done

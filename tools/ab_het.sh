#!/usr/bin/env bash
# Interleaved A/B of the hetero (config 4) pipelined step: the tree's libsbr.so ("new") against
# lib_var/$BASE and the lib_var variants in $VARS, REPS rounds; hetero GPU tests first.
set -u
OUT=gpurun_out/${TAG:-r06_het}
mkdir -p $OUT
VL=replication-social-bank-runs_amd/lib_var
H="--workload hetero --steps 20 --warmup 2 --no-cpu-baseline"
timeout -k 10 900 python -u -m pytest tests/test_hetero.py -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/tests.out 2>&1 || exit 1
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${BASE:-base} new ${VARS:-}; do
    L=""; NV="--no-verify"
    [ $v != new ] && L="env SBR_LIB=$VL/$v/libsbr.so"
    [ $v = new ] && [ $rep = 1 ] && NV=""
    timeout -k 10 300 $L python -u bench.py $H $NV > $OUT/het_${v}_$rep.out 2>&1 || exit 1
  done
done

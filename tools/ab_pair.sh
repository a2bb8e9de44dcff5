#!/usr/bin/env bash
# Interleaved A/B of the tree's libsbr.so against lib_var/$BASE (driver-style config-3 runs, then
# 50-step runs), REPS rounds; GPU tests first when TESTK is set.
set -u
OUT=gpurun_out/${TAG:-r06_ab}
mkdir -p $OUT
VL=replication-social-bank-runs_amd/lib_var
D="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
if [ -n "${TESTK:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$TESTK" > $OUT/tests.out 2>&1 || exit 1
fi
for rep in $(seq 1 ${REPS:-2}); do
  timeout -k 10 300 env SBR_LIB=$VL/${BASE:-base}/libsbr.so python -u bench.py $D --no-verify > $OUT/drv_base_$rep.out 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py $D > $OUT/drv_new_$rep.out 2>&1 || exit 1
done
timeout -k 10 300 env SBR_LIB=$VL/${BASE:-base}/libsbr.so python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-verify > $OUT/b50_base.out 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline > $OUT/b50_new.out 2>&1 || exit 1
# extra latency-shaped lines when EXTRA is set (single sweep, config 1, the 1/8 shard)
if [ -n "${EXTRA:-}" ]; then
  for v in base new; do
    L=""; [ $v = base ] && L="env SBR_LIB=$VL/${BASE:-base}/libsbr.so"
    timeout -k 10 300 $L python -u bench.py --shard-of 8 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/s8_$v.out 2>&1 || exit 1
    timeout -k 10 300 $L python -u bench.py --shard-of 8 --steps 50 --warmup 5 --no-cpu-baseline > $OUT/s8k50_$v.out 2>&1 || exit 1
    timeout -k 10 300 $L python -u bench.py --no-pipeline --steps 20 --warmup 2 --no-cpu-baseline > $OUT/single_$v.out 2>&1 || exit 1
    timeout -k 10 300 $L python -u bench.py --workload config1 --steps 50 --warmup 3 --no-cpu-baseline > $OUT/config1_$v.out 2>&1 || exit 1
  done
fi

#!/usr/bin/env bash
# A/B (round 6): the fused hazard normalisation (lib vs lib_var/base), and the cost of the
# timing events / per-grid events around the equilibrium launches (bench with timing off,
# lib vs lib_var/noevg).  Driver-style config-3 runs, interleaved.
set -u
OUT=gpurun_out/${TAG:-r06_ab}
mkdir -p $OUT
VL=replication-social-bank-runs_amd/lib_var
NT='import sys; sys.path.insert(0, "."); import bench, sbr; sbr.Engine.timing_enable = lambda self, on: None; sbr.Engine.timing_read = lambda self, stream=None: (1.0, 1.0, 1); sys.argv = ["bench.py", "--gpus", "1", "--steps", "20", "--warmup", "5", "--no-cpu-baseline", "--no-verify"]; bench.main()'
D="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
for rep in 1 2; do
  timeout -k 10 300 env SBR_LIB=$VL/base/libsbr.so python -u bench.py $D --no-verify > $OUT/drv_base_$rep.out 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py $D > $OUT/drv_new_$rep.out 2>&1 || exit 1
done
timeout -k 10 300 python -u -c "$NT" > $OUT/drv_new_notiming.out 2>&1 || exit 1
timeout -k 10 300 env SBR_LIB=$VL/noevg/libsbr.so python -u -c "$NT" > $OUT/drv_noevg_notiming.out 2>&1 || exit 1

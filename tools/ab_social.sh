set -u
OUT=gpurun_out/r06_soc1
mkdir -p $OUT
VL=replication-social-bank-runs_amd/lib_var
timeout -k 10 900 python -u -m pytest tests/test_gpu_social.py -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/tests.out 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 300 env SBR_LIB=$VL/base/libsbr.so python -u bench.py --workload social --steps 1 --warmup 0 --no-cpu-baseline --no-verify > $OUT/soc_base_$rep.out 2>&1 || exit 1
  NV="--no-verify"; [ $rep = 1 ] && NV=""
  timeout -k 10 300 python -u bench.py --workload social --steps 1 --warmup 0 --no-cpu-baseline $NV > $OUT/soc_new_$rep.out 2>&1 || exit 1
done

# A/B 30: learning-side priorities of the pipelined baseline batch. cur = learning streams at
# the greatest priority + hazard waves at s_setprio 3 (shipped); lo = learning streams at the
# lowest priority; np = hazard kernel without s_setprio.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/replication-social-bank-runs_amd/lib
for lib in libsbr_lo libsbr_np; do
SBR_LIB=$L/$lib.so timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/ab30_pytest_$lib.log 2>&1 || { tail -30 gpurun_out/ab30_pytest_$lib.log; exit 1; }
tail -1 gpurun_out/ab30_pytest_$lib.log
done
for lib in libsbr_cur libsbr_lo libsbr_np libsbr_cur libsbr_lo libsbr_np; do
  SBR_LIB=$L/$lib.so timeout -k 10 200 python bench.py --warmup 2 --no-cpu-baseline > gpurun_out/ab30_$lib.json 2> gpurun_out/ab30_$lib.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab30_$lib.json'));print('$lib', round(d['value']/1e9,4), round(d['ms_per_step'],4), d['kernel_ms_per_step'])"
done

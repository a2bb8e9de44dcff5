# A/B 29: learning slots of the pipelined baseline batch (3 = v13; 4, 5). With 3 the learning
# of batch k+3 (~4.4 ms incl. hazard) starts when equilibrium k ends and must finish within
# two equilibrium kernels (~4.2 ms): the trace shows 200-600 us stalls before some launches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/replication-social-bank-runs_amd/lib
for n in 4 5; do
SBR_LIB=$L/libsbr_s$n.so timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline.py tests/test_interest.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/ab29_pytest_s$n.log 2>&1 || { tail -30 gpurun_out/ab29_pytest_s$n.log; exit 1; }
tail -1 gpurun_out/ab29_pytest_s$n.log
done
for lib in libsbr_s3 libsbr_s4 libsbr_s5 libsbr_s3 libsbr_s4 libsbr_s5; do
  SBR_LIB=$L/$lib.so timeout -k 10 200 python bench.py --warmup 2 --no-cpu-baseline > gpurun_out/ab29_$lib.json 2> gpurun_out/ab29_$lib.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab29_$lib.json'));print('$lib', round(d['value']/1e9,4), round(d['ms_per_step'],4), d['kernel_ms_per_step'])"
done
SBR_LIB=$L/libsbr_s5.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab29 -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/prof_ab29.log 2>&1 || exit 1
echo rocprof ok

# A/B 27: pipelined baseline batch with one equilibrium stream (libsbr_1s, shipped) vs two
# (libsbr_2s: odd batches on a second stream, so batch k+1's workgroups fill batch k's tail).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/replication-social-bank-runs_amd/lib
SBR_LIB=$L/libsbr_2s.so timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline.py tests/test_interest.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/ab27_pytest.log 2>&1 || { tail -30 gpurun_out/ab27_pytest.log; exit 1; }
tail -1 gpurun_out/ab27_pytest.log
for lib in libsbr_1s libsbr_2s libsbr_1s libsbr_2s; do
  SBR_LIB=$L/$lib.so timeout -k 10 200 python bench.py --warmup 2 --no-cpu-baseline > gpurun_out/ab27_$lib.json 2> gpurun_out/ab27_$lib.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab27_$lib.json'));print('$lib', round(d['value']/1e9,4), round(d['ms_per_step'],4), d['kernel_ms_per_step'])"
done
export TMPDIR=/tmp
SBR_LIB=$L/libsbr_2s.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab27 -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/prof_ab27.log 2>&1 || exit 1
echo rocprof ok

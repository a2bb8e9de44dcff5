# A/B: hetero equilibrium occupancy — LDS slab capped at 7168 doubles + 2 waves/SIMD (libsbr),
# 5376 + 3 waves/SIMD (libsbr_h3) vs 1 workgroup per CU (libsbr_prev); hetero parity first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/replication-social-bank-runs_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_hetero.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/ab20_pytest.log 2>&1 || { tail -30 gpurun_out/ab20_pytest.log; exit 1; }
tail -1 gpurun_out/ab20_pytest.log
SBR_LIB=$L/libsbr_h3.so timeout -k 10 600 python -u -m pytest tests/test_hetero.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/ab20_pytest_h3.log 2>&1 || { tail -30 gpurun_out/ab20_pytest_h3.log; exit 1; }
tail -1 gpurun_out/ab20_pytest_h3.log
for rep in 1 2; do
for lib in libsbr_prev libsbr libsbr_h3; do
  SBR_LIB=$L/$lib.so timeout -k 10 300 python bench.py --workload hetero --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab20_$lib.json 2> gpurun_out/ab20_$lib.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab20_$lib.json'));print('hetero $lib', round(d['value']/1e6,4), round(d['ms_per_step'],2), d['kernel_ms_per_step'])"
done
done

# A/B: crossing-scan block interiors read 8 (libsbr) / 16 (libsbr_c16) entries per round trip
# vs one at a time (libsbr_prev); baseline + hetero (shared sbr_scan.h); parity first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/replication-social-bank-runs_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline.py tests/test_interest.py tests/test_hetero.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/ab14_pytest.log 2>&1 || { tail -30 gpurun_out/ab14_pytest.log; exit 1; }
tail -1 gpurun_out/ab14_pytest.log
SBR_LIB=$L/libsbr_c16.so timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/ab14_pytest_c16.log 2>&1 || { tail -30 gpurun_out/ab14_pytest_c16.log; exit 1; }
tail -1 gpurun_out/ab14_pytest_c16.log
for lib in libsbr_prev libsbr libsbr_c16 libsbr_prev libsbr libsbr_c16; do
  SBR_LIB=$L/$lib.so timeout -k 10 300 python bench.py --warmup 2 --no-cpu-baseline --phases > gpurun_out/ab14_$lib.json 2> gpurun_out/ab14_$lib.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab14_$lib.json'));print('$lib', round(d['value']/1e9,4), round(d['kernel_ms_per_step']['equilibrium'],3), d.get('eq_phase_ms'))"
done
for lib in libsbr_prev libsbr; do
  SBR_LIB=$L/$lib.so timeout -k 10 300 python bench.py --workload hetero --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab14_hetero_$lib.json 2> gpurun_out/ab14_hetero_$lib.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab14_hetero_$lib.json'));print('hetero $lib', round(d['value']/1e6,4), d['kernel_ms_per_step'])"
done

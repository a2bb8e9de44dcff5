# A/B: 16-wave blocks forced to 64 VGPRs (8 waves/SIMD) vs the 12-wave / 80-VGPR default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/replication-social-bank-runs_amd/lib
SBR_LIB=$L/libsbr_e1024w8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/ab11_pytest.log 2>&1 || { tail -30 gpurun_out/ab11_pytest.log; exit 1; }
tail -1 gpurun_out/ab11_pytest.log
for lib in libsbr libsbr_e1024w8 libsbr libsbr_e1024w8; do
  SBR_LIB=$L/$lib.so timeout -k 10 300 python bench.py --warmup 2 --no-cpu-baseline --phases > gpurun_out/ab11_$lib.json 2> gpurun_out/ab11_$lib.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab11_$lib.json'));print('$lib', round(d['value']/1e9,4), round(d['kernel_ms_per_step']['equilibrium'],3), d.get('eq_phase_ms'))"
done

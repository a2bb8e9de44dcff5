# A/B: AW path with the brackets' two knots held in registers and slid forward (no search
# or lerp-operand reloads per knot) at 6 waves/SIMD (80 VGPRs, libsbr) and unconstrained
# (84 VGPRs -> 5 waves/SIMD, libsbr_w5) vs the previous library; parity first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/replication-social-bank-runs_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline.py tests/test_interest.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/ab13_pytest.log 2>&1 || { tail -30 gpurun_out/ab13_pytest.log; exit 1; }
tail -1 gpurun_out/ab13_pytest.log
SBR_LIB=$L/libsbr_w5.so timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/ab13_pytest_w5.log 2>&1 || { tail -30 gpurun_out/ab13_pytest_w5.log; exit 1; }
tail -1 gpurun_out/ab13_pytest_w5.log
for lib in libsbr_prev libsbr libsbr_w5 libsbr_prev libsbr libsbr_w5; do
  SBR_LIB=$L/$lib.so timeout -k 10 300 python bench.py --warmup 2 --no-cpu-baseline --phases > gpurun_out/ab13_$lib.json 2> gpurun_out/ab13_$lib.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab13_$lib.json'));print('$lib', round(d['value']/1e9,4), round(d['kernel_ms_per_step']['equilibrium'],3), d.get('eq_phase_ms'))"
done

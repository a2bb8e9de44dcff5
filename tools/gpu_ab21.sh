# A/B: AW_max pass-1 window (8-blocks each side of the predicted peak): 6 (shipped) vs 4, 5, 8.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/replication-social-bank-runs_amd/lib
for lib in libsbr_w4 libsbr_w5 libsbr_w8; do
  SBR_LIB=$L/$lib.so timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline.py -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/ab21_pytest_$lib.log 2>&1 || { tail -30 gpurun_out/ab21_pytest_$lib.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/ab21_pytest_$lib.log)"
done
for rep in 1 2; do
for lib in libsbr libsbr_w4 libsbr_w5 libsbr_w8; do
  SBR_LIB=$L/$lib.so timeout -k 10 300 python bench.py --warmup 2 --no-cpu-baseline --phases > gpurun_out/ab21_$lib.json 2> gpurun_out/ab21_$lib.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab21_$lib.json'));print('$lib', round(d['value']/1e9,4), round(d['kernel_ms_per_step']['equilibrium'],3), d.get('eq_phase_ms'))"
done
done

# A/B: knot-interval reciprocal table in the equilibrium kernel's LDS slab (lerp_rcp:
# 3 dependent steps per lookup division instead of 11) vs the previous library; parity first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline.py tests/test_interest.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/ab12_pytest.log 2>&1 || { tail -30 gpurun_out/ab12_pytest.log; exit 1; }
tail -1 gpurun_out/ab12_pytest.log
L=$PWD/replication-social-bank-runs_amd/lib
for lib in libsbr_prev libsbr libsbr_prev libsbr; do
  SBR_LIB=$L/$lib.so timeout -k 10 300 python bench.py --warmup 2 --no-cpu-baseline --phases > gpurun_out/ab12_$lib.json 2> gpurun_out/ab12_$lib.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab12_$lib.json'));print('$lib', round(d['value']/1e9,4), round(d['kernel_ms_per_step']['equilibrium'],3), d.get('eq_phase_ms'))"
done

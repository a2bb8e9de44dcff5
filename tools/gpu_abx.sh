# Generic baseline A/B: bash tools/gpu_abx.sh TAG lib1 lib2 ...  (libs under package lib/).
# Parity (baseline + interest GPU tests) on the shipped libsbr first, then alternating benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=$1; shift
L=$PWD/replication-social-bank-runs_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline.py tests/test_interest.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for rep in 1 2; do
for lib in "$@"; do
  SBR_LIB=$L/$lib.so timeout -k 10 300 python bench.py --warmup 2 --no-cpu-baseline --phases > gpurun_out/${TAG}_$lib.json 2> gpurun_out/${TAG}_$lib.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$lib.json'));print('$lib', round(d['value']/1e9,4), round(d['kernel_ms_per_step']['equilibrium'],3), d.get('eq_phase_ms'))"
done
done

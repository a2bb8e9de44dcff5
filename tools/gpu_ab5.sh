set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/replication-social-bank-runs_amd/lib
for lib in libsbr_base libsbr_b0; do
  SBR_LIB=$L/$lib.so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --phases > gpurun_out/ab5_$lib.json 2> gpurun_out/ab5_$lib.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab5_$lib.json'));print('$lib', round(d['value']/1e6,1), round(d['ms_per_step'],3), d['kernel_ms_per_step'], d['eq_phase_ms'])"
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_baseline.py -q -m gpu --timeout 170 --timeout-method thread > gpurun_out/pytest_base.log 2>&1
echo "pytest rc=$?"
tail -2 gpurun_out/pytest_base.log

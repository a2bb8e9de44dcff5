set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/replication-social-bank-runs_amd/lib
for lib in libsbr_w6 libsbr_ilerp; do
  SBR_LIB=$L/$lib.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --phases > gpurun_out/ab3_$lib.json 2> gpurun_out/ab3_$lib.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab3_$lib.json'));print('$lib', round(d['value']/1e6,1), d['kernel_ms_per_step'], d['eq_phase_ms'])"
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_baseline.py -q -m gpu --timeout 170 --timeout-method thread > gpurun_out/pytest_base.log 2>&1
echo "pytest rc=$?"
tail -2 gpurun_out/pytest_base.log

set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_hetero.py -v -m gpu --timeout 170 --timeout-method thread > gpurun_out/pytest_hetero.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_hetero.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python bench.py --workload hetero --steps 1 --warmup 1 --no-cpu-baseline --phases > gpurun_out/hetero_ph.json 2> gpurun_out/hetero_ph.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/hetero_ph.json'));print(round(d['value']/1e6,2), d['kernel_ms_per_step'], d['eq_phase_ms'])"
fi

set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/replication-social-bank-runs_amd/lib
for lib in libsbr_base libsbr_rcp; do
  SBR_LIB=$L/$lib.so timeout -k 10 300 python bench.py --workload hetero --steps 1 --warmup 1 --no-cpu-baseline --phases > gpurun_out/ab6_$lib.json 2> gpurun_out/ab6_$lib.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab6_$lib.json'));print('$lib', round(d['value']/1e6,2), d['eq_phase_ms'])"
done
timeout -k 10 400 python -u -m pytest tests/test_hetero.py -q -m gpu --timeout 170 --timeout-method thread > gpurun_out/pytest_hetero.log 2>&1
echo "pytest rc=$?"; tail -1 gpurun_out/pytest_hetero.log

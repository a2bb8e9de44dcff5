# A/B: hetero AW_max pass-1 window around the best 8-block (0 = shipped, 1/2/4).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/replication-social-bank-runs_amd/lib
for lib in libsbr libsbr_hw1 libsbr_hw2 libsbr_hw4; do
  SBR_LIB=$L/$lib.so timeout -k 10 300 python bench.py --workload hetero --steps 2 --warmup 1 --no-cpu-baseline --phases > gpurun_out/ab9_$lib.json 2> gpurun_out/ab9_$lib.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab9_$lib.json'));print('$lib', round(d['value']/1e6,3), d['eq_phase_ms'])"
done
SBR_LIB=$L/libsbr_hw2.so timeout -k 10 400 python -u -m pytest tests/test_hetero.py -q -m gpu --timeout 170 --timeout-method thread > gpurun_out/ab9_pytest.log 2>&1
echo "pytest rc=$?"; tail -1 gpurun_out/ab9_pytest.log

# A/B: hetero AW_max / validity searches started from hints advanced by the knot distance
# (shifted arguments move with the knots) vs the previous library; hetero parity first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/replication-social-bank-runs_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_hetero.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/ab18_pytest.log 2>&1 || { tail -30 gpurun_out/ab18_pytest.log; exit 1; }
tail -1 gpurun_out/ab18_pytest.log
for lib in libsbr_prev libsbr libsbr_prev libsbr; do
  SBR_LIB=$L/$lib.so timeout -k 10 300 python bench.py --workload hetero --steps 3 --warmup 1 --no-cpu-baseline --phases > gpurun_out/ab18_$lib.json 2> gpurun_out/ab18_$lib.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab18_$lib.json'));print('hetero $lib', round(d['value']/1e6,4), d['kernel_ms_per_step'], d.get('eq_phase_ms'))"
done

# A/B: AW_max slope-bound pruning with pass-1 windows 0/1/2/3/6 vs the previous library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
( while true; do date +%T >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline.py tests/test_interest.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/ab7_pytest.log 2>&1 || { tail -30 gpurun_out/ab7_pytest.log; exit 1; }
tail -1 gpurun_out/ab7_pytest.log
L=$PWD/replication-social-bank-runs_amd/lib
for lib in libsbr_prev libsbr_w0 libsbr_w1 libsbr libsbr_w3 libsbr_w6 libsbr_prev libsbr; do
  SBR_LIB=$L/$lib.so timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --phases > gpurun_out/ab7_$lib.json 2> gpurun_out/ab7_$lib.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab7_$lib.json'));print('$lib', round(d['value']/1e9,4), round(d['kernel_ms_per_step']['equilibrium'],3), d.get('eq_phase_ms'))"
done

# Round check: full GPU parity suite, smoke, default bench (the driver's command),
# interest bench + its rocprof kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
( while true; do date +%T >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest tests/ -m gpu -v --timeout 170 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
echo "bench ok"
timeout -k 10 400 python bench.py --workload interest --steps 3 --warmup 1 > gpurun_out/interest_bench.json 2> gpurun_out/interest_bench.err || exit 1
echo "interest bench ok"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_interest -o run --output-format csv -- python bench.py --workload interest --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_interest.log 2>&1 || exit 1
echo "rocprof ok"

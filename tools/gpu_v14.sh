# v14 round evidence: full GPU suite, smoke, default bench + rocprof kernel stats, hetero bench + rocprof.
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
cat gpurun_out/bench_default.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || exit 1
echo "rocprof ok"
timeout -k 10 400 python bench.py --workload hetero --steps 10 --warmup 2 > gpurun_out/hetero_bench.json 2> gpurun_out/hetero_bench.err || exit 1
cat gpurun_out/hetero_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_hetero -o run --output-format csv -- python bench.py --workload hetero --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_hetero.log 2>&1 || exit 1
echo "hetero rocprof ok"

# Final headline evidence: PMC passes (HBM traffic), default bench (driver's command)
# reading the fresh traffic, rocprof kernel stats of the same command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
( while true; do date +%T >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
bash tools/pmc.sh > gpurun_out/pmc_run.log 2>&1 || { tail -5 gpurun_out/pmc_run.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_summary.txt gpurun_out/traffic.json fig5_2048x2048 > /dev/null || exit 1
cp gpurun_out/traffic.json profiles/traffic_latest.json
echo "pmc ok"
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
echo "bench ok"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || exit 1
echo "rocprof ok"

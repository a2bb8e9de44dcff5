# Extension bench lines: hetero (config 4) and social (config 5 per-GPU share), with rocprof stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
( while true; do date +%T >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python bench.py --workload hetero --steps 3 --warmup 1 > gpurun_out/hetero_bench.json 2> gpurun_out/hetero_bench.err || exit 1
echo "hetero ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_hetero -o run --output-format csv -- python bench.py --workload hetero --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/hetero_prof.log 2>&1 || exit 1
echo "hetero rocprof ok"
timeout -k 10 900 python bench.py --workload social --steps 1 --warmup 0 > gpurun_out/social_bench.json 2> gpurun_out/social_bench.err || exit 1
echo "social ok"

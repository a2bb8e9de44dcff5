# Headline bench (default args = the driver's) + rocprof kernel stats of the same command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
echo "bench ok"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1 || exit 1
echo "rocprof ok"

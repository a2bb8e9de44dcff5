set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --workload social --steps 1 --warmup 0 --social-prof > gpurun_out/social_full.json 2> gpurun_out/social_full.err || exit 1
echo "full ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_social -o social -- python bench.py --workload social --steps 1 --warmup 0 --social-cols 8 > gpurun_out/social_prof_run.log 2>&1 || exit 1
echo "rocprof ok"

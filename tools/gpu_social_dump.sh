set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
( while true; do date +%T >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python bench.py --workload social --steps 1 --warmup 0 --no-cpu-baseline --social-dump gpurun_out/social_dump.npz > gpurun_out/social_bench2.json 2> gpurun_out/social_bench2.err || exit 1
echo "social ok"

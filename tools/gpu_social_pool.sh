set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
( while true; do date +%T >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u -m pytest tests/test_gpu_social.py -x -v --timeout 240 --timeout-method thread > gpurun_out/pool3_pytest.log 2>&1 || exit 1
echo "tests ok"
timeout -k 10 900 python bench.py --workload social --steps 1 --warmup 0 --no-cpu-baseline --social-dump gpurun_out/social_dump5.npz > gpurun_out/social_bench5.json 2> gpurun_out/social_bench5.err || exit 1
echo "bench ok"

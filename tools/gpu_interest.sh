set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
( while true; do date +%T >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u -m pytest tests/test_interest.py -x -v --timeout 240 --timeout-method thread > gpurun_out/interest_pytest.log 2>&1 || exit 1
echo "tests ok"
timeout -k 10 400 python bench.py --workload interest --steps 3 --warmup 1 > gpurun_out/interest_bench.json 2> gpurun_out/interest_bench.err || exit 1
echo "bench ok"

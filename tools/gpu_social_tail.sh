set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
( while true; do date +%T >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 1000 python -u tools/social_tail_probe.py 6.032345649864243 > gpurun_out/social_tail.jsonl 2> gpurun_out/social_tail.err || exit 1
echo "tail ok"

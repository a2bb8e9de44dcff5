set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_social.py -v --timeout 300 --timeout-method thread > gpurun_out/social_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 240 python bench.py --workload social --steps 1 --warmup 0 --social-max-iter 3 > gpurun_out/social_probe.json 2> gpurun_out/social_probe.err
  echo "probe rc=$?"
fi

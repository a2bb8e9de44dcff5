# Full GPU check: parity tests, social probes, short baseline bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -v --timeout 170 --timeout-method thread 2>&1 | tee gpurun_out/pytest_gpu.log
rc=$?
echo "pytest rc=$rc"
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  for c in 1 64; do
    timeout -k 10 240 python bench.py --workload social --steps 1 --warmup 0 --social-max-iter 2 --social-cols $c --social-prof > gpurun_out/social_prof_c$c.json 2> gpurun_out/social_prof_c$c.err || exit 1
  done
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_short.json 2> gpurun_out/bench_short.err || exit 1
  echo "bench ok"
fi

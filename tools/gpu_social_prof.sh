set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for c in 1 64; do
  timeout -k 10 240 python bench.py --workload social --steps 1 --warmup 0 --social-max-iter 3 --social-cols $c --social-prof > gpurun_out/social_prof_c$c.json 2> gpurun_out/social_prof_c$c.err || exit 1
  echo "prof c=$c ok"
done

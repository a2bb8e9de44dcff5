set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in libsbr libsbr_exp_nolookup; do
  for c in 1 64; do
    SBR_LIB=$PWD/replication-social-bank-runs_amd/lib/$lib.so timeout -k 10 240 python bench.py --workload social --steps 1 --warmup 0 --social-max-iter 2 --social-cols $c --social-prof > gpurun_out/exp_${lib}_c$c.json 2> gpurun_out/exp_${lib}_c$c.err || exit 1
  done
done

set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/replication-social-bank-runs_amd/lib
for lib in libsbr_prev libsbr; do
  SBR_LIB=$L/$lib.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_$lib -o run --output-format csv -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-pipeline > gpurun_out/ab2_$lib.json 2> gpurun_out/ab2_$lib.err || exit 1
  echo "$lib done"
done

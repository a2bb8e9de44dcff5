# A/B: baseline bench with the previous commit's libsbr vs the working tree's.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/replication-social-bank-runs_amd/lib
for lib in libsbr_prev libsbr libsbr_prev libsbr; do
  SBR_LIB=$L/$lib.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$lib.json 2> gpurun_out/ab_$lib.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_$lib.json'));print('$lib', round(d['value']/1e6,1), d['kernel_ms_per_step'])"
done

set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/replication-social-bank-runs_amd/lib
for lib in libsbr_nod0 libsbr libsbr_nod0 libsbr; do
  SBR_LIB=$L/$lib.so timeout -k 10 300 python bench.py --workload hetero --steps 1 --warmup 1 --no-cpu-baseline --phases > gpurun_out/ab6_$lib.json 2> gpurun_out/ab6_$lib.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab6_$lib.json'));print('$lib', round(d['value']/1e6,2), d['eq_phase_ms'])"
done

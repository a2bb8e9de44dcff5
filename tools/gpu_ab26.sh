# A/B 26: NULL-stream handling of the *_dev entry points. prev = NULL -> private
# non-blocking stream (unordered with torch's default stream); null = launch on the HIP
# null stream; libsbr = private stream fenced to the null stream (fork/join events).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$PWD/replication-social-bank-runs_amd/lib
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/ab26_pytest.log 2>&1 || { tail -30 gpurun_out/ab26_pytest.log; exit 1; }
tail -1 gpurun_out/ab26_pytest.log
for lib in libsbr_prev libsbr_null libsbr libsbr_prev libsbr_null libsbr; do
  SBR_LIB=$L/$lib.so timeout -k 10 200 python bench.py --warmup 2 --no-cpu-baseline > gpurun_out/ab26_$lib.json 2> gpurun_out/ab26_$lib.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab26_$lib.json'));print('$lib', round(d['value']/1e9,4), round(d['ms_per_step'],4), d['kernel_ms_per_step'])"
done
timeout -k 10 300 python bench.py --workload hetero --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab26_hetero.json 2> gpurun_out/ab26_hetero.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/ab26_hetero.json'));print('hetero', round(d['value']/1e6,2), d['run_fraction'], d['stiff_switch_fraction'])"

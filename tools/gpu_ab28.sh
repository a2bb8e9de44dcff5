# A/B 28: event flags. base = timing events with the default system-scope fence and
# DisableTiming-only dependency events (v13); t = timing events without the system fence;
# libsbr = t + dependency events released to device scope.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/replication-social-bank-runs_amd/lib
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 170 --timeout-method thread > gpurun_out/ab28_pytest.log 2>&1 || { tail -30 gpurun_out/ab28_pytest.log; exit 1; }
tail -1 gpurun_out/ab28_pytest.log
for lib in libsbr_base libsbr_t libsbr libsbr_base libsbr_t libsbr; do
  SBR_LIB=$L/$lib.so timeout -k 10 200 python bench.py --warmup 2 --no-cpu-baseline > gpurun_out/ab28_$lib.json 2> gpurun_out/ab28_$lib.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab28_$lib.json'));print('$lib', round(d['value']/1e9,4), round(d['ms_per_step'],4), d['kernel_ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab28 -o run --output-format csv -- python bench.py --no-cpu-baseline > gpurun_out/prof_ab28.log 2>&1 || exit 1
echo rocprof ok
timeout -k 10 300 python bench.py --workload hetero --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab28_hetero.json 2> gpurun_out/ab28_hetero.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/ab28_hetero.json'));print('hetero', round(d['value']/1e6,2), d['run_fraction'], d['stiff_switch_fraction'], d['kernel_ms_per_step'])"

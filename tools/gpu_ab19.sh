# Hetero pipelined batch sweep (sbr_sweep_hetero_batch_dev): parity (hetero GPU tests incl.
# batch == single sweeps), then the config-4 bench serial (--no-pipeline) vs pipelined.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hetero.py -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/ab19_pytest.log 2>&1 || { tail -30 gpurun_out/ab19_pytest.log; exit 1; }
tail -1 gpurun_out/ab19_pytest.log
for mode in "--no-pipeline" "" "--no-pipeline" ""; do
  tag=${mode:+serial}; tag=${tag:-pipelined}
  timeout -k 10 300 python bench.py --workload hetero --steps 10 --warmup 2 --no-cpu-baseline $mode > gpurun_out/ab19_$tag.json 2> gpurun_out/ab19_$tag.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab19_$tag.json'));print('hetero $tag', round(d['value']/1e6,4), round(d['ms_per_step'],2), d['kernel_ms_per_step'])"
done

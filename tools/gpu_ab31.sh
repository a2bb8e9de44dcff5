# Diagnostic 31: default bench vs the same with per-launch timing events off (ms_per_step only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in on off on off; do
  if [ $v = on ]; then timeout -k 10 200 python bench.py --warmup 2 --no-cpu-baseline > gpurun_out/ab31_$v.json 2> gpurun_out/ab31_$v.err || exit 1
  else timeout -k 10 200 python tools/bench_notiming_probe.py > gpurun_out/ab31_$v.json 2> gpurun_out/ab31_$v.err || exit 1; fi
  python -c "import json;d=json.load(open('gpurun_out/ab31_$v.json'));print('timing_$v', round(d['value']/1e9,4), round(d['ms_per_step'],4))"
done

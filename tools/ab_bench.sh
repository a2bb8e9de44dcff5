#!/usr/bin/env bash
# A/B of libsbr variants (tools/build_variant.sh) on the default pipelined bench:
#   VARIANTS="hz0 lr0" bash tools/ab_bench.sh   (base = lib/libsbr.so)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
for v in base ${VARIANTS:-}; do
  if [ "$v" = base ]; then lib=replication-social-bank-runs_amd/lib/libsbr.so; else lib=replication-social-bank-runs_amd/lib_var/$v/libsbr.so; fi
  SBR_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/$v.json" 2> "$OUT/$v.err"
  rc=$?
  python3 -c "import json,sys; d=json.loads(open('$OUT/$v.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['kernel_ms_per_step'].items()})" || true
  [ $rc -ne 0 ] && { echo "$v failed rc=$rc"; tail -5 "$OUT/$v.err"; exit $rc; }
done
exit 0

#!/usr/bin/env bash
# PMC counter passes (tools/pmc.sh) for the baseline (config 3) and hetero (config 4)
# equilibrium kernels, summarised into profiles/pmc_latest.json (bench.py's traffic and
# frac_executed), then a hetero bench line with the per-phase breakdown.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r02_pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
PMC_OUT=$OUT/base bash tools/pmc.sh > "$OUT/base_run.log" 2>&1 || { tail -5 "$OUT/base_run.log"; exit 1; }
python tools/pmc_summary.py "$OUT/base" "$OUT/pmc_base.txt" fig5_2048x2048 profiles/pmc_latest.json > /dev/null || exit 1
echo "base pmc ok"
PMC_OUT=$OUT/het BENCH_ARGS="--workload hetero" bash tools/pmc.sh > "$OUT/het_run.log" 2>&1 || { tail -5 "$OUT/het_run.log"; exit 1; }
python tools/pmc_summary.py "$OUT/het" "$OUT/pmc_het.txt" hetero_K8_1024x1024 profiles/pmc_latest.json > /dev/null || exit 1
cp profiles/pmc_latest.json "$OUT/pmc_latest.json"
echo "hetero pmc ok"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
tail -1 "$OUT/bench.json"
timeout -k 10 400 python -u bench.py --workload hetero --steps 10 --warmup 2 --no-cpu-baseline --phases > "$OUT/hetero.json" 2> "$OUT/hetero.err" || exit 1
tail -1 "$OUT/hetero.json"

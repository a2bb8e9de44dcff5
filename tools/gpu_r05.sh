#!/usr/bin/env bash
# Round-5 GPU steps: STEPS selects a subset (in order); each GPU step has its own time limit
# and the first failure ends the script.  TESTK narrows the pytest step (-k expression).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r05}
mkdir -p "$OUT"
export TMPDIR=/tmp
( while true; do date +%T >> "$OUT/heartbeat.log"; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() { # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc" | tee -a "$OUT/steps.log"
  tail -c 1500 "$OUT/$name.out"; echo
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.err"; exit $rc; fi
}
for s in ${STEPS:-tests smoke bench single}; do
  case $s in
    tests) run tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"} ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 300 python -u bench.py ;;
    single) run single 300 python -u bench.py --no-pipeline --steps 20 --warmup 2 --no-cpu-baseline ;;
    ready) run ready 300 python -u bench.py --no-pipeline --ready --steps 20 --warmup 2 --no-cpu-baseline ;;
    prof) run prof 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    profsingle) run profsingle 300 rocprofv3 --kernel-trace --stats -d "$OUT/profsingle" -o run --output-format csv -- python3 bench.py --no-pipeline --steps 20 --warmup 2 --no-cpu-baseline ;;
    hetero) run hetero 600 python -u bench.py --workload hetero --steps 20 --warmup 2 --phases ;;
    interest) run interest 600 python -u bench.py --workload interest --steps 3 --warmup 1 ;;
    social) run social 600 python -u bench.py --workload social --steps 1 --warmup 0 ;;
    config1) run config1 300 python -u bench.py --workload config1 --steps 50 --warmup 3 ;;
    phases) run phases 300 python -u bench.py --phases --steps 10 --warmup 2 --no-cpu-baseline ;;
    wgtime) run wgtime 300 env SBR_LIB=replication-social-bank-runs_amd/lib_var/wgtime/libsbr.so WG_OUT=$OUT/wgtime.npz python -u tools/wgtime.py ;;
    phasevars) for v in ${VARS:-}; do run phases_$v 300 env SBR_LIB=replication-social-bank-runs_amd/lib_var/$v/libsbr.so python -u bench.py --phases --steps 10 --warmup 2 --no-cpu-baseline; done ;;
    pmc) PMC_OUT=$OUT/pmc bash tools/pmc.sh > "$OUT/pmc.out" 2>&1; echo "pmc rc=$?" | tee -a "$OUT/steps.log" ;;
    pmceq) run pmceq_valu 180 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$OUT/pmceq_valu" -o pass -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify
           for fl in 0x100 0x200 0; do run pmceq_lds_$fl 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES --output-format csv -d "$OUT/pmceq_lds_$fl" -o pass -- python3 tools/eq_diag_run.py $fl; done ;;
    pmcphase) for fl in 0x100 0x200 0; do run pmcph_$fl 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/pmcph_$fl" -o pass -- python3 tools/eq_diag_run.py $fl; done ;;
    socprobe) run socprobe 600 python -u tools/social_step_probe.py ${PROBE_ITERS:-8} && run socprobe_nocoop 600 env SBR_LIB=replication-social-bank-runs_amd/lib_var/nocoop/libsbr.so python -u tools/social_step_probe.py ${PROBE_ITERS:-8} ;;
    socphase) run socphase 600 python -u tools/social_phase_probe.py ${PROBE_ITERS:-8} && run socphase_nocoop 600 env SBR_LIB=replication-social-bank-runs_amd/lib_var/nocoop/libsbr.so python -u tools/social_phase_probe.py ${PROBE_ITERS:-8} ;;
    soctrace) run soctrace 600 env SBR_SOCIAL_TRACE=1 python -u bench.py --workload social --steps 1 --warmup 0 --no-cpu-baseline ;;
    soctracevar) run soctrace_$VAR 600 env SBR_SOCIAL_TRACE=1 SBR_LIB=replication-social-bank-runs_amd/lib_var/$VAR/libsbr.so python -u bench.py --workload social --steps 1 --warmup 0 --no-cpu-baseline ;;
    socdump) run socdump 600 python -u bench.py --workload social --steps 1 --warmup 0 --no-cpu-baseline --social-dump $OUT/social_dump.npz ;;
    vartests) for v in ${VARS:-}; do run tests_$v 900 env SBR_LIB=replication-social-bank-runs_amd/lib_var/$v/libsbr.so python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"}; done ;;
    hetvars) for v in ${VARS:-}; do run hetero_$v 600 env SBR_LIB=replication-social-bank-runs_amd/lib_var/$v/libsbr.so python -u bench.py --workload hetero --steps 10 --warmup 2 --phases --no-cpu-baseline; done ;;
    pmcall) for w in ${PMCW:-base hetero interest socbulk soclone}; do
              case $w in
                base) BA="--steps 4 --warmup 2" ;;  # whole 2-grid launches only (SBR_LEARN_GROUP)
                hetero) BA="--workload hetero --steps 2 --warmup 1" ;;
                interest) BA="--workload interest --steps 1 --warmup 1" ;;
                socbulk) BA="--workload social --steps 1 --warmup 0 --social-max-iter 16" ;;
                soclone) BA="--workload social --steps 1 --warmup 0 --social-cols 2 --social-max-iter 16" ;;
              esac
              PMC_OUT=$OUT/pmc_$w BENCH_ARGS="$BA" bash tools/pmc.sh > "$OUT/pmc_$w.out" 2>&1; rc=$?
              echo "pmc_$w rc=$rc" | tee -a "$OUT/steps.log"; if [ $rc -ne 0 ]; then exit $rc; fi
            done ;;
    socprof) run socprof 300 python -u bench.py --workload social --steps 1 --warmup 0 --social-max-iter 16 --social-prof --no-cpu-baseline --no-verify ;;
    knotsprobevars) for v in ${VARS:-}; do run knotsprobe_$v 300 env SBR_LIB=replication-social-bank-runs_amd/lib_var/$v/libsbr.so python -u tools/knots_probe.py 2000; done ;;
    benchvars) for v in ${VARS:-}; do run bench_$v 300 env SBR_LIB=replication-social-bank-runs_amd/lib_var/$v/libsbr.so python -u bench.py --no-cpu-baseline; done ;;
    socialvars) for v in ${VARS:-}; do run social_$v 600 env SBR_LIB=replication-social-bank-runs_amd/lib_var/$v/libsbr.so python -u bench.py --workload social --steps 1 --warmup 0 --no-cpu-baseline --no-verify; done ;;
    socprofvars) for v in ${VARS:-}; do run socprof_$v 300 env SBR_LIB=replication-social-bank-runs_amd/lib_var/$v/libsbr.so python -u bench.py --workload social --steps 1 --warmup 0 --social-max-iter 16 --social-prof --no-cpu-baseline --no-verify; done ;;
    config2) run config2 300 python -u bench.py --workload config2 --steps 20 --warmup 2 ;;
    dropin) run dropin 600 python -u bench.py --workload dropin --steps 30 ;;
    knotsprobe) run knotsprobe 300 python -u tools/knots_probe.py 2000 && run knotsprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/knotsprof" -o run --output-format csv -- python3 tools/knots_probe.py 500 ;;
    dpp) run dpp 60 ./tools/micro/dpp_newbcast ;;
    drv) run drv 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 ;;
    strong) for v in ${SHARDS:-8 4 2}; do run strong${v}_k20 300 python -u bench.py --shard-of $v --steps 20 --warmup 5 --no-cpu-baseline && run strong${v}_k50 300 python -u bench.py --shard-of $v --steps 50 --warmup 5; done ;;
    strongvars) for v in ${VARS:-}; do run strong8_$v 300 env SBR_LIB=replication-social-bank-runs_amd/lib_var/$v/libsbr.so python -u bench.py --shard-of 8 --steps 20 --warmup 5 --no-cpu-baseline; done ;;
    profstrong) run profstrong 300 rocprofv3 --kernel-trace --stats -d "$OUT/profstrong" -o run --output-format csv -- python3 bench.py --shard-of 8 --steps 20 --warmup 5 --no-cpu-baseline ;;
    hetero2) run hetero2 600 python -u bench.py --workload hetero --steps 10 --warmup 2 --phases --no-cpu-baseline ;;
    socprof2) run socprof2 300 python -u bench.py --workload social --steps 1 --warmup 0 --social-max-iter 16 --social-prof --no-cpu-baseline --no-verify ;;
    multihost) run multihost 300 python -u bench.py --workload multihost --steps 10 --warmup 2 ;;
    drv50) run drv50 300 python -u bench.py --gpus 1 --steps 50 --warmup 5 ;;
    profconfig1) run profconfig1 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/profconfig1" -o run --output-format csv -- python3 bench.py --workload config1 --steps 50 --warmup 3 ;;
    soclone) run soclone 300 python -u bench.py --workload social --steps 1 --warmup 0 --social-cols 2 --social-max-iter 16 --social-prof --no-cpu-baseline --no-verify ;;
    soclonevars) for v in ${VARS:-}; do run soclone_$v 300 env SBR_LIB=replication-social-bank-runs_amd/lib_var/$v/libsbr.so python -u bench.py --workload social --steps 1 --warmup 0 --social-cols 2 --social-max-iter 16 --social-prof --no-cpu-baseline --no-verify; done ;;
    interestvars) for v in ${VARS:-}; do run interest_$v 600 env SBR_LIB=replication-social-bank-runs_amd/lib_var/$v/libsbr.so python -u bench.py --workload interest --steps 3 --warmup 1 --no-cpu-baseline; done ;;
    drvvars) for v in ${VARS:-}; do run drv_$v 300 env SBR_LIB=replication-social-bank-runs_amd/lib_var/$v/libsbr.so python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline; done ;;
    singlevars) for v in ${VARS:-}; do run single_$v 300 env SBR_LIB=replication-social-bank-runs_amd/lib_var/$v/libsbr.so python -u bench.py --no-pipeline --steps 20 --warmup 2 --no-cpu-baseline; done ;;
    config1vars) for v in ${VARS:-}; do run config1_$v 300 env SBR_LIB=replication-social-bank-runs_amd/lib_var/$v/libsbr.so python -u bench.py --workload config1 --steps 50 --warmup 3 --no-cpu-baseline; done ;;
    abrep) for i in 1 2; do run rep${i}_base 300 python -u bench.py --no-cpu-baseline --no-verify && for v in ${VARS:-}; do run rep${i}_$v 300 env SBR_LIB=replication-social-bank-runs_amd/lib_var/$v/libsbr.so python -u bench.py --no-cpu-baseline --no-verify; done && run rep${i}_drvbase 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-verify && for v in ${VARS:-}; do run rep${i}_drv$v 300 env SBR_LIB=replication-social-bank-runs_amd/lib_var/$v/libsbr.so python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-verify; done; done ;;
    knots) run knots 600 python -u -m pytest tests/test_gpu_knots.py tests/test_gpu_baseline.py -x -v --timeout 300 --timeout-method thread ${KTESTK:+-k "$KTESTK"} ;;
  esac
done

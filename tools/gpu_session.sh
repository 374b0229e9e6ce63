#!/bin/bash
# One GPU session on the box: each step under its own timeout; stop at the
# first step that crashes (rc > 1) so nothing else touches a faulted GPU.
#   tools/gpu_session.sh tests smoke bench bench_cfg3 ab_cfg2 prof_cfg2 pmc_cfg2 sq_long
# Knobs (environment of the session script only, never read by the library):
#   K=<pytest -k expr> for ktests; VARIANTS / PERCU / ROUNDS / REPS / PAIR=1 /
#   TAG (log name suffix) for ab_*; PMCS for pmc_*.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
# heartbeat: every step has its own timeout, so a hung step is ended by that,
# not by gpurun's silence limit (long bench / profile steps print at the end)
( while sleep 50; do echo "[hb $(date +%T)]"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
PYT="python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread"
for step in "$@"; do
  echo "[step $step start $(date +%T)]"
  case $step in
    tests)   timeout -k 10 900 $PYT tests -m gpu > gpurun_out/gpu_tests.log 2>&1; rc=$?
             grep -c PASSED gpurun_out/gpu_tests.log
             tail -4 gpurun_out/gpu_tests.log ;;
    ttests)  timeout -k 10 900 $PYT tests -m "gpu and tuning" --tuning > gpurun_out/gpu_ttests.log 2>&1; rc=$?
             tail -4 gpurun_out/gpu_ttests.log ;;
    ktests)  timeout -k 10 600 $PYT tests -m gpu -k "$K" > gpurun_out/gpu_ktests.log 2>&1; rc=$?
             tail -15 gpurun_out/gpu_ktests.log | cut -c1-300 ;;
    kttests) timeout -k 10 600 $PYT tests -m gpu -k "$K" --tuning > gpurun_out/gpu_kttests.log 2>&1; rc=$?
             tail -15 gpurun_out/gpu_kttests.log | cut -c1-300 ;;
    smoke)   timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tee gpurun_out/smoke.log; rc=$?
             tail -1 gpurun_out/smoke.log ;;
    bench)   timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1; rc=$?
             tail -1 gpurun_out/bench.log | cut -c1-600 ;;
    bench_*) cfg=${step#bench_}
             timeout -k 10 300 python bench.py --config $cfg > "gpurun_out/$step.log" 2>&1; rc=$?
             tail -1 "gpurun_out/$step.log" | cut -c1-600 ;;
    ab_*)    w=${step#ab_}
             timeout -k 10 400 python tools/abbench.py --work $w --variants ${VARIANTS:-0} --per-cu ${PERCU:-0} --rounds ${ROUNDS:-5} --reps ${REPS:-10} ${PAIR:+--pair} > "gpurun_out/$step${TAG:-}.log" 2>&1; rc=$?
             grep -v amdgpu.ids "gpurun_out/$step${TAG:-}.log" | cut -c1-260 ;;
    prof_*)  cfg=${step#prof_}; d="gpurun_out/$step"
             timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$d" -o run --output-format csv -- python3 bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-host > "$d.log" 2>&1; rc=$?
             python3 -c "import csv,sys; [print(r['Name'][:90], r['Calls'], r['AverageNs']) for r in csv.DictReader(open(sys.argv[1])) if 'pdht' in r['Name']]" "$d/run_kernel_stats.csv" ;;
    hyg_*)   cfg=${step#hyg_}; d="gpurun_out/hyg/$cfg"; mkdir -p "$d"
             # one bench line and the rocprof kernel trace + stats OF THAT RUN (cfg2 without the
             # configs[4] block, which has its own step: hyg_config4)
             extra=""; [ "$cfg" = cfg2 ] && extra="--no-config4"
             timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$d" -o run --output-format csv -- python3 bench.py --config $cfg $extra ${HYGARGS:-} > "$d/bench.json" 2> "$d/bench.err"; rc=$?
             tail -1 "$d/bench.json" | cut -c1-300 ;;
    pmc_*)   cfg=${step#pmc_}; rc=0; i=0
             # PMCS: counter groups separated by ';' (one rocprofv3 pass each)
             IFS=';' read -ra groups <<< "${PMCS:-FETCH_SIZE;WRITE_SIZE}"
             for grp in "${groups[@]}"; do
               i=$((i+1))
               timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_${cfg}_$i" -o run --output-format csv -- python3 bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline --no-host --no-config4 > gpurun_out/pmc_${cfg}_$i.log 2>&1 || { rc=$?; break; }
             done ;;
    sq_*)    cfg=${step#sq_}
             timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/sq_$cfg" -o run --output-format csv -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-host > gpurun_out/sq_$cfg.log 2>&1; rc=$?
             tail -3 gpurun_out/sq_$cfg.log | cut -c1-300 ;;
    profab_*) w=${step#profab_}; d="gpurun_out/$step"
             # rocprof kernel stats of the A/B harness's workload (product only)
             timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$d" -o run --output-format csv -- python3 tools/abbench.py --work $w --variants ${VARIANTS:-0} --rounds ${ROUNDS:-3} --reps ${REPS:-10} ${PAIR:+--pair} > "$d.log" 2>&1; rc=$?
             python3 -c "import csv,sys; [print(r['Name'][:90], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs']) for r in csv.DictReader(open(sys.argv[1])) if 'pdht' in r['Name']]" "$d/run_kernel_stats.csv" ;;
    sqab_*)  w=${step#sqab_}
             # SQ counters of the A/B harness's variants (one rocprofv3 pass; kernels told apart by name)
             timeout -s KILL 200 rocprofv3 --pmc ${PMCS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS} --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/sqab_$w" -o run --output-format csv -- python3 tools/abbench.py --work $w --variants ${VARIANTS:-0} --rounds 1 --reps 3 > gpurun_out/sqab_$w.log 2>&1; rc=$?
             python3 tools/pmc_summary.py gpurun_out/sqab_$w/run_counter_collection.csv ;;
    rehearse2) # the N = 2 path end to end on one GPU: 2 ranks, gloo collectives, both ranks on device 0
             timeout -k 10 500 python bench.py --gpus 2 --dist-backend gloo > gpurun_out/rehearse2.log 2>&1; rc=$?
             tail -1 gpurun_out/rehearse2.log | cut -c1-900 ;;
    rehearse2_*) cfg=${step#rehearse2_}  # the N = 2 gloo rehearsal of another config
             timeout -k 10 500 python bench.py --gpus 2 --dist-backend gloo --config $cfg > "gpurun_out/$step.log" 2>&1; rc=$?
             tail -1 "gpurun_out/$step.log" | cut -c1-900 ;;
    clk_*)   cfg=${step#clk_}  # per-dispatch clock: GRBM_GUI_ACTIVE cycles over the traced duration
             timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/clk_$cfg" -o run --output-format csv -- python3 bench.py --config $cfg --steps ${STEPS:-50} --warmup ${WARM:-10} --no-cpu-baseline --no-host > gpurun_out/clk_$cfg.log 2>&1; rc=$?
             tail -1 gpurun_out/clk_$cfg.log | cut -c1-300 ;;
    rehearse4) # N = 4 the same way: 4 ranks on device 0 (configs[4] = 4 x 256M keys)
             timeout -k 10 800 python bench.py --gpus 4 --dist-backend gloo > gpurun_out/rehearse4.log 2>&1; rc=$?
             tail -1 gpurun_out/rehearse4.log | cut -c1-1500 ;;
    rehearse8) # N = 8, the driver's scaling run, the same way: 8 ranks on device 0 (cfg2 shards 0..7,
             # configs[4] = 8 x 128M keys, the CPU baseline on rank 0 while the others wait)
             timeout -k 10 900 python bench.py --gpus 8 --dist-backend gloo > gpurun_out/rehearse8.log 2>&1; rc=$?
             tail -1 gpurun_out/rehearse8.log | cut -c1-1500 ;;
    torchrun1) timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-host > gpurun_out/torchrun1.log 2>&1; rc=$?
             tail -1 gpurun_out/torchrun1.log | cut -c1-600 ;;
    *) echo "unknown step $step"; rc=0 ;;
  esac
  echo "[step $step rc=$rc]"
  [ $rc -le 1 ] || exit $rc
done

#!/bin/bash
# One GPU session on the box: each step under its own timeout; stop at the
# first step that crashes (rc > 1) so nothing else touches a faulted GPU.
#   tools/gpu_session.sh tests smoke bench kbench kbench_crc prof
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for step in "$@"; do
  case $step in
    tests)   timeout -k 10 700 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?
             tail -4 gpurun_out/gpu_tests.log ;;
    smoke)   timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
             tail -1 gpurun_out/smoke.log ;;
    bench)   timeout -k 10 240 python bench.py > gpurun_out/bench.log 2>&1; rc=$?
             tail -1 gpurun_out/bench.log ;;
    bench_*) cfg=${step#bench_}; v=${cfg#*@}; [ "$v" = "$cfg" ] && v=0; cfg=${cfg%@*}
             timeout -k 10 300 python bench.py --config $cfg --variant $v --no-cpu-baseline > "gpurun_out/$step.log" 2>&1; rc=$?
             tail -1 "gpurun_out/$step.log" ;;
    kbench)  timeout -k 10 300 python tools/kbench.py > gpurun_out/kbench.log 2>&1; rc=$?
             grep -v amdgpu.ids gpurun_out/kbench.log | cut -c1-200 ;;
    kbench_pc) timeout -k 10 400 python tools/kbench.py --variants 0,15 --per-cu 3,4,5 --rounds 7 > gpurun_out/kbench_pc.log 2>&1; rc=$?
             grep -v amdgpu.ids gpurun_out/kbench_pc.log | cut -c1-200 ;;
    kbench_crc_pc) timeout -k 10 400 python tools/kbench.py --algo crc128 --variants 0,15 --per-cu 2,4,6 --rounds 5 > gpurun_out/kbench_crc_pc.log 2>&1; rc=$?
             grep -v amdgpu.ids gpurun_out/kbench_crc_pc.log | cut -c1-200 ;;
    kbench_crc) timeout -k 10 300 python tools/kbench.py --algo crc128 > gpurun_out/kbench_crc.log 2>&1; rc=$?
             grep -v amdgpu.ids gpurun_out/kbench_crc.log | cut -c1-200 ;;
    prof)    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host > gpurun_out/prof.log 2>&1; rc=$?
             head -3 gpurun_out/prof/run_kernel_stats.csv | cut -c1-200 ;;
    prof_*)  cfg=${step#prof_}; v=${cfg#*@}; [ "$v" = "$cfg" ] && v=0; cfg=${cfg%@*}; d="gpurun_out/$step"
             timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$d" -o run --output-format csv -- python3 bench.py --config $cfg --variant $v --steps 20 --warmup 3 --no-cpu-baseline --no-host > "$d.log" 2>&1; rc=$?
             python3 -c "import csv,sys; [print(r['Name'][:70], r['Calls'], r['AverageNs']) for r in csv.DictReader(open(sys.argv[1])) if 'pdht' in r['Name']]" "$d/run_kernel_stats.csv" ;;
    pmc_*)   cfg=${step#pmc_}; rc=0; i=0
             # PMCS: counter groups separated by ';' (one rocprofv3 pass each)
             IFS=';' read -ra groups <<< "${PMCS:-FETCH_SIZE;WRITE_SIZE}"
             for grp in "${groups[@]}"; do
               i=$((i+1))
               timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_${cfg}_$i" -o run --output-format csv -- python3 bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline --no-host > gpurun_out/pmc_${cfg}_$i.log 2>&1 || { rc=$?; break; }
             done ;;
    pmc)     rc=0
             for ctr in FETCH_SIZE WRITE_SIZE; do
               timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$ctr" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host > gpurun_out/pmc_$ctr.log 2>&1 || { rc=$?; break; }
             done ;;
    vartests) timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider -k "var or cfg3 or host or smoke" > gpurun_out/gpu_vartests.log 2>&1; rc=$?
             tail -3 gpurun_out/gpu_vartests.log ;;
    ktests)  timeout -k 10 300 python -m pytest tests -m gpu -x -q -p no:cacheprovider -k "$K" > gpurun_out/gpu_ktests.log 2>&1; rc=$?
             tail -15 gpurun_out/gpu_ktests.log | cut -c1-300 ;;
    varbench)timeout -k 10 300 python tools/varbench.py --variants ${VARIANTS:-0,11,12,13,14,10} > gpurun_out/varbench.log 2>&1; rc=$?
             grep -v amdgpu.ids gpurun_out/varbench.log ;;
    torchrun1) timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-host > gpurun_out/torchrun1.log 2>&1; rc=$?
             tail -1 gpurun_out/torchrun1.log | cut -c1-400 ;;
    placebench) timeout -k 10 300 python tools/placebench.py --variants ${PVARIANTS:-0,16,17} > gpurun_out/placebench.log 2>&1; rc=$?
             grep -v amdgpu.ids gpurun_out/placebench.log | cut -c1-220 ;;
    bucketbench) timeout -k 10 300 python tools/bucketbench.py --variants ${BVARIANTS:-0,41} ${BARGS:-} >> gpurun_out/bucketbench.log 2>&1; rc=$?
             grep -v amdgpu.ids gpurun_out/bucketbench.log | cut -c1-400 ;;
    counters) timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1; rc=$?; rc=0 ;;
    sq_*)    cfg=${step#sq_}
             timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/sq_$cfg" -o run --output-format csv -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-host > gpurun_out/sq_$cfg.log 2>&1; rc=$?
             tail -3 gpurun_out/sq_$cfg.log | cut -c1-300 ;;
    *) echo "unknown step $step"; rc=0 ;;
  esac
  echo "[step $step rc=$rc]"
  [ $rc -le 1 ] || exit $rc
done

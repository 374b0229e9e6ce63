#!/bin/bash
# PMC passes over an A/B workload (tools/abbench.py), one rocprofv3 run per
# counter group (a group within the per-block limits), each in its own
# directory; prints the per-dispatch means per kernel.
#   W=bucket8krot VARIANTS=0,290 tools/pmc_ab.sh "SQ_WAVE_CYCLES SQ_WAIT_ANY" "FETCH_SIZE" "WRITE_SIZE"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  d="gpurun_out/pmc_${W}_$i"
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace -d "$GRAFT_REPO_ROOT/$d" -o run --output-format csv -- \
    python3 tools/abbench.py --work "$W" --variants "${VARIANTS:-0}" --rounds 1 --reps 3 > "$d.log" 2>&1 || exit $?
  echo "== $grp"
  python3 tools/pmc_summary.py "$d/run_counter_collection.csv"
done

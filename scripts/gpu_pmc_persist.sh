#!/bin/bash
# Clock / MFMA-busy PMC of the persistent recurrences: the fp32 ones (c2 shape, scripts/f32_step_ab.py)
# and the bf16 ones (c3, and the c4 / c5 rank shapes: scripts/persist_ab.py), each counter set in its own rocprofv3 run, plus a
# kernel trace for the durations.  scripts/pmc_persist.py folds them.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/pmc_persist
mkdir -p $D
export TMPDIR=/tmp
for w in ${WORKLOADS:-f32 bf16 c4 c5}; do
  case $w in
    f32) CMD="scripts/f32_step_ab.py --only auto --iters 1";;
    bf16) CMD="scripts/persist_ab.py --iters 1";;
    c4) CMD="scripts/persist_ab.py --iters 1 --B 80 --T 160";;
    c5) CMD="scripts/persist_ab.py --iters 1 --B 320 --T 180";;
  esac
  timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d $D/${w}_pmc -o p -- python3 $CMD > $D/${w}_pmc.log 2>&1 || { echo "$w pmc rc=$?"; tail -5 $D/${w}_pmc.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/${w}_trace -o p -- python3 $CMD > $D/${w}_trace.log 2>&1 || { echo "$w trace rc=$?"; exit 1; }
done
find $D -name "*.csv" | head

#!/bin/bash
# PMC counters for the kernel micro-bench (own run; --pmc never combined with tracing).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
for set in "${PMC_SETS[@]:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE}"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc -o pass$i -- python3 ${PMC_SCRIPT:-scripts/kbench.py} > gpurun_out/pmc/pass$i.log 2>&1 || { echo "pmc pass $i failed rc=$?"; tail -5 gpurun_out/pmc/pass$i.log; exit 1; }
done
ls gpurun_out/pmc

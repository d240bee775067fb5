#!/bin/bash
# PMC passes over scripts/pmc_kernels.py (isolated K2 + fp32 GEMM launches); each pass its own run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
sets=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
      "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
      "FETCH_SIZE"
      "WRITE_SIZE"
      "TCC_HIT_sum TCC_MISS_sum")
i=0
for set in "${sets[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc2 -o pass$i -- python3 scripts/pmc_kernels.py > gpurun_out/pmc2/pass$i.log 2>&1 || { echo "pass $i rc=$?"; tail -3 gpurun_out/pmc2/pass$i.log; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc2 -o trace -- python3 scripts/pmc_kernels.py > gpurun_out/pmc2/trace.log 2>&1
echo trace rc=$?
ls gpurun_out/pmc2 | head -30

#!/bin/bash
# PMC passes (clock, MFMA busy, waits) over scripts/gemm_pmc.py; GEMM_ENVS selects our variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/gpmc
export TMPDIR=/tmp
sets=("GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES"
      "GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_LDS SQ_WAVES")
for kv in ${GEMM_ENVS:-SV_GEMM_PIPE=1}; do
  i=0
  for set in "${sets[@]}"; do
    i=$((i+1))
    env $kv timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/gpmc -o ${kv}_pass$i -- python3 scripts/gemm_pmc.py > gpurun_out/gpmc/${kv}_pass$i.log 2>&1 || { echo "pass $kv $i rc=$?"; tail -3 gpurun_out/gpmc/${kv}_pass$i.log; exit 1; }
  done
  env $kv timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gpmc -o ${kv}_trace -- python3 scripts/gemm_pmc.py > gpurun_out/gpmc/${kv}_trace.log 2>&1 || exit 1
done
ls gpurun_out/gpmc | head -40

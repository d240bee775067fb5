#!/bin/bash
# PMC of the c3 dx GEMM, fragment-order A (product) vs row-major A (noafr build): one counter set per
# rocprofv3 run over scripts/persist_ab.py --iters 1; folded by scripts/pmc_kernels.py
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; D=gpurun_out/afr_pmc; mkdir -p $D
i=0
for v in prod noafr; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  for set in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $D/${v}_$i -o p -- python3 scripts/persist_ab.py $L --iters 1 > $D/${v}_$i.log 2>&1 || { echo "$v $set rc=$?"; tail -5 $D/${v}_$i.log; exit 1; }
  done
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $D/${v}_trace -o p -- python3 scripts/persist_ab.py $L --iters 1 > $D/${v}_trace.log 2>&1 || { echo "$v trace rc=$?"; exit 1; }
done
echo done

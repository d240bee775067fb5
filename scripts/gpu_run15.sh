#!/bin/bash
# fp32 NT GEMM column-group width (SV_GF_GROUP: 4 = tree; gf3 / gf6 / gf12 A/B builds): time at the
# c2 shapes (scripts/gemm_bench.py) and the FETCH_SIZE pass of each (scripts/gpu_gemm_traffic.sh)
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1; mkdir -p gpurun_out/r15
for i in 1 2; do
  for L in prod gf3 gf6 gf12; do
    LIBARG=""; [ "$L" != prod ] && LIBARG="--lib scripts/ab/libsv_ge2e_$L.so"
    timeout -k 10 200 python scripts/gemm_bench.py --bias --reps 10 --shapes Gx,dx $LIBARG > gpurun_out/r15/gemm_${L}_$i.log 2>&1 || { echo "gemm $L failed"; tail -5 gpurun_out/r15/gemm_${L}_$i.log; exit 1; }
    echo "$L $(tail -n 1 gpurun_out/r15/gemm_${L}_$i.log)"
  done
done
ABLIBS="gf3 gf6 gf12" bash scripts/gpu_gemm_traffic.sh > gpurun_out/r15/traffic.log 2>&1 || { echo "traffic failed"; tail -5 gpurun_out/r15/traffic.log; exit 1; }
echo traffic done

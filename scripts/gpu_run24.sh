#!/bin/bash
# fp32 K1: persistent gemm_f32_256p_kernel (prod) vs the one-shot gemm_f32_256_kernel (nopers), exact fp32 both
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1; mkdir -p gpurun_out/r24
for i in 1 2 3; do
  for L in prod nopers; do
    LIBARG=""; [ "$L" != prod ] && LIBARG="--lib scripts/ab/libsv_ge2e_$L.so"
    timeout -k 10 200 python scripts/gemm_bench.py --bias --reps 10 --shapes Gx $LIBARG > gpurun_out/r24/gemm_${L}_$i.log 2>&1 || { echo "gemm $L failed"; tail -5 gpurun_out/r24/gemm_${L}_$i.log; exit 1; }
    echo "$L $(tail -n 1 gpurun_out/r24/gemm_${L}_$i.log)"
  done
done

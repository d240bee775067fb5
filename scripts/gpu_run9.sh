#!/bin/bash
# fp32 persistent K1 (next tile's k-tile 0 during the last k-tile) vs the previous tree (base)
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1; mkdir -p gpurun_out/r10
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r10/pt_kernels.log 2>&1 || { echo "kernel tests rc=$?"; tail -30 gpurun_out/r10/pt_kernels.log; exit 1; }
tail -1 gpurun_out/r10/pt_kernels.log
for i in 1 2; do
  for L in prod base; do
    LIBARG=""; [ "$L" != prod ] && LIBARG="--lib scripts/ab/libsv_ge2e_$L.so"
    timeout -k 10 200 python scripts/gemm_bench.py --bias --reps 10 --shapes Gx,dx $LIBARG > gpurun_out/r10/gemm_${L}_$i.log 2>&1 || { echo "gemm $L failed"; tail -5 gpurun_out/r10/gemm_${L}_$i.log; exit 1; }
    echo "$L $(tail -n 1 gpurun_out/r10/gemm_${L}_$i.log)"
  done
done
for i in 1 2; do
  for L in prod base; do
    LIBARG=""; [ "$L" != prod ] && LIBARG="--lib scripts/ab/libsv_ge2e_$L.so"
    timeout -k 10 200 python scripts/f32_step_ab.py --only auto --iters 5 $LIBARG > gpurun_out/r10/c2_${L}_$i.log 2>&1 || { echo "c2 $L failed"; tail -5 gpurun_out/r10/c2_${L}_$i.log; exit 1; }
    echo "c2 $L $(tail -n 1 gpurun_out/r10/c2_${L}_$i.log | cut -c1-200)"
  done
done

#!/bin/bash
# GEMM epilogue A/B: product (persistent fp32 K1, bias loads batched / staged in LDS) against the
# previous tree (base), the product without the persistent fp32 form (gfp0) and a no-store
# diagnostic build (nost); then the c2 / c3 stacks prod vs base, alternated.
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1; mkdir -p gpurun_out/r8
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r8/pt_kernels.log 2>&1 || { echo "kernel tests rc=$?"; tail -30 gpurun_out/r8/pt_kernels.log; exit 1; }
tail -1 gpurun_out/r8/pt_kernels.log
for i in 1 2; do
  for L in prod base gfp0 nost; do
    LIBARG=""; [ "$L" != prod ] && LIBARG="--lib scripts/ab/libsv_ge2e_$L.so"
    timeout -k 10 200 python scripts/gemm_bench.py --bf16 --bias --reps 10 --shapes Gx,dx $LIBARG > gpurun_out/r8/gemm_${L}_$i.log 2>&1 || { echo "gemm $L failed"; tail -5 gpurun_out/r8/gemm_${L}_$i.log; exit 1; }
    echo "$L $(tail -n 1 gpurun_out/r8/gemm_${L}_$i.log)"
  done
done
for i in 1 2; do
  for L in prod base; do
    LIBARG=""; [ "$L" != prod ] && LIBARG="--lib scripts/ab/libsv_ge2e_$L.so"
    timeout -k 10 200 python scripts/f32_step_ab.py --only auto --iters 5 $LIBARG > gpurun_out/r8/c2_${L}_$i.log 2>&1 || { echo "c2 $L failed"; tail -5 gpurun_out/r8/c2_${L}_$i.log; exit 1; }
    echo "c2 $L $(tail -n 1 gpurun_out/r8/c2_${L}_$i.log | cut -c1-260)"
    timeout -k 10 200 python scripts/persist_ab.py --iters 5 $LIBARG > gpurun_out/r8/c3_${L}_$i.log 2>&1 || { echo "c3 $L failed"; tail -5 gpurun_out/r8/c3_${L}_$i.log; exit 1; }
    echo "c3 $L $(tail -n 1 gpurun_out/r8/c3_${L}_$i.log | cut -c1-260)"
  done
done

#!/bin/bash
# (1) fp32 model tests (persistent backward with the cross-half A prefetch);
# (2) c2 step: prod (cross-half prefetch) vs noxpf, twice, one box;
# (3) bf16 K1 GEMM check (no bias: bf16 out == RNE of fp32 out) and column-group A/B of the persistent bf16 K1
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1; mkdir -p gpurun_out/r13
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_status.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r13/pt_model.log 2>&1 || { echo "model tests rc=$?"; tail -30 gpurun_out/r13/pt_model.log; exit 1; }
tail -1 gpurun_out/r13/pt_model.log
for i in 1 2; do
  for L in prod noxpf; do
    LIBARG=""; [ "$L" != prod ] && LIBARG="--lib scripts/ab/libsv_ge2e_$L.so"
    timeout -k 10 200 python scripts/f32_step_ab.py --only auto --iters 5 $LIBARG > gpurun_out/r13/c2_${L}_$i.log 2>&1 || { echo "c2 $L failed"; tail -5 gpurun_out/r13/c2_${L}_$i.log; exit 1; }
    echo "c2 $L $(tail -n 1 gpurun_out/r13/c2_${L}_$i.log | cut -c1-300)"
  done
done
timeout -k 10 200 python scripts/gemm_bench.py --bf16 --check --reps 4 --shapes Gx > gpurun_out/r13/gemm_check.log 2>&1 || { echo "gemm check failed"; tail -5 gpurun_out/r13/gemm_check.log; exit 1; }
echo "check $(tail -n 1 gpurun_out/r13/gemm_check.log)"
for i in 1 2; do
  for L in prod grp2 grp3 grp4 grp6; do
    LIBARG=""; [ "$L" != prod ] && LIBARG="--lib scripts/ab/libsv_ge2e_$L.so"
    timeout -k 10 200 python scripts/gemm_bench.py --bf16 --bias --reps 10 --shapes Gx $LIBARG > gpurun_out/r13/gemm_${L}_$i.log 2>&1 || { echo "gemm $L failed"; tail -5 gpurun_out/r13/gemm_${L}_$i.log; exit 1; }
    echo "$L $(tail -n 1 gpurun_out/r13/gemm_${L}_$i.log)"
  done
done

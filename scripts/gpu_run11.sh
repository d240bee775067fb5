#!/bin/bash
# fp32 cell activations (v_exp/v_rcp forms): full GPU suite, forward phase stamps, c2 A/B vs base
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1; mkdir -p gpurun_out/r12
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r12/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r12/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r12/pytest_gpu.log
timeout -k 10 200 python scripts/f32_step_ab.py --only auto --iters 3 --stamps --lib scripts/ab/libsv_ge2e_pfst.so > gpurun_out/r12/pfst.log 2>&1 || { echo "stamps failed"; tail -5 gpurun_out/r12/pfst.log; exit 1; }
tail -n 1 gpurun_out/r12/pfst.log
for i in 1 2; do
  for L in prod base; do
    LIBARG=""; [ "$L" != prod ] && LIBARG="--lib scripts/ab/libsv_ge2e_$L.so"
    timeout -k 10 200 python scripts/f32_step_ab.py --only auto --iters 5 $LIBARG > gpurun_out/r12/c2_${L}_$i.log 2>&1 || { echo "c2 $L failed"; tail -5 gpurun_out/r12/c2_${L}_$i.log; exit 1; }
    echo "c2 $L $(tail -n 1 gpurun_out/r12/c2_${L}_$i.log | cut -c1-230)"
  done
done

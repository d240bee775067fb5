#!/bin/bash
# fp32 persistent backward: hand-off stores straight from registers (prod) vs read back from the
# LDS dG tile (ldsho, the previous kernel); phase stamps of both (pfst / ldshost); model tests on prod
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1; mkdir -p gpurun_out/r19
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_status.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r19/pt_model.log 2>&1 || { echo "model tests rc=$?"; tail -30 gpurun_out/r19/pt_model.log; exit 1; }
tail -1 gpurun_out/r19/pt_model.log
for i in 1 2; do
  for L in prod ldsho; do
    LIBARG=""; [ "$L" != prod ] && LIBARG="--lib scripts/ab/libsv_ge2e_$L.so"
    timeout -k 10 200 python scripts/f32_step_ab.py --only auto --iters 5 $LIBARG > gpurun_out/r19/c2_${L}_$i.log 2>&1 || { echo "c2 $L failed"; tail -5 gpurun_out/r19/c2_${L}_$i.log; exit 1; }
    echo "c2 $L $(tail -n 1 gpurun_out/r19/c2_${L}_$i.log | cut -c1-300)"
  done
done
for L in pfst ldshost; do
  timeout -k 10 200 python scripts/f32_step_ab.py --only auto --iters 3 --stamps --lib scripts/ab/libsv_ge2e_$L.so > gpurun_out/r19/st_${L}.log 2>&1 || { echo "stamps $L failed"; tail -5 gpurun_out/r19/st_${L}.log; exit 1; }
  echo "$L $(tail -n 1 gpurun_out/r19/st_${L}.log)"
done

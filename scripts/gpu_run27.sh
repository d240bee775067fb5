#!/bin/bash
# fp32 persistent backward: raw barrier after the hand-off poll (prod) vs __syncthreads (sync); gradients bitwise, tests, A/B, stamps
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1; mkdir -p gpurun_out/r27
for L in prod sync; do
  LIBARG=""; [ "$L" != prod ] && LIBARG="--lib scripts/ab/libsv_ge2e_$L.so"
  timeout -k 10 200 python scripts/f32_bwd_dump.py $LIBARG gpurun_out/r27/g_$L.pt >> gpurun_out/r27/dump.log 2>&1 || { echo "dump $L failed"; tail -20 gpurun_out/r27/dump.log; exit 1; }
done
echo "prod vs sync $(python scripts/f32_bwd_dump.py --compare gpurun_out/r27/g_prod.pt gpurun_out/r27/g_sync.pt | cut -c1-80)"
rm -f gpurun_out/r27/*.pt
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_status.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r27/pt_model.log 2>&1 || { echo "model tests rc=$?"; tail -30 gpurun_out/r27/pt_model.log; exit 1; }
tail -1 gpurun_out/r27/pt_model.log
for i in 1 2 3; do
  for L in prod sync; do
    LIBARG=""; [ "$L" != prod ] && LIBARG="--lib scripts/ab/libsv_ge2e_$L.so"
    timeout -k 10 200 python scripts/f32_step_ab.py --only auto --iters 5 $LIBARG > gpurun_out/r27/c2_${L}_$i.log 2>&1 || { echo "c2 $L failed"; tail -5 gpurun_out/r27/c2_${L}_$i.log; exit 1; }
    echo "c2 $L $(tail -n 1 gpurun_out/r27/c2_${L}_$i.log | cut -c1-300)"
  done
done
timeout -k 10 200 python scripts/f32_step_ab.py --only auto --iters 3 --stamps --lib scripts/ab/libsv_ge2e_pfst.so > gpurun_out/r27/st_pfst.log 2>&1 || { echo "stamps failed"; tail -5 gpurun_out/r27/st_pfst.log; exit 1; }
echo "pfst $(tail -n 1 gpurun_out/r27/st_pfst.log | cut -c1-1200)"

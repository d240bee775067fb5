#!/bin/bash
# fp32 persistent backward, cross-half A prefetch with the epilogue's first wait at vmcnt(P):
# prod (wave 0 polls + barrier) vs wpoll (every wave polls, no barrier) vs noxpf; model tests on prod
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1; mkdir -p gpurun_out/r14
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r14/pt_model.log 2>&1 || { echo "model tests rc=$?"; tail -30 gpurun_out/r14/pt_model.log; exit 1; }
tail -1 gpurun_out/r14/pt_model.log
for i in 1 2; do
  for L in prod wpoll noxpf; do
    LIBARG=""; [ "$L" != prod ] && LIBARG="--lib scripts/ab/libsv_ge2e_$L.so"
    timeout -k 10 200 python scripts/f32_step_ab.py --only auto --iters 5 $LIBARG > gpurun_out/r14/c2_${L}_$i.log 2>&1 || { echo "c2 $L failed"; tail -5 gpurun_out/r14/c2_${L}_$i.log; exit 1; }
    echo "c2 $L $(tail -n 1 gpurun_out/r14/c2_${L}_$i.log | cut -c1-300)"
  done
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_precision.py -x -q -s --timeout 300 --timeout-method thread -k "chunks or c5_rank or c3_full" > gpurun_out/r14/pt_chunks.log 2>&1 || { echo "chunk tests rc=$?"; tail -30 gpurun_out/r14/pt_chunks.log; exit 1; }
grep -E "MEASURED|passed|failed" gpurun_out/r14/pt_chunks.log
timeout -k 10 400 python -u scripts/rank_shapes.py --steps 5 --warmup 2 > gpurun_out/r14/rank_shapes.log 2>&1 || { echo "rank shapes rc=$?"; tail -30 gpurun_out/r14/rank_shapes.log; exit 1; }
grep '^{' gpurun_out/r14/rank_shapes.log

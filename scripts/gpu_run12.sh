#!/bin/bash
# (1) every multi-GPU bench line's per-rank shape alone on this GPU (scripts/rank_shapes.py);
# (2) bf16 K1 (persistent 8-phase, bf16 out): prod (store tail drained behind k-tile 0's phases 0-2)
#     vs noast (drained before k-tile 0) vs g8nost (no C stores: diagnostic, invalid results)
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1; mkdir -p gpurun_out/r12
timeout -k 10 200 python scripts/gemm_bench.py --bf16 --bias --check --reps 4 --shapes Gx > gpurun_out/r12/gemm_check.log 2>&1 || { echo "gemm check failed"; tail -5 gpurun_out/r12/gemm_check.log; exit 1; }
echo "check $(tail -n 1 gpurun_out/r12/gemm_check.log)"
for i in 1 2; do
  for L in prod noast g8nost; do
    LIBARG=""; [ "$L" != prod ] && LIBARG="--lib scripts/ab/libsv_ge2e_$L.so"
    timeout -k 10 200 python scripts/gemm_bench.py --bf16 --bias --reps 10 --shapes Gx,dx $LIBARG > gpurun_out/r12/gemm_${L}_$i.log 2>&1 || { echo "gemm $L failed"; tail -5 gpurun_out/r12/gemm_${L}_$i.log; exit 1; }
    echo "$L $(tail -n 1 gpurun_out/r12/gemm_${L}_$i.log)"
  done
done
timeout -k 10 400 python -u scripts/rank_shapes.py --steps 5 --warmup 2 > gpurun_out/r12/rank_shapes.log 2>&1 || { echo "rank shapes rc=$?"; tail -30 gpurun_out/r12/rank_shapes.log; exit 1; }
grep '^{' gpurun_out/r12/rank_shapes.log

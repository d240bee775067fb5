#!/bin/bash
# fp32 persistent backward A-fragment weight k-groups in LDS: 24 (prod) vs 20 vs 28 (c2 stack A/B, 3 rounds)
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1; mkdir -p gpurun_out/r33
for i in 1 2 3; do
  for L in prod nl20 nl28; do
    LIBARG=""; [ "$L" != prod ] && LIBARG="--lib scripts/ab/libsv_ge2e_$L.so"
    timeout -k 10 200 python scripts/f32_step_ab.py --only auto --iters 5 $LIBARG > gpurun_out/r33/c2_${L}_$i.log 2>&1 || { echo "c2 $L failed"; tail -5 gpurun_out/r33/c2_${L}_$i.log; exit 1; }
    echo "c2 $L $(tail -n 1 gpurun_out/r33/c2_${L}_$i.log | cut -c1-300)"
  done
done

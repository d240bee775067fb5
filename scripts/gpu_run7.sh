#!/bin/bash
# fp32 persistent vs per-step schedule at small batches (d-vector per-file call, c5 rank, c1)
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1; mkdir -p gpurun_out
for cfg in "128 24" "320 180" "20 160" "640 160"; do
  set -- $cfg
  for s in persist per_step; do
    timeout -k 10 200 python scripts/f32_step_ab.py --only $s --iters 3 --B $1 --T $2 > gpurun_out/f32sched_$1_$2_$s.log 2>&1 || { echo "$cfg $s failed"; tail -3 gpurun_out/f32sched_$1_$2_$s.log; exit 1; }
    echo "B=$1 T=$2 $s $(tail -n 1 gpurun_out/f32sched_$1_$2_$s.log | cut -c1-300)"
  done
done

#!/bin/bash
# fp32 K1 (persistent 256p GEMM) with non-temporal C stores (k1nt) vs base: isolated rate + c2 step
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-f32k1}; mkdir -p $O
for r in 1 2 3; do
for v in base ${ABV:-k1nt}; do
  echo "== $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/gemm_bench.py --shapes Gx --bias --reps 5 --lib scripts/ab/libsv_ge2e_$v.so >> $O/ab.log 2>&1 || { echo "gemm $v rc=$?"; tail -5 $O/ab.log; exit 1; }
  timeout -k 10 200 python -u scripts/f32_step_ab.py --lib scripts/ab/libsv_ge2e_$v.so --only persist --iters 3 >> $O/ab.log 2>&1 || { echo "f32 $v rc=$?"; tail -5 $O/ab.log; exit 1; }
done
done
grep -E '^(==|\{"lib|\{"B)' $O/ab.log | cut -c1-220

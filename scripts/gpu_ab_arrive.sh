#!/bin/bash
# last arriver skips its next poll (al: -DSV_ARRIVE_LAST=1) vs product: c4 rank-shape wavefronts and
# the c3 persistent recurrences (bf16)
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-arrive}; mkdir -p $O
for r in 1 2 3; do
for v in prod ${ABV:-al}; do
  L="--lib scripts/ab/libsv_ge2e_$v.so"; [ $v = prod ] && L=""
  echo "== $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/wave_stamps.py $L --iters 10 >> $O/ab.log 2>&1 || { echo "c4 $v rc=$?"; tail -5 $O/ab.log; exit 1; }
  timeout -k 10 200 python -u scripts/persist_ab.py $L --iters 5 >> $O/ab.log 2>&1 || { echo "c3 $v rc=$?"; tail -5 $O/ab.log; exit 1; }
  [ -n "$F32" ] && { timeout -k 10 200 python -u scripts/f32_step_ab.py $L --only persist --iters 3 >> $O/ab.log 2>&1 || { echo "f32 $v rc=$?"; tail -5 $O/ab.log; exit 1; }; }
done
done
grep -E '^(==|\{)' $O/ab.log | cut -c1-250

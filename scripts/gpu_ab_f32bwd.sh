#!/bin/bash
# fp32 persistent backward A/B: product vs scripts/ab/libsv_ge2e_${B:-syncbar}.so (f32_step_ab, 3 rounds)
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-f32bwd}; mkdir -p $O
for r in 1 2 3; do
for v in prod ${B:-syncbar}; do
  L="--lib scripts/ab/libsv_ge2e_$v.so"; [ $v = prod ] && L=""
  echo "== f32 $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/f32_step_ab.py $L --only persist --iters 3 >> $O/ab.log 2>&1 || { echo "f32 $v rc=$?"; tail -5 $O/ab.log; exit 1; }
done
done
grep -E '^(==|\{"persist)' $O/ab.log | cut -c1-300

#!/bin/bash
# c5-rank bf16 stack timings (scripts/persist_ab.py --B 320 --T 180), product vs VARIANTS, 3 rounds
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-p16ab}; mkdir -p $O
for r in 1 2 3; do for v in prod $VARIANTS; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  echo "== $v" >> $O/ab.log
  timeout -k 10 120 python -u scripts/persist_ab.py $L --B 320 --T 180 --iters 5 >> $O/ab.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/ab.log; exit 1; }
done; done
grep -E '^(==|\{)' $O/ab.log | cut -c1-200
echo done

#!/bin/bash
# c4-rank bf16 stack timings (scripts/persist_ab.py --B 80, 2 rounds) and one kernel trace each for
# the product and the A/B builds in VARIANTS
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-dwab}; mkdir -p $O
V="prod ${VARIANTS:-nodw}"
for r in 1 2; do for v in $V; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  echo "== $v" >> $O/ab.log
  timeout -k 10 120 python -u scripts/persist_ab.py $L --B 80 --T 160 --iters 5 >> $O/ab.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/ab.log; exit 1; }
done; done
grep -E '^(==|\{)' $O/ab.log | cut -c1-200
for v in $V; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$v -o run -- python3 scripts/persist_ab.py $L --B 80 --T 160 --iters 5 > $O/$v.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/$v.log; exit 1; }
done
echo done

#!/bin/bash
# bf16 stack A/B of the persistent + stream-K GEMM forms: product vs scripts/ab/libsv_ge2e_{$VARIANTS}.so
# at c3 (B 640, T 160), the c4 rank (B 80, T 160) and the c5 rank (B 320, T 180); persist_ab.py, 3 rounds
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-g8sk}; mkdir -p $O
VARIANTS=${VARIANTS:-"dwoff nosk"}
for r in 1 2 3; do
for shape in "640 160" "80 160" "320 180"; do
set -- $shape
for v in prod $VARIANTS; do
  L="--lib scripts/ab/libsv_ge2e_$v.so"; [ $v = prod ] && L=""
  echo "== $v B=$1 T=$2" >> $O/ab.log
  timeout -k 10 200 python -u scripts/persist_ab.py $L --B $1 --T $2 --iters 5 >> $O/ab.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/ab.log; exit 1; }
done
done
done
grep -E '^(==|\{)' $O/ab.log | cut -c1-300

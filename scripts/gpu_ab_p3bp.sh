#!/bin/bash
# persist3 backward A-fragment prefetch depth 10 with 14 W_hh^T k-steps in LDS (p10) vs product (8 / 12)
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-p3bp}; mkdir -p $O
V=${ABV:-p10}
timeout -k 10 200 python -u scripts/bitident_ab.py --B 640 --out $O/prod.pt > $O/bi.log 2>&1 || { echo "prod rc=$?"; tail -5 $O/bi.log; exit 1; }
timeout -k 10 200 python -u scripts/bitident_ab.py --B 640 --lib scripts/ab/libsv_ge2e_$V.so --out $O/ab.pt >> $O/bi.log 2>&1 || { echo "$V rc=$?"; tail -5 $O/bi.log; exit 1; }
python scripts/bitident_ab.py --compare $O/prod.pt $O/ab.pt || { echo "differs"; exit 1; }
rm -f $O/*.pt
for r in 1 2 3; do
for v in prod $V; do
  L="--lib scripts/ab/libsv_ge2e_$v.so"; [ $v = prod ] && L=""
  echo "== $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/persist_ab.py $L --iters 5 >> $O/ab.log 2>&1 || { echo "c3 $v rc=$?"; tail -5 $O/ab.log; exit 1; }
done
done
grep -E '^(==|\{)' $O/ab.log | cut -c1-200

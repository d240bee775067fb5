#!/bin/bash
# backward wavefront with its hand-off in two halves of unit blocks (hv: -DSV_WB_HALVES=1) vs product:
# bit-identity at the c4 rank shape (and B = 96, 192 rows), timing, phase stamps
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-halves}; mkdir -p $O
for B in 80 96 640; do
  timeout -k 10 200 python -u scripts/bitident_ab.py --B $B --out $O/prod_$B.pt > $O/bi.log 2>&1 || { echo "prod $B rc=$?"; tail -5 $O/bi.log; exit 1; }
  timeout -k 10 200 python -u scripts/bitident_ab.py --B $B --lib scripts/ab/libsv_ge2e_hv.so --out $O/hv_$B.pt >> $O/bi.log 2>&1 || { echo "hv $B rc=$?"; tail -5 $O/bi.log; exit 1; }
  python scripts/bitident_ab.py --compare $O/prod_$B.pt $O/hv_$B.pt || { echo "B=$B differs"; exit 1; }
done
rm -f $O/*.pt
for r in 1 2 3; do
for v in prod hv; do
  L="--lib scripts/ab/libsv_ge2e_$v.so"; [ $v = prod ] && L=""
  echo "== $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/wave_stamps.py $L --iters 10 >> $O/ab.log 2>&1 || { echo "c4 $v rc=$?"; tail -5 $O/ab.log; exit 1; }
  timeout -k 10 200 python -u scripts/persist_ab.py $L --iters 5 >> $O/ab.log 2>&1 || { echo "c3 $v rc=$?"; tail -5 $O/ab.log; exit 1; }
done
done
for v in wst hvst; do
  echo "== $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/wave_stamps.py --lib scripts/ab/libsv_ge2e_$v.so --iters 5 >> $O/ab.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/ab.log; exit 1; }
done
grep -E '^(==|\{)' $O/ab.log | cut -c1-200

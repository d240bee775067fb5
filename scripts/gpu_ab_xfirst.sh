#!/bin/bash
# wavefront forward: x-part before the own-h wait + h tile in two LDS objects (xf) vs product
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-xfirst}; mkdir -p $O
for r in 1 2 3; do
for v in prod xf; do
  L="--lib scripts/ab/libsv_ge2e_$v.so"; [ $v = prod ] && L=""
  echo "== $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/wave_stamps.py $L --iters 10 >> $O/ab.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/ab.log; exit 1; }
done
done
for v in wst xfst; do
  echo "== $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/wave_stamps.py --lib scripts/ab/libsv_ge2e_$v.so --iters 5 >> $O/ab.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/ab.log; exit 1; }
done
cat $O/ab.log | cut -c1-400

#!/bin/bash
# the weight-gradient GEMMs in the persistent + stream-K form (-DSV_G8_SK_DW=1: no slab reduce) at the
# c4 / c5 rank shapes vs the split-K slabs + reduce (product): 3 interleaved rounds of persist_ab.py
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-skdwc4}; mkdir -p $O
for r in 1 2 3; do for v in prod skdw; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  for shp in "--B 80 --T 160" "--B 320 --T 180"; do
    echo "== $v $shp" >> $O/ab.log
    timeout -k 10 200 python -u scripts/persist_ab.py $L $shp --iters 10 >> $O/ab.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/ab.log; exit 1; }
  done
done; done
grep -E '^(==|\{)' $O/ab.log | cut -c1-200
echo done

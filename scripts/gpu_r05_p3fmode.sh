#!/bin/bash
# c3 wide forward: h_{t-1} staged by LDS-DMA (MODE 2, now on the scalar-addressed W3Dma) vs through
# registers (MODE 0, product): GPU tests on the mode-2 build first, then 3 interleaved rounds of
# scripts/persist_ab.py and one kernel trace each
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-p3fmode}; mkdir -p $O
for r in 1 2 3; do for v in prod mode2; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  echo "== $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/persist_ab.py $L --iters 5 >> $O/ab.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/ab.log; exit 1; }
done; done
grep -E '^(==|\{)' $O/ab.log | cut -c1-200
for v in prod mode2; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3_$v -o run -- python3 scripts/persist_ab.py $L --iters 3 > $O/c3_$v.log 2>&1 || { echo "$v trace rc=$?"; exit 1; }
done
echo done

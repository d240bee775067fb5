#!/bin/bash
# kernel traces of the c4-rank bf16 stack (scripts/persist_ab.py --B 80) for the product and the
# A/B builds in VARIANTS
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-dwtrace}; mkdir -p $O
for v in prod ${VARIANTS:-nodw}; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 scripts/persist_ab.py $L --B 80 --T 160 --iters 5 > $O/$v.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/$v.log; exit 1; }
  grep '^{' $O/$v.log | cut -c1-200
done
echo done

#!/bin/bash
# kernel traces of one c5 rank's GE2E (scripts/ge2e_c5rank.py) for the product library and the A/B
# builds named in VARIANTS (scripts/ab/libsv_ge2e_<v>.so)
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-ge2eprof}; mkdir -p $O
for v in prod $VARIANTS; do
  L="--lib scripts/ab/libsv_ge2e_$v.so"; [ $v = prod ] && L=""
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 scripts/ge2e_c5rank.py --iters 20 $L > $O/$v.log 2>&1 || { echo "$v rc=$?"; tail -3 $O/$v.log; exit 1; }
done
echo done

#!/bin/bash
# c3 dx GEMM: fragment-order A read from the recurrence's hand-off (product) vs row-major dG written by
# the recurrence (noafr, -DSV_BF16_AFRAG=0): c3 stack timings (scripts/persist_ab.py, 3 rounds), one
# kernel trace each, and the isolated row-major dx for reference (scripts/gemm_bench.py); VARIANTS
# picks other A/B builds (krot: -DSV_G8_KROT=5, the fragment-order A walked in a rotated K order)
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-afr}; mkdir -p $O
for r in 1 2 3; do for v in ${VARIANTS:-prod noafr}; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  echo "== bf16 $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/persist_ab.py $L --iters 5 >> $O/ab.log 2>&1 || { echo "bf16 $v rc=$?"; tail -5 $O/ab.log; exit 1; }
done; done
grep -E '^(==|\{)' $O/ab.log | cut -c1-300
for v in ${VARIANTS:-prod noafr}; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 scripts/persist_ab.py $L --iters 2 > $O/$v.log 2>&1 || { echo "$v trace rc=$?"; exit 1; }
done
timeout -k 10 200 python -u scripts/gemm_bench.py --bf16 --shapes dx --reps 6 > $O/iso.log 2>&1 || { echo "iso rc=$?"; tail -5 $O/iso.log; exit 1; }
cat $O/iso.log
echo done

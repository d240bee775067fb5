#!/bin/bash
# fp32 persistent backward helper-prefetch A/B: product vs scripts/ab/libsv_ge2e_{$VARIANTS}.so:
# f32_step_ab (persistent schedule, 3 rounds) and one FETCH_SIZE + one WRITE_SIZE pass per build
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-pf32}; mkdir -p $O
VARIANTS=${VARIANTS:-"ahead1 nopf"}
for r in 1 2 3; do
for v in prod $VARIANTS; do
  L="--lib scripts/ab/libsv_ge2e_$v.so"; [ $v = prod ] && L=""
  echo "== f32 $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/f32_step_ab.py $L --only persist --iters 3 >> $O/ab.log 2>&1 || { echo "f32 $v rc=$?"; tail -5 $O/ab.log; exit 1; }
done
done
grep -E '^(==|\{"persist)' $O/ab.log | cut -c1-300
for v in prod $VARIANTS; do
  L="--lib scripts/ab/libsv_ge2e_$v.so"; [ $v = prod ] && L=""
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${v}_$c -o p -- python3 scripts/f32_step_ab.py $L --only persist --iters 1 > $O/pmc_${v}_$c.log 2>&1 || { echo "pmc $v $c rc=$?"; tail -5 $O/pmc_${v}_$c.log; exit 1; }
  done
done
echo done

#!/bin/bash
# Parameterised A/B timing on one GPU box: the product library against A/B builds
# (`make ab NAME=x FLAGS=...` -> scripts/ab/libsv_ge2e_x.so, built in the build container and
# un-ignored for the call), interleaved over ROUNDS rounds.
#   SHAPE = c2 (fp32 stack, scripts/f32_step_ab.py --only persist) | c3 | c4 | c5 (bf16 stack,
#           scripts/persist_ab.py at 640 x T160 / 80 x T160 / 320 x T180)
#   VARIANTS = "x y ..." (A/B build names), ROUNDS (default 3), TAG (output directory under gpurun_out/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/${TAG:-ab}; mkdir -p $O
case ${SHAPE:-c3} in
  c2) CMD="scripts/f32_step_ab.py --only persist --iters 3"; PAT='^(==|\{"persist)';;
  c3) CMD="scripts/persist_ab.py --B 640 --T 160 --iters 5"; PAT='^(==|\{)';;
  c4) CMD="scripts/persist_ab.py --B 80 --T 160 --iters 5"; PAT='^(==|\{)';;
  c5) CMD="scripts/persist_ab.py --B 320 --T 180 --iters 5"; PAT='^(==|\{)';;
  *) echo "unknown SHAPE $SHAPE"; exit 2;;
esac
for r in $(seq ${ROUNDS:-3}); do
  for v in prod $VARIANTS; do
    L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
    echo "== ${SHAPE:-c3} $v" >> $O/ab.log
    timeout -k 10 200 python -u $CMD $L >> $O/ab.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/ab.log; exit 1; }
  done
done
grep -E "$PAT" $O/ab.log | cut -c1-300
echo done

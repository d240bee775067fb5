#!/bin/bash
# non-temporal C stores: fp32 GEMMs (c2 step) and the bf16 K1 / dx (c3 stack), A/B builds vs base
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-ntc}; mkdir -p $O
for r in 1 2; do
for v in base fnt; do
  echo "== f32 $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/f32_step_ab.py --lib scripts/ab/libsv_ge2e_$v.so --only persist --iters 3 >> $O/ab.log 2>&1 || { echo "f32 $v rc=$?"; tail -5 $O/ab.log; exit 1; }
done
for v in base bnt; do
  echo "== bf16 $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/persist_ab.py --lib scripts/ab/libsv_ge2e_$v.so --iters 5 >> $O/ab.log 2>&1 || { echo "bf16 $v rc=$?"; tail -5 $O/ab.log; exit 1; }
done
done
grep -E '^(==|\{)' $O/ab.log | cut -c1-400

#!/bin/bash
# A/B of the wide bf16 backward's early operand DMA (SV_P3B_EARLY_EW): timings (product vs the
# late-DMA build, alternated), phase stamps of both, then the bf16 persistent parity tests.
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-p3b}; mkdir -p $O
for r in 1 2 3; do
for v in prod p3b_late; do
  L="--lib scripts/ab/libsv_ge2e_$v.so"; [ $v = prod ] && L=""
  echo "== $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/persist_ab.py $L --iters 5 >> $O/ab.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/ab.log; exit 1; }
done
done
for v in p3b_stamp p3b_late_stamp; do
  echo "== $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/persist_ab.py --lib scripts/ab/libsv_ge2e_$v.so --iters 3 >> $O/ab.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/ab.log; exit 1; }
done
for r in 1 2; do
for v in wst wst_late; do
  echo "== $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/wave_stamps.py --lib scripts/ab/libsv_ge2e_$v.so --iters 5 >> $O/ab.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/ab.log; exit 1; }
done
done
for r in 1 2 3; do
for v in prod p3b_late; do
  L="--lib scripts/ab/libsv_ge2e_$v.so"; [ $v = prod ] && L=""
  echo "== f32 $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/f32_step_ab.py $L --only persist --iters 3 >> $O/ab.log 2>&1 || { echo "f32 $v rc=$?"; tail -5 $O/ab.log; exit 1; }
done
done
grep -E '^(==|\{)' $O/ab.log | cut -c1-600
timeout -k 10 600 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_persist.py tests/test_gpu_model.py -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log

#!/bin/bash
# the 16-row wide-tile bf16 backward (c5 rank, 320 rows) vs the 32 x 32 tile (no16 = -DSV_PBWD16=0):
# its GPU tests, then c5-rank stack timings (scripts/persist_ab.py --B 320 --T 180, 3 rounds) and traces
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-p16}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_persist.py tests/test_gpu_precision.py > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|Error|assert" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
grep MEASURED $O/pytest.log | grep -E "persist16|c5_rank" | head; tail -1 $O/pytest.log
for r in 1 2 3; do for v in prod ${VARIANTS:-no16}; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  echo "== $v" >> $O/ab.log
  timeout -k 10 120 python -u scripts/persist_ab.py $L --B 320 --T 180 --iters 5 >> $O/ab.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/ab.log; exit 1; }
done; done
grep -E '^(==|\{)' $O/ab.log | cut -c1-200
for v in prod ${VARIANTS:-no16}; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 scripts/persist_ab.py $L --B 320 --T 180 --iters 5 > $O/$v.log 2>&1 || { echo "$v trace rc=$?"; tail -5 $O/$v.log; exit 1; }
done
echo done

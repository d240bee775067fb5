#!/bin/bash
# c3 wide backward: the dG^T stores under the hand-off drain (SV_P3B_OVL=1, prod) vs after the arrival
# (head = previous tree): GPU tests, then 4 interleaved rounds of scripts/persist_ab.py at c3 and one
# kernel trace each
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-p3ovl}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_persist.py tests/test_gpu_precision.py tests/test_gpu_model.py > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|Error|assert" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3 4; do for v in prod head; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  echo "== $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/persist_ab.py $L --iters 5 >> $O/ab.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/ab.log; exit 1; }
done; done
for v in prod head; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3_$v -o run -- python3 scripts/persist_ab.py $L --iters 3 > $O/c3_$v.log 2>&1 || { echo "$v trace rc=$?"; exit 1; }
done
echo done

#!/bin/bash
# bf16 wide / wavefront backward with the packed-fp32 cell (product) vs the scalar cell (scalarcell)
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-pkcell}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_precision.py -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
for v in prod scalarcell; do
  L="--lib scripts/ab/libsv_ge2e_$v.so"; [ $v = prod ] && L=""
  echo "== bf16 $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/persist_ab.py $L --iters 5 >> $O/ab.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/ab.log; exit 1; }
done
done
grep -E '^(==|\{)' $O/ab.log | cut -c1-200

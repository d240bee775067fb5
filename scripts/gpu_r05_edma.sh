#!/bin/bash
# fp32 persistent backward: the next half-step's operand DMA inside the k-loop (product: 12 k-groups
# before its end, two operand image sets) vs the r04 placement (edma0) / 24 k-groups (edma24):
# c2 step timings (scripts/f32_step_ab.py, 3 rounds), c2 GPU parity tests
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-edma}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_model.py tests/test_gpu_persist.py > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|Error" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do for v in prod ${VARIANTS:-edma0 edma24}; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  echo "== f32 $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/f32_step_ab.py $L --only persist --iters 3 >> $O/ab.log 2>&1 || { echo "f32 $v rc=$?"; tail -5 $O/ab.log; exit 1; }
done; done
grep -E '^(==|\{"persist)' $O/ab.log | cut -c1-300
echo done

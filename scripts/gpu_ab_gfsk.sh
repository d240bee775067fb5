#!/bin/bash
# fp32 dx GEMM stream-K form (product) vs the one-shot kernel (nosk)
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-gfsk}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_persist.py tests/test_dvector.py tests/test_gpu_dropin_cpu.py -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
for v in prod nosk; do
  L="--lib scripts/ab/libsv_ge2e_$v.so"; [ $v = prod ] && L=""
  echo "== f32 $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/f32_step_ab.py $L --only persist --iters 3 >> $O/ab.log 2>&1 || { echo "f32 $v rc=$?"; tail -5 $O/ab.log; exit 1; }
done
done
grep -E '^(==|\{"persist)' $O/ab.log | cut -c1-300

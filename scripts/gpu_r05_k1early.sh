#!/bin/bash
# fp32 persistent K1 (gemm_f32_256p_kernel): the next tile's k-tile 1 DMA'd before the C stores and
# k-tile 0's wait counting them (product, SV_GF_EARLY=1) vs the old drain (early0) vs a no-store
# diagnostic (nostore, results invalid): GEMM tests, then c2 step timings (scripts/f32_step_ab.py,
# 3 rounds) and one kernel trace each
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-k1early}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_model.py > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|Error|assert" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
grep MEASURED $O/pytest.log | grep -E "c2" | head; tail -1 $O/pytest.log
for r in 1 2 3; do for v in prod early0 nostore; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  echo "== f32 $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/f32_step_ab.py $L --only persist --iters 3 >> $O/ab.log 2>&1 || { echo "f32 $v rc=$?"; tail -5 $O/ab.log; exit 1; }
done; done
grep -E '^(==|\{"persist)' $O/ab.log | cut -c1-200
for v in prod early0 nostore; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 scripts/f32_step_ab.py $L --only persist --iters 1 > $O/$v.log 2>&1 || { echo "$v trace rc=$?"; exit 1; }
done
echo done

#!/bin/bash
# fragment-order A without runtime divisions (fp32 dx and bf16 dx) vs the previous tree (head):
# GPU tests, c2 and c3 step A/B (3 rounds each) and one kernel trace per build and config
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-afdiv2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_persist.py tests/test_gpu_precision.py tests/test_gpu_model.py > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|Error|assert" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do for v in prod head; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  echo "== f32 $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/f32_step_ab.py $L --only persist --iters 3 >> $O/ab.log 2>&1 || { echo "f32 $v rc=$?"; tail -5 $O/ab.log; exit 1; }
  echo "== bf16 $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/persist_ab.py $L --iters 5 >> $O/ab.log 2>&1 || { echo "bf16 $v rc=$?"; tail -5 $O/ab.log; exit 1; }
done; done
grep -E '^(==|\{)' $O/ab.log | cut -c1-220
for v in prod head; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/f32_$v -o run -- python3 scripts/f32_step_ab.py $L --only persist --iters 1 > $O/f32_$v.log 2>&1 || { echo "$v trace rc=$?"; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bf16_$v -o run -- python3 scripts/persist_ab.py $L --iters 2 > $O/bf16_$v.log 2>&1 || { echo "$v trace rc=$?"; exit 1; }
done
echo done

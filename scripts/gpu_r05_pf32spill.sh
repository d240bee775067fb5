#!/bin/bash
# fp32 persistent backward without the hoisted per-row bias predicates (136 -> 24 SGPRs spilled to
# VGPR lanes) vs the previous tree (head): fp32 GPU tests, c2 step A/B (4 interleaved rounds), one
# kernel trace each
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-pf32spill}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_persist.py tests/test_gpu_model.py > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|Error|assert" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3 4; do for v in prod head; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  echo "== f32 $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/f32_step_ab.py $L --only persist --iters 3 >> $O/ab.log 2>&1 || { echo "f32 $v rc=$?"; tail -5 $O/ab.log; exit 1; }
done; done
grep -E '^(==|\{"persist)' $O/ab.log | cut -c1-200
for v in prod head; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/f32_$v -o run -- python3 scripts/f32_step_ab.py $L --only persist --iters 1 > $O/f32_$v.log 2>&1 || { echo "$v trace rc=$?"; exit 1; }
done
echo done

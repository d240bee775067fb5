#!/bin/bash
# the c4 wavefront backward's and the c5 rank's (32 x 32 tiles) dG^T stores under the hand-off drain
# (prod) vs after the arrival (head = previous tree): GPU tests, then 3 interleaved rounds of
# scripts/persist_ab.py at the c4 / c5 rank shapes and one kernel trace each
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-ovl45}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_persist.py tests/test_gpu_precision.py tests/test_gpu_model.py tests/test_gpu_sharded.py > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|Error|assert" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do for v in prod head; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  for shp in "--B 80 --T 160" "--B 320 --T 180"; do
    echo "== $v $shp" >> $O/ab.log
    timeout -k 10 200 python -u scripts/persist_ab.py $L $shp --iters 10 >> $O/ab.log 2>&1 || { echo "$v $shp rc=$?"; tail -5 $O/ab.log; exit 1; }
  done
done; done
for v in prod head; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4_$v -o run -- python3 scripts/persist_ab.py $L --B 80 --T 160 --iters 3 > $O/c4_$v.log 2>&1 || { echo "$v trace rc=$?"; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5_$v -o run -- python3 scripts/persist_ab.py $L --B 320 --T 180 --iters 3 > $O/c5_$v.log 2>&1 || { echo "$v trace rc=$?"; exit 1; }
done
echo done

#!/bin/bash
# wavefront forward with the next x tile's DMA in the h-part (product) vs the off-chain placement
# (wst_late), stamp builds; bf16 persistent / precision tests on the product; hipBLASLt kernel names
# for the c3 dx / K1 shapes.
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-w3x}; mkdir -p $O
for r in 1 2 3; do
for v in wst wst_late; do
  echo "== $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/wave_stamps.py --lib scripts/ab/libsv_ge2e_$v.so --iters 5 >> $O/ab.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/ab.log; exit 1; }
done
done
grep -E '^(==|\{)' $O/ab.log | cut -c1-300
timeout -k 10 600 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_persist.py -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_gemm -o run -- python3 scripts/gemm_bench.py --bf16 --torch --reps 3 --shapes Gx,dx > $O/prof_gemm.log 2>&1 || { echo "prof rc=$?"; tail -5 $O/prof_gemm.log; exit 1; }
find $O/prof_gemm -name "*kernel_stats.csv" | head -1 | xargs cut -c1-200

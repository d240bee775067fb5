#!/bin/bash
# the c4 wavefront's weight gradients as whole-K tiles of all layers in one launch (prod,
# gemm_bf16_8qf_kernel) vs the per-layer split-K slabs + reduce (head = previous tree): GPU tests,
# then 3 interleaved rounds of scripts/persist_ab.py at the c4 rank shape and one kernel trace each
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-fullk}; mkdir -p $O
[ -n "$SKIPTEST" ] || timeout -k 10 600 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_persist.py tests/test_gpu_precision.py tests/test_gpu_model.py > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|Error|assert" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
[ -n "$SKIPTEST" ] || tail -1 $O/pytest.log
for r in 1 2 3; do for v in ${VARIANTS:-prod head}; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  echo "== $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/persist_ab.py $L --B 80 --T 160 --iters 10 >> $O/ab.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/ab.log; exit 1; }
done; done
for v in ${VARIANTS:-prod head}; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4_$v -o run -- python3 scripts/persist_ab.py $L --B 80 --T 160 --iters 3 > $O/c4_$v.log 2>&1 || { echo "$v trace rc=$?"; exit 1; }
done
grep -E '^(==|\{)' $O/ab.log | cut -c1-200
echo done

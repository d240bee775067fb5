#!/bin/bash
# layer-wavefront forward (c4 rank) with the x / h tile DMA addresses in scalar arithmetic (prod) vs the
# previous tree (head): GPU tests of the persistent / wavefront paths, c4-rank stack A/B (4 interleaved
# rounds of scripts/persist_ab.py --B 80 --T 160) and one kernel trace each
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-w3dma}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_persist.py tests/test_gpu_precision.py > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|Error|assert" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3 4; do for v in prod head; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  echo "== c4 $v" >> $O/ab.log
  timeout -k 10 200 python -u scripts/persist_ab.py $L --B 80 --T 160 --iters 10 >> $O/ab.log 2>&1 || { echo "c4 $v rc=$?"; tail -5 $O/ab.log; exit 1; }
done; done
grep -E '^(==|\{)' $O/ab.log | cut -c1-200
for v in prod head; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4_$v -o run -- python3 scripts/persist_ab.py $L --B 80 --T 160 --iters 3 > $O/c4_$v.log 2>&1 || { echo "$v trace rc=$?"; exit 1; }
done
echo done

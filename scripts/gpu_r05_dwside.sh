#!/bin/bash
# r05: the wavefront's weight gradients beside it (gemm_bf16_8qw_kernel) vs after it (A/B build
# nodw = -DSV_WAVE_DW_SIDE=0): bit identity at the c4 rank shape, stack timings, a c4 bench trace,
# then the GPU tests that run the layer wavefront
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-dwside}; mkdir -p $O
timeout -k 10 120 python -u scripts/bitident_ab.py --out $O/prod.pt > $O/bit_prod.log 2>&1 || { echo "bit prod rc=$?"; tail -5 $O/bit_prod.log; exit 1; }
timeout -k 10 120 python -u scripts/bitident_ab.py --lib scripts/ab/libsv_ge2e_nodw.so --out $O/nodw.pt > $O/bit_nodw.log 2>&1 || { echo "bit nodw rc=$?"; tail -5 $O/bit_nodw.log; exit 1; }
python scripts/bitident_ab.py --compare $O/prod.pt $O/nodw.pt; echo "compare rc=$?"
for r in 1 2 3; do for v in prod nodw; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  echo "== $v" >> $O/ab.log
  timeout -k 10 120 python -u scripts/persist_ab.py $L --B 80 --T 160 --iters 5 >> $O/ab.log 2>&1 || { echo "$v rc=$?"; tail -5 $O/ab.log; exit 1; }
done; done
grep -E '^(==|\{)' $O/ab.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o run -- python3 bench.py --preset c4 --steps 5 --warmup 2 --no-cpu-baseline --no-vendor --no-extras --fwd-steps 1 > $O/c4.log 2>&1 || { echo "c4 trace rc=$?"; tail -5 $O/c4.log; exit 1; }
grep '^{' $O/c4.log | cut -c1-200
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_precision.py tests/test_gpu_persist.py > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|Error" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
echo done

#!/bin/bash
# fp32 persistent recurrences: their GPU tests, then A/B timing of the fp32 step (persistent vs
# per-step; and the A/B builds under scripts/ab/ named in $ABLIBS) and GEMM timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
T=${TAG:-f32p}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py -x -v -s --timeout 200 --timeout-method thread -k "${TESTK:-c1_matches or c2_against or f32_persistent}" > gpurun_out/pt_$T.log 2>&1
  rc=$?
  grep -E "MEASURED|PASSED|FAILED|Error|error" gpurun_out/pt_$T.log | head -40
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python scripts/f32_step_ab.py > gpurun_out/ab_$T.log 2>&1 || { echo "ab rc=$?"; tail -5 gpurun_out/ab_$T.log; exit 1; }
tail -1 gpurun_out/ab_$T.log
for L in $ABLIBS; do
  timeout -k 10 300 python scripts/f32_step_ab.py --lib scripts/ab/libsv_ge2e_$L.so --only auto > gpurun_out/ab_${T}_$L.log 2>&1 || { echo "ab $L rc=$?"; tail -5 gpurun_out/ab_${T}_$L.log; exit 1; }
  tail -1 gpurun_out/ab_${T}_$L.log
done
timeout -k 10 200 python scripts/gemm_bench.py --bf16 --check --reps 10 > gpurun_out/gemm_$T.log 2>&1 || { echo "gemm rc=$?"; exit 1; }
tail -1 gpurun_out/gemm_$T.log

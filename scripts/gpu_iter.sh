#!/bin/bash
# One iteration on the GPU box: GEMM timings (product build, and the 16x16x4 A/B build when
# present), the bf16 / DP parity tests, then a short bench.  Stops at the first crash.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
T=${TAG:-it}
timeout -k 10 200 python scripts/gemm_bench.py --bf16 --torch --check --reps 10 > gpurun_out/gemm_$T.log 2>&1 || { echo "gemm rc=$?"; tail -5 gpurun_out/gemm_$T.log; exit 1; }
tail -1 gpurun_out/gemm_$T.log
if [ -f scripts/ab/libsv_ge2e_m16.so ]; then
  timeout -k 10 200 python scripts/gemm_bench.py --reps 10 --lib scripts/ab/libsv_ge2e_m16.so > gpurun_out/gemm_m16_$T.log 2>&1 || { echo "m16 rc=$?"; exit 1; }
  tail -1 gpurun_out/gemm_m16_$T.log
fi
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_persist.py tests/test_gpu_precision.py tests/test_gpu_dp.py} -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_$T.log 2>&1
rc=$?
tail -3 gpurun_out/pt_$T.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$T.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/bench_$T.log; exit 1; }
grep "ms/step" gpurun_out/bench_$T.log

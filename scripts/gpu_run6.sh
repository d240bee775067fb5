#!/bin/bash
# A/B of the fp32 c2 stack (product vs an A/B build, alternated twice), then the fp32 model tests
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1; mkdir -p gpurun_out
T=${TAG:-ab}; AB=${AB:-dws0}
for i in 1 2; do
  timeout -k 10 200 python scripts/f32_step_ab.py --only auto --iters 5 > gpurun_out/f32ab_prod_${T}_$i.log 2>&1 || { echo "prod failed"; tail -3 gpurun_out/f32ab_prod_${T}_$i.log; exit 1; }
  echo "prod $(tail -n 1 gpurun_out/f32ab_prod_${T}_$i.log)"
  timeout -k 10 200 python scripts/f32_step_ab.py --only auto --iters 5 --lib scripts/ab/libsv_ge2e_$AB.so > gpurun_out/f32ab_${AB}_${T}_$i.log 2>&1 || { echo "ab failed"; exit 1; }
  echo "$AB $(tail -n 1 gpurun_out/f32ab_${AB}_${T}_$i.log)"
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_dp.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_$T.log 2>&1
rc=$?; tail -2 gpurun_out/pt_$T.log; exit $rc

#!/bin/bash
# A/B bench runs over env settings: AB_ENVS="VAR=a VAR=b,VAR2=c ..." (one short bench per
# setting; commas join several variables into one setting).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for kv in ${AB_ENVS}; do
  env ${kv//,/ } timeout -k 10 300 python bench.py --steps ${AB_STEPS:-5} --warmup 2 --no-cpu-baseline ${AB_ARGS} > gpurun_out/ab_$kv.log 2>&1 || { echo "ab $kv failed"; tail -5 gpurun_out/ab_$kv.log; exit 1; }
  echo "$kv $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$kv.log | head -1) $(grep -o '"bf16": {[^}]*' gpurun_out/ab_$kv.log | grep -o '"ms_per_step": [0-9.]*')"
done

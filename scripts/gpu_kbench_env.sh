#!/bin/bash
# kbench over env settings: KB_ENVS="VAR=a VAR=b,VAR2=c" (commas join variables).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for kv in ${KB_ENVS}; do
  env ${kv//,/ } timeout -k 10 300 python scripts/kbench.py > gpurun_out/kb_$kv.log 2>&1 || { echo "kb $kv failed"; tail -5 gpurun_out/kb_$kv.log; exit 1; }
  echo "$kv $(grep '^{"variant' gpurun_out/kb_$kv.log | cut -c1-200)"
done

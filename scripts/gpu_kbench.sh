#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-1 2}; do
  SV_STEP_VARIANT=$v timeout -k 10 300 python scripts/kbench.py >> gpurun_out/kbench.log 2>&1 || exit $?
done
tail -n 4 gpurun_out/kbench.log

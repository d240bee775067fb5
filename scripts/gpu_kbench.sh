#!/bin/bash
# standalone step-kernel / GEMM timings (scripts/kbench.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/kbench.py >> gpurun_out/kbench.log 2>&1 || exit $?
tail -n 4 gpurun_out/kbench.log

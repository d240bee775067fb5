#!/bin/bash
# Persistent bf16 backward: parity tests, then c3 A/B over schedules and prefetch depths.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_persist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pbwd_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pbwd_pytest.log; exit 1; }
tail -2 gpurun_out/pbwd_pytest.log
AB_ENVS="${PB_ENVS:-SV_PERSIST_BWD=0 SV_PERSIST_BWD=1 SV_PERSIST_BWD=1,SV_PBWD_DW_SIDE=0 SV_PERSIST_BWD=1,SV_PBWD_P=4 SV_PERSIST_BWD=1,SV_PBWD_P=16}" \
AB_ARGS="--dtype bf16 --no-vendor --no-f32x --fwd-steps 1" bash scripts/gpu_ab.sh

#!/bin/bash
# iteration: d-vector GEMM path tests + timing
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1; mkdir -p gpurun_out
T=${TAG:-d1}
timeout -k 10 400 python -u -m pytest tests/test_dvector.py -x -v --timeout 300 --timeout-method thread -s > gpurun_out/pt_$T.log 2>&1
rc=$?; grep -E "MEASURED|passed|failed|Error|error" gpurun_out/pt_$T.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/dvec_bench.py > gpurun_out/dvec_$T.log 2>&1; rc=$?; tail -5 gpurun_out/dvec_$T.log; exit $rc

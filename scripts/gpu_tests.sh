#!/bin/bash
# pytest -m gpu (verbose, with MEASURED tolerance lines) into gpurun_out/pytest_gpu.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 ${PYTEST_TIMEOUT:-1000} python -u -m pytest ${TESTS:-tests} -m gpu -x -v -s --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "MEASURED|PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -120
tail -5 gpurun_out/pytest_gpu.log
exit $rc

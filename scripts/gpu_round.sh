#!/bin/bash
# One GPU call: pytest -m gpu, then (if no crash) a short bench.  Stops at the first
# fault/abort/timeout (exit codes other than 0/1 from pytest).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
if [ -n "$SKIP_BENCH" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:---steps 5 --warmup 2} > gpurun_out/bench.log 2>&1
brc=$?
echo "bench rc=$brc"
tail -5 gpurun_out/bench.log
exit $brc

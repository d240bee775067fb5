#!/bin/bash
# r05 checkpoint: pytest -m gpu (verbose, MEASURED lines), then the default bench line.
# Usage: TAG=r501 [BENCH_ARGS=...] bash scripts/gpu_ckpt_r05.sh ; stops at the first failure.
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-r501}; mkdir -p $O
if [ -z "$NO_TESTS" ]; then
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v -s -rA --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
fi
timeout -k 10 900 python -u bench.py $BENCH_ARGS > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-400
echo done

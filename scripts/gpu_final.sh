#!/bin/bash
# the round-end tiers as the driver runs them: pytest -m gpu, smoke(), bench.py (defaults)
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/final/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/final/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/final/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/final/bench.log; exit 1; }
grep '^{' gpurun_out/final/bench.log | cut -c1-400

#!/bin/bash
# checkpoint part A: pytest -m gpu and the default bench line
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; mkdir -p gpurun_out/ckpt
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/ckpt/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/ckpt/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/ckpt/pytest_gpu.log
timeout -k 10 600 python bench.py > gpurun_out/ckpt/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/ckpt/bench.log; exit 1; }
grep '^{' gpurun_out/ckpt/bench.log | cut -c1-300

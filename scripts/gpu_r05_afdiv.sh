#!/bin/bash
# c3 dx GEMM on the fragment-order A after the per-fill runtime division left its k-loop (product)
# vs row-major dG (noafr): GPU tests of the bf16 paths first, then scripts/gpu_r05_afr.sh's A/B
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-afdiv}; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_persist.py tests/test_gpu_precision.py tests/test_gpu_model.py > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; grep -E "FAILED|Error|assert" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
TAG=${TAG:-afdiv} bash scripts/gpu_r05_afr.sh

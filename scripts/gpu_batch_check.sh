#!/bin/bash
# bf16 path after batching its per-step casts / zeroings: parity tests, then the c4 rank timeline
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-batch}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_persist.py tests/test_dvector.py tests/test_gpu_dp.py tests/test_gpu_model.py -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
TAG=${TAG:-batch}/c4 bash scripts/gpu_prof_c4.sh

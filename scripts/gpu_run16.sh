#!/bin/bash
# bf16 row chunks incl. the wavefront halves: precision + model + DP tests, then the per-rank shapes
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1; mkdir -p gpurun_out/r16
timeout -k 10 600 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_model.py tests/test_gpu_dp.py tests/test_gpu_status.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r16/pt.log 2>&1 || { echo "tests rc=$?"; grep -E "MEASURED|Error|error|FAIL" gpurun_out/r16/pt.log | tail -30; exit 1; }
grep -E "MEASURED c4_4rank|MEASURED c5_2rank|passed|failed" gpurun_out/r16/pt.log
timeout -k 10 400 python -u scripts/rank_shapes.py --steps 5 --warmup 2 > gpurun_out/r16/rank_shapes.log 2>&1 || { echo "rank shapes rc=$?"; tail -30 gpurun_out/r16/rank_shapes.log; exit 1; }
grep '^{' gpurun_out/r16/rank_shapes.log

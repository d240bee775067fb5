#!/bin/bash
# Round checkpoint on one GPU box: pytest -m gpu, the full bench line, then rocprofv3
# kernel-trace summaries of the fp32 (c2) and bf16 (c3) steps.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ckpt
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/ckpt/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/ckpt/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/ckpt/pytest_gpu.log
fi
timeout -k 10 600 python bench.py > gpurun_out/ckpt/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/ckpt/bench.log; exit 1; }
grep '^{' gpurun_out/ckpt/bench.log | cut -c1-400
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ckpt/prof_f32 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-vendor --no-bf16 --fwd-steps 1 > gpurun_out/ckpt/prof_f32.log 2>&1 || { echo "prof f32 failed"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ckpt/prof_bf16 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-vendor --no-extras --dtype bf16 --fwd-steps 1 > gpurun_out/ckpt/prof_bf16.log 2>&1 || { echo "prof bf16 failed"; exit 1; }
echo done

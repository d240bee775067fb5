#!/bin/bash
# Round checkpoint on one GPU box: pytest -m gpu (verbose, MEASURED lines kept), the full bench
# line, then rocprofv3 kernel-trace summaries of the fp32 (c2) and bf16 (c3) steps.  Stops at the
# first failure.  TAG names the output directory; SKIP_TESTS / SKIP_PROF skip those parts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ckpt}; mkdir -p $O
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1500 python -u -m pytest tests -m gpu -v -s -rA --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
timeout -k 10 900 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-600
if [ -z "$SKIP_PROF" ]; then
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_f32 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-vendor --no-bf16 --no-f32x --no-extras --fwd-steps 1 > $O/prof_f32.log 2>&1 || { echo "prof f32 failed"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bf16 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-vendor --no-extras --dtype bf16 --fwd-steps 1 > $O/prof_bf16.log 2>&1 || { echo "prof bf16 failed"; exit 1; }
fi
echo done

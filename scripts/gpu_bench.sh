#!/bin/bash
# The default bench line (as the driver runs it), then rocprofv3 kernel-trace summaries of the
# fp32 (c2) and bf16 (c3) steps.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ckpt
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/ckpt/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/ckpt/bench.log; exit 1; }
grep '^{' gpurun_out/ckpt/bench.log | cut -c1-600
[ -n "$NO_PROF" ] && exit 0
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ckpt/prof_f32 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-vendor --no-bf16 --no-f32x --fwd-steps 1 > gpurun_out/ckpt/prof_f32.log 2>&1 || { echo "prof f32 failed"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ckpt/prof_bf16 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-vendor --preset c3 --fwd-steps 1 > gpurun_out/ckpt/prof_bf16.log 2>&1 || { echo "prof bf16 failed"; exit 1; }
echo done

#!/bin/bash
# checkpoint part B: rocprofv3 kernel-trace summaries of the fp32 (c2) and bf16 (c3) steps
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; mkdir -p gpurun_out/ckpt
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ckpt/prof_f32 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-vendor --no-bf16 --fwd-steps 1 > gpurun_out/ckpt/prof_f32.log 2>&1 || { echo "prof f32 failed"; tail -5 gpurun_out/ckpt/prof_f32.log; exit 1; }
grep '^{' gpurun_out/ckpt/prof_f32.log | cut -c1-200
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ckpt/prof_bf16 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-vendor --no-extras --dtype bf16 --fwd-steps 1 > gpurun_out/ckpt/prof_bf16.log 2>&1 || { echo "prof bf16 failed"; tail -5 gpurun_out/ckpt/prof_bf16.log; exit 1; }
grep '^{' gpurun_out/ckpt/prof_bf16.log | cut -c1-200
echo done

#!/bin/bash
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1; mkdir -p gpurun_out/r22
timeout -k 10 200 python scripts/f32_bwd_dump.py gpurun_out/r22/p1.pt > gpurun_out/r22/dump.log 2>&1 || { echo "dump failed"; tail -20 gpurun_out/r22/dump.log; exit 1; }
timeout -k 10 200 python scripts/f32_bwd_dump.py --lib scripts/ab/libsv_ge2e_base.so gpurun_out/r22/b1.pt >> gpurun_out/r22/dump.log 2>&1 || { echo "dump failed"; tail -20 gpurun_out/r22/dump.log; exit 1; }
echo "prod vs base $(python scripts/f32_bwd_dump.py --compare gpurun_out/r22/p1.pt gpurun_out/r22/b1.pt)"
rm -f gpurun_out/r22/*.pt

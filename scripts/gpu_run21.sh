#!/bin/bash
# run-to-run determinism of the c2 fp32 backward (base twice, prod twice) and prod vs base
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1; mkdir -p gpurun_out/r21
for n in 1 2; do
  timeout -k 10 200 python scripts/f32_bwd_dump.py gpurun_out/r21/p$n.pt > gpurun_out/r21/dump.log 2>&1 || { echo "dump failed"; tail -20 gpurun_out/r21/dump.log; exit 1; }
  timeout -k 10 200 python scripts/f32_bwd_dump.py --lib scripts/ab/libsv_ge2e_base.so gpurun_out/r21/b$n.pt >> gpurun_out/r21/dump.log 2>&1 || { echo "dump failed"; tail -20 gpurun_out/r21/dump.log; exit 1; }
done
echo "prod vs prod $(python scripts/f32_bwd_dump.py --compare gpurun_out/r21/p1.pt gpurun_out/r21/p2.pt)"
echo "base vs base $(python scripts/f32_bwd_dump.py --compare gpurun_out/r21/b1.pt gpurun_out/r21/b2.pt)"
echo "prod vs base $(python scripts/f32_bwd_dump.py --compare gpurun_out/r21/p1.pt gpurun_out/r21/b1.pt)"
rm -f gpurun_out/r21/*.pt

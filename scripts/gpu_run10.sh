#!/bin/bash
# phase stamps of the fp32 persistent forward (c2)
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1; mkdir -p gpurun_out/r11
timeout -k 10 200 python scripts/f32_step_ab.py --only auto --iters 3 --stamps --lib scripts/ab/libsv_ge2e_pfst.so > gpurun_out/r11/pfst.log 2>&1 || { echo "failed"; tail -5 gpurun_out/r11/pfst.log; exit 1; }
tail -n 1 gpurun_out/r11/pfst.log

#!/bin/bash
# the wavefront's weight gradients as one queue launch after it (product build) vs per layer
# (perlayer = -DSV_WAVE_DW_QUEUE=0): bit identity, then scripts/gpu_r05_dwab.sh's timings + traces
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-dwq}; mkdir -p $O
timeout -k 10 120 python -u scripts/bitident_ab.py --out /tmp/prod.pt > $O/bit_prod.log 2>&1 || { echo "bit prod rc=$?"; tail -5 $O/bit_prod.log; exit 1; }
timeout -k 10 120 python -u scripts/bitident_ab.py --lib scripts/ab/libsv_ge2e_perlayer.so --out /tmp/pl.pt > $O/bit_pl.log 2>&1 || { echo "bit pl rc=$?"; tail -5 $O/bit_pl.log; exit 1; }
python scripts/bitident_ab.py --compare /tmp/prod.pt /tmp/pl.pt; echo "compare rc=$?"
TAG=${TAG:-dwq} VARIANTS=perlayer bash scripts/gpu_r05_dwab.sh

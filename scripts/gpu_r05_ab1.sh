#!/bin/bash
# r05 A/B: GE2E cols kernel (prod vs kb2) traces, then the fp32 backward helper prefetch (prod =
# per-half triggers vs nosplit vs nopf): step times and HBM traffic
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
TAG=ab1_ge2e VARIANTS=kb2 bash scripts/gpu_ge2e_prof.sh || exit 1
TAG=ab1_pf32 VARIANTS="nosplit nopf" bash scripts/gpu_ab_pf32.sh || exit 1

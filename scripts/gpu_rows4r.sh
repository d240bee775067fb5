#!/bin/bash
# GE2E rows kernel A/B: parity tests of the product library, then c5-rank traces (prod vs rows16)
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-rows4r}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  ${TESTS:-tests/test_gpu_sharded.py tests/test_gpu_kernels.py tests/test_gpu_dropin_launcher.py} > $O/pytest.log 2>&1 \
  || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
VARIANTS="${VARIANTS:-rows16}" TAG=${TAG:-rows4r} bash scripts/gpu_ge2e_prof.sh

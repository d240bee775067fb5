#!/bin/bash
# r05 checkpoint: scripts/gpu_checkpoint.sh (pytest -m gpu, bench line, rocprofv3 c2 / c3 traces),
# then the HBM-traffic PMC passes (scripts/gpu_pmc_traffic.sh) the bench's roofline.traffic reads
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r503} bash scripts/gpu_checkpoint.sh || exit 1
bash scripts/gpu_pmc_traffic.sh || exit 1
echo ckpt-done

#!/bin/bash
# bf16 GEMM rates at the c3 shapes (random vs zero operands)
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-gemm_rate}; mkdir -p $O
timeout -k 10 300 python -u scripts/gemm_bench.py --bf16 --torch --reps 6 > $O/rand.log 2>&1 || { echo "rand rc=$?"; tail -5 $O/rand.log; exit 1; }
timeout -k 10 300 python -u scripts/gemm_bench.py --bf16 --reps 6 --fill zeros > $O/zeros.log 2>&1 || { echo "zeros rc=$?"; tail -5 $O/zeros.log; exit 1; }
cat $O/rand.log $O/zeros.log | grep '^{'

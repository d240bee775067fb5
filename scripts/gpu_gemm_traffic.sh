#!/bin/bash
# HBM-traffic PMC passes over scripts/gemm_traffic.py (isolated GEMM launches at the c2/c3 shapes):
# FETCH_SIZE and WRITE_SIZE each in its own rocprofv3 run, nothing traced beside them.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/gemm_traffic
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o p -- python3 scripts/gemm_traffic.py > $D/fetch.log 2>&1 || { echo "fetch rc=$?"; tail -5 $D/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o p -- python3 scripts/gemm_traffic.py > $D/write.log 2>&1 || { echo "write rc=$?"; tail -5 $D/write.log; exit 1; }
for L in $ABLIBS; do  # A/B builds: their fetch pass only (WRITE_SIZE is layout-independent)
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/ab_$L -o p -- python3 scripts/gemm_traffic.py --lib scripts/ab/libsv_ge2e_$L.so > $D/ab_$L.log 2>&1 || { echo "$L rc=$?"; exit 1; }
done
find $D -name "*.csv" | head

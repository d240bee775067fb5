#!/bin/bash
# r05: the bf16 stream-K GEMM forms (A/B builds sk = -DSV_G8_SK=1: dx, skdw = -DSV_G8_SK_DW=1: weight
# gradients) against the product: kernel traces of the bf16 stack (scripts/persist_ab.py) at c3
# (B 640, T 160) and the c4 rank (B 80, T 160)
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-r05sk}; mkdir -p $O
for v in prod ${VARIANTS:-sk skdw}; do
  L=""; [ $v != prod ] && L="--lib scripts/ab/libsv_ge2e_$v.so"
  for B in 640 80; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_$B -o run -- python3 scripts/persist_ab.py $L --B $B --T 160 --iters 5 > $O/${v}_$B.log 2>&1 || { echo "$v $B rc=$?"; tail -5 $O/${v}_$B.log; exit 1; }
    grep '^{' $O/${v}_$B.log | cut -c1-250
  done
done
echo done

#!/bin/bash
# HBM-traffic PMC passes over short bench runs (fp32 c2 and bf16 c3 steps) and the c4 / c5 rank
# shapes' bf16 stacks: FETCH_SIZE and WRITE_SIZE each in its own rocprofv3 run (no tracing
# combined with --pmc).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/pmc_traffic
mkdir -p $D
export TMPDIR=/tmp
ARGS_F32="--steps 2 --warmup 1 --no-cpu-baseline --no-vendor --no-bf16 --no-f32x --no-extras --fwd-steps 1"
ARGS_BF16="--steps 2 --warmup 1 --no-cpu-baseline --no-vendor --no-extras --preset c3 --fwd-steps 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/f32_fetch -o p -- python3 bench.py $ARGS_F32 > $D/f32_fetch.log 2>&1 || { echo "f32 fetch rc=$?"; tail -5 $D/f32_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/f32_write -o p -- python3 bench.py $ARGS_F32 > $D/f32_write.log 2>&1 || { echo "f32 write rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/bf16_fetch -o p -- python3 bench.py $ARGS_BF16 > $D/bf16_fetch.log 2>&1 || { echo "bf16 fetch rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/bf16_write -o p -- python3 bench.py $ARGS_BF16 > $D/bf16_write.log 2>&1 || { echo "bf16 write rc=$?"; exit 1; }
# the rank shapes' bf16 stacks (c4: the layer wavefronts; c5: the 32 x 32 persistent tiles)
for r in "c4 80 160" "c5 320 180"; do set -- $r
  for c in FETCH_SIZE WRITE_SIZE; do n=$([ $c = FETCH_SIZE ] && echo fetch || echo write)
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $D/${1}_$n -o p -- python3 scripts/persist_ab.py --B $2 --T $3 --iters 2 > $D/${1}_$n.log 2>&1 || { echo "$1 $n rc=$?"; exit 1; }
  done
done
find $D -name "*.csv" | head

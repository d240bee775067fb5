#!/bin/bash
# r04 checkpoint: pytest -m gpu (verbose, MEASURED lines),
# the full bench line, rocprofv3 kernel-trace summaries (fp32 c2, bf16 c3) and the HBM-traffic PMC
# passes.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-r412}; mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -s -rA --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 900 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_f32 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-vendor --no-bf16 --no-f32x --no-extras --fwd-steps 1 > $O/prof_f32.log 2>&1 || { echo "prof f32 failed"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bf16 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-vendor --no-extras --dtype bf16 --fwd-steps 1 > $O/prof_bf16.log 2>&1 || { echo "prof bf16 failed"; exit 1; }
D=$O/pmc_traffic; mkdir -p $D
ARGS_F32="--steps 2 --warmup 1 --no-cpu-baseline --no-vendor --no-bf16 --no-f32x --no-extras --fwd-steps 1"
ARGS_BF16="--steps 2 --warmup 1 --no-cpu-baseline --no-vendor --no-extras --preset c3 --fwd-steps 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/f32_fetch -o p -- python3 bench.py $ARGS_F32 > $D/f32_fetch.log 2>&1 || { echo "f32 fetch rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/f32_write -o p -- python3 bench.py $ARGS_F32 > $D/f32_write.log 2>&1 || { echo "f32 write rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/bf16_fetch -o p -- python3 bench.py $ARGS_BF16 > $D/bf16_fetch.log 2>&1 || { echo "bf16 fetch rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/bf16_write -o p -- python3 bench.py $ARGS_BF16 > $D/bf16_write.log 2>&1 || { echo "bf16 write rc=$?"; exit 1; }
echo done

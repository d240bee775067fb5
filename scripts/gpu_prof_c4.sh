#!/bin/bash
# rocprofv3 kernel trace of the c4 rank shape (N = 8 x M = 10, T = 160, bf16: the layer wavefronts); PN / PT: another rank shape (c5: PN=32 PT=180)
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-c4prof}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --N ${PN:-8} --T ${PT:-160} --dtype bf16 --steps 5 --warmup 2 --no-cpu-baseline --no-vendor --no-bf16 --no-f32x --no-extras --fwd-steps 1 > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -5 $O/prof.log; exit 1; }
grep '^{' $O/prof.log | cut -c1-200
python3 scripts/trace_timeline.py $(find $O/prof -name "*kernel_trace.csv" | head -1) 3 > $O/timeline.txt 2>&1; head -30 $O/timeline.txt

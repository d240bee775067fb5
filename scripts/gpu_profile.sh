#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC counters here).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 bench.py ${PROF_BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline --fwd-steps 1} > gpurun_out/prof_bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"
tail -3 gpurun_out/prof_bench.log
find gpurun_out/prof -name "*stats*" | head
exit $rc

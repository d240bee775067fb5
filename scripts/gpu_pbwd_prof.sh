#!/bin/bash
# bf16 stack backward timing + kernel stats per schedule
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pbprof
export TMPDIR=/tmp
for kv in ${PB_ENVS:-SV_PERSIST_BWD=0 SV_PERSIST_BWD=1}; do
  env ${kv//,/ } timeout -k 10 120 python scripts/pbwd_bench.py || exit 1
  env ${kv//,/ } PB_ITERS=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pbprof -o $kv -- python3 scripts/pbwd_bench.py > gpurun_out/pbprof/$kv.log 2>&1 || exit 1
  python -c "
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print('   ', r['Name'].split('(')[0][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')" gpurun_out/pbprof/${kv}_kernel_stats.csv
done

#!/bin/bash
# L2 request rates of the c3 bf16 persistent recurrences (scripts/persist_ab.py --iters 1): two
# rocprofv3 --pmc passes, each its own run, nothing traced beside them.  Folded by the python below.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/pmc_l2; mkdir -p $D; export TMPDIR=/tmp
i=0
for set in "GRBM_GUI_ACTIVE TCC_REQ_sum TCC_HIT_sum TCC_READ_sum" "GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $D/p$i -o p -- python3 scripts/persist_ab.py --iters 1 > $D/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -4 $D/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmc_l2/p*/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "persist3" not in k and "gemm_bf16" not in k: continue
        agg[k[:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        print(f.split("/")[2], k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY

#!/bin/bash
# PMC passes over scripts/gemm_pmc_bf16.py (each pass its own run; never combined with tracing)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bpmc
export TMPDIR=/tmp
sets=("GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES"
      "GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT")
i=0
for set in "${sets[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/bpmc -o pass$i -- python3 scripts/gemm_pmc_bf16.py > gpurun_out/bpmc/pass$i.log 2>&1 || { echo "pass $i rc=$?"; tail -3 gpurun_out/bpmc/pass$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/bpmc/pass*_counter_collection.csv")):
    rows = list(csv.DictReader(open(f)))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        if "gemm_bf16_256" not in r["Kernel_Name"]:
            continue
        key = (r["Grid_Size"] if "Grid_Size" in r else r.get("Grid_Size_X", "?"), r["Kernel_Name"][:40])
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for key, d in agg.items():
        print(f.split("/")[-1], key, {k: round(sum(v) / len(v), 1) for k, v in d.items()})
PY

#!/bin/bash
# bf16 K1 (persistent 8-phase, bf16 out) tile order A/B: row-major vs column groups of 6 / 3
cd "$GRAFT_REPO_ROOT"; export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp; O=gpurun_out/${TAG:-k1order}; mkdir -p $O
for L in ${LIBS:-g0 g6 g3 g0 g6 g3}; do
  timeout -k 10 200 python -u scripts/gemm_bench.py --bf16 --shapes Gx --bias --reps 10 --lib scripts/ab/libsv_ge2e_$L.so >> $O/time.log 2>&1 || { echo "$L rc=$?"; tail -5 $O/time.log; exit 1; }
done
grep '^{' $O/time.log
D=$O/traffic; mkdir -p $D
for L in ${TLIBS:-g0 g6 g3}; do
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/f_$L -o p -- python3 scripts/gemm_traffic.py --lib scripts/ab/libsv_ge2e_$L.so > $D/f_$L.log 2>&1 || { echo "$L fetch rc=$?"; tail -3 $D/f_$L.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, os
O = os.environ.get("TAG", "k1order")
for f in sorted(glob.glob(f"gpurun_out/{O}/traffic/f_*/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "8qp" in r["Kernel_Name"]:
            agg[r["Dispatch_Id"]].append(float(r["Counter_Value"]))
    vals = [sum(v) for v in agg.values()]
    print(f.split("/")[3], "8qp FETCH_SIZE per launch (KB, raw):", [round(v) for v in vals])
PY

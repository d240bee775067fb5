"""Fold scripts/gpu_pmc_persist.sh's f32 / bf16 runs for the GEMMs: per (kernel, grid) the average
duration (kernel trace), the effective clock GRBM_GUI_ACTIVE / 8 / duration and the MFMA-busy
fraction SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles x 1024 SIMDs), as pmc_persist.py does for the
recurrences.  Usage: python scripts/pmc_gemm.py gpurun_out/pmc_persist"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1]
PREFIX = ("gemm_f32_256", "gemm_f32_narrow", "gemm_bf16_8q", "gemm_bf16_kernel", "gemm_bf16_narrow")


def grid(r):
    if "Grid_Size" in r:
        return int(r["Grid_Size"])
    return int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1)) * int(r.get("Grid_Size_Z", 1))


def key(r):
    n = r["Kernel_Name"]
    for pre in ("void ", "(anonymous namespace)::"):
        if n.startswith(pre):
            n = n[len(pre):]
    short = n.split("(")[0]
    if not short.startswith(PREFIX):
        return None
    return f"{short} grid={grid(r)}"


out = {}
for w in ("f32", "bf16", "c4", "c5"):
    tr = glob.glob(os.path.join(d, f"{w}_trace", "**", "*kernel_trace.csv"), recursive=True)
    pm = glob.glob(os.path.join(d, f"{w}_pmc", "**", "*counter_collection.csv"), recursive=True)
    if not tr or not pm:
        continue
    dur = defaultdict(list)
    for r in csv.DictReader(open(tr[0])):
        k = key(r)
        if k:
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    cnt = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(pm[0])):
        k = key(r)
        if k:
            cnt[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in dur:
        if k not in cnt or not cnt[k]["GRBM_GUI_ACTIVE"]:
            continue
        t = sum(dur[k]) / len(dur[k])
        gui = sum(cnt[k]["GRBM_GUI_ACTIVE"]) / len(cnt[k]["GRBM_GUI_ACTIVE"])
        mf = sum(cnt[k]["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(cnt[k]["SQ_VALU_MFMA_BUSY_CYCLES"])
        out[f"{w}:{k}"] = {"launches": len(dur[k]), "avg_us": round(t * 1e6, 1),
                           "clock_GHz": round(gui / 8 / t / 1e9, 3), "mfma_busy_frac": round(mf / (gui / 8 * 1024), 4)}
print(json.dumps(out, indent=1))

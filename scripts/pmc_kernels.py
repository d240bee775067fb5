"""Fold per-kernel PMC runs (any counter sets, one rocprofv3 run each, plus a kernel trace) for
kernels whose name contains one of the given substrings: mean counter value per launch and the mean
traced duration.  Usage: python scripts/pmc_kernels.py <dir> <prefix> <substr> [<substr> ...]
(<dir>/<prefix>_*/**/p_counter_collection.csv and <dir>/<prefix>_trace/**/p_kernel_trace.csv)"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d, pre, subs = sys.argv[1], sys.argv[2], sys.argv[3:]


def match(n):
    for s in subs:
        if s in n:
            return s
    return None


out = defaultdict(dict)
for f in glob.glob(os.path.join(d, f"{pre}_*", "**", "*counter_collection.csv"), recursive=True):
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = match(r["Kernel_Name"])
        if k:
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        for c, v in cs.items():
            out[k][c] = sum(v) / len(v)
for f in glob.glob(os.path.join(d, f"{pre}_trace", "**", "*kernel_trace.csv"), recursive=True):
    dur = defaultdict(list)
    for r in csv.DictReader(open(f)):
        k = match(r["Kernel_Name"])
        if k:
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    for k, v in dur.items():
        out[k]["avg_us"] = sum(v) / len(v)
        out[k]["launches"] = len(v)
for k, cs in out.items():
    if "GRBM_GUI_ACTIVE" in cs and "avg_us" in cs:
        cs["clock_GHz"] = cs["GRBM_GUI_ACTIVE"] / 8 / cs["avg_us"] / 1e3
        cs["mfma_busy_frac"] = cs["SQ_VALU_MFMA_BUSY_CYCLES"] / (cs["GRBM_GUI_ACTIVE"] / 8 * 1024)
print(json.dumps({k: {c: round(v, 4) for c, v in cs.items()} for k, cs in out.items()}, indent=1))

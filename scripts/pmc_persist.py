"""Fold scripts/gpu_pmc_persist.sh: per persistent-recurrence kernel, the average launch duration
(kernel trace; the c4 / c5 rank shapes' kernels keyed "c4:..." / "c5:..."), the effective clock GRBM_GUI_ACTIVE / 8 / duration (MI355X_MICROARCH.md, DVFS
give-back) and the MFMA-busy fraction SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles x 1024 SIMDs).
Usage: python scripts/pmc_persist.py gpurun_out/pmc_persist"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1]
KERNELS = ("lstm_persist_fwd_f32_kernel", "lstm_persist_bwd_f32_h2_kernel", "lstm_persist3_fwd_bf16_kernel",
           "lstm_persist3_bwd_bf16_kernel", "lstm_persist2_fwd_bf16_kernel", "lstm_persist2_bwd_bf16_kernel",
           "lstm_wave3_fwd_bf16_kernel", "lstm_wave_bwd_bf16_kernel")
out = {}
for w in ("f32", "bf16", "c4", "c5"):
    tr = glob.glob(os.path.join(d, f"{w}_trace", "**", "*kernel_trace.csv"), recursive=True)
    pm = glob.glob(os.path.join(d, f"{w}_pmc", "**", "*counter_collection.csv"), recursive=True)
    if not tr or not pm:
        continue
    dur = defaultdict(list)
    for r in csv.DictReader(open(tr[0])):
        for k in KERNELS:
            if r["Kernel_Name"].startswith("void " + k):
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    cnt = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(pm[0])):
        for k in KERNELS:
            if r["Kernel_Name"].startswith("void " + k):
                cnt[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in dur:
        if k not in cnt:
            continue
        t = sum(dur[k]) / len(dur[k])
        gui = sum(cnt[k]["GRBM_GUI_ACTIVE"]) / len(cnt[k]["GRBM_GUI_ACTIVE"])
        mf = sum(cnt[k]["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(cnt[k]["SQ_VALU_MFMA_BUSY_CYCLES"])
        clk = gui / 8 / t  # (the profiled launch; the traced one gives the duration)
        out[k if w in ("f32", "bf16") else f"{w}:{k}"] = {"launches": len(dur[k]), "avg_us": round(t * 1e6, 1), "clock_GHz": round(clk / 1e9, 3),
                  "mfma_busy_frac": round(mf / (gui / 8 * 1024), 4)}
print(json.dumps(out, indent=1))

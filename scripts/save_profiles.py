"""Copy a gpu_checkpoint.sh run (gpurun_out/ckpt) into profiles/<tag>_*: kernel stats, timelines,
the bench line and the roofline cross-check (rocprof average of the K1-shape GEMM vs the bench's
live HIP-event number).  Usage: python scripts/save_profiles.py r01_v7"""
import csv
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
ck = os.path.join(ROOT, "gpurun_out", "ckpt")
prof = os.path.join(ROOT, "profiles")
for d in ("f32", "bf16"):
    shutil.copy(os.path.join(ck, f"prof_{d}", "run_kernel_stats.csv"), os.path.join(prof, f"{tag}_{d}_kernel_stats.csv"))
    with open(os.path.join(prof, f"{tag}_{d}_timeline.txt"), "w") as f:
        subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "trace_timeline.py"),
                        os.path.join(ck, f"prof_{d}", "run_kernel_trace.csv"), "2"], stdout=f, check=True)
lines = [ln for ln in open(os.path.join(ck, "bench.log")) if ln.startswith("{")]
open(os.path.join(prof, f"{tag}_bench.json.log"), "w").write(lines[-1])
b = json.loads(lines[-1])
rows = list(csv.DictReader(open(os.path.join(ck, "prof_f32", "run_kernel_trace.csv"))))
sel = [r for r in rows if r["Kernel_Name"].startswith("void gemm_km_kernel<128, 128, 0")
       and int(r["Grid_Size_X"]) == 19200 * 256]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in sel]
M, N, K = 102400, 3072, 768
with open(os.path.join(prof, f"{tag}_roofline_check.txt"), "w") as f:
    f.write("rocprofv3 kernel trace of `bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-vendor --no-bf16 "
            "--fwd-steps 1`\n")
    f.write("roofline kernel gemm_km_kernel<128,128,0> at the K1 shape (grid 19200 WGs: M 102400 x N 3072 / 128^2, "
            "K 768):\n")
    f.write(f"  launches {len(d)}, avg {sum(d) / len(d):.1f} us (min {min(d):.1f}, max {max(d):.1f})\n")
    f.write(f"  -> {2 * M * N * K / (sum(d) / len(d)) / 1e6:.1f} TFLOP/s; bench.py live HIP-event value: "
            f"{b['roofline']['achieved']} TF, {b['roofline']['avg_launch_us']} us\n")
print(open(os.path.join(prof, f"{tag}_roofline_check.txt")).read())
print(b["ms_per_step"], b.get("bf16", {}).get("ms_per_step"), b.get("f32_bf16x6", {}).get("ms_per_step"),
      b.get("vendor_baseline", {}).get("ms_per_step"), b.get("cpu_baseline", {}).get("sec_per_step"),
      b["roofline"]["frac"], b.get("roofline_step_kernel", {}).get("achieved"))

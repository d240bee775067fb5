"""Copy a gpu_checkpoint.sh run (gpurun_out/ckpt) into profiles/<tag>_*: kernel stats, timelines,
the bench line and the roofline cross-check (rocprof average of the K1-shape GEMM vs the bench's
live HIP-event number).  Usage: python scripts/save_profiles.py r01_v7 [gpurun_out subdirectory, default ckpt]"""
import csv
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) < 2 or sys.argv[1].startswith("-"):
    sys.exit(__doc__)
tag = sys.argv[1]
ck = os.path.join(ROOT, "gpurun_out", sys.argv[2] if len(sys.argv) > 2 else "ckpt")
prof = os.path.join(ROOT, "profiles")
for d in ("f32", "bf16"):
    shutil.copy(os.path.join(ck, f"prof_{d}", "run_kernel_stats.csv"), os.path.join(prof, f"{tag}_{d}_kernel_stats.csv"))
    with open(os.path.join(prof, f"{tag}_{d}_timeline.txt"), "w") as f:
        subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "trace_timeline.py"),
                        os.path.join(ck, f"prof_{d}", "run_kernel_trace.csv"), "2"], stdout=f, check=True)
lines = [ln for ln in open(os.path.join(ck, "bench.log")) if ln.startswith("{")]
open(os.path.join(prof, f"{tag}_bench.json.log"), "w").write(lines[-1])
b = json.loads(lines[-1])
# the roofline cross-check compares each trace with the bench line its OWN profiled run printed
# (the in-step kernel times depend on that run's concurrency; the full bench.log line is another run)
pf = {d: json.loads([ln for ln in open(os.path.join(ck, f"prof_{d}.log")) if ln.startswith("{")][-1])
      for d in ("f32", "bf16")}
def durations(d, prefix, grid=None, start=False):
    """Durations (us) of the matching launches in time order ((start, us) pairs with start=True)."""
    rows = csv.DictReader(open(os.path.join(ck, f"prof_{d}", "run_kernel_trace.csv")))
    sel = sorted((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows
                 if r["Kernel_Name"].startswith(prefix) and (grid is None or int(r["Grid_Size_X"]) == grid))
    return sel if start else [us for _, us in sel]


def line(f, what, d, bench_us, flops):
    avg = sum(d) / len(d)
    f.write(f"{what}: rocprofv3 {len(d)} launches, avg {avg:.1f} us (min {min(d):.1f}, max {max(d):.1f}) = "
            f"{flops / avg / 1e6:.1f} TFLOP/s; bench.py live value {bench_us} us\n")


B, T, H = 640, 160, 768
with open(os.path.join(prof, f"{tag}_roofline_check.txt"), "w") as f:
    f.write("rocprofv3 kernel traces of `bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-vendor --no-bf16 "
            "--fwd-steps 1` (f32, c2) and `... --dtype bf16` (c3) against the bench line of the same tree\n")
    rf = pf["f32"]["roofline"]
    if rf["kernel"].startswith("lstm_persist_bwd_f32_h2_kernel"):
        # one launch per layer: the headline run's timed steps are its launches [L, 4 L)
        d = durations("f32", "void lstm_persist_bwd_f32_h2_kernel")
        line(f, "roofline (c2 headline): lstm_persist_bwd_f32_h2_kernel, the 3 timed steps' launches", d[3:12],
             rf["avg_launch_us"], 2.0 * B * T * H * 4 * H)
        d = durations("f32", "void lstm_persist_fwd_f32_kernel")
        line(f, "roofline_fwd (c2 headline): lstm_persist_fwd_f32_kernel, the 3 timed steps' launches", d[3:12],
             pf["f32"]["roofline_fwd"]["avg_launch_us"], 2.0 * B * T * H * 4 * H)
    else:
        # the headline run's timed steps: launches [warmup, warmup + steps) x L*T of the first run
        d = durations("f32", "void lstm_step_bwd_v2_kernel")
        line(f, "roofline (c2 headline): lstm_step_bwd_v2_kernel (K3), the 3 timed steps' launches",
             d[480:4 * 480], rf["avg_launch_us"], 2.0 * B * H * 4 * H)
    rg = pf["f32"].get("roofline_gemm")
    if rg:
        # bench.py times 5 isolated launches at the K1 shape after the steps: the last 5 of that grid
        # (the 5 launches right before roofline_step_kernel's first lstm_step_fwd_v2_kernel: the
        # persistent GEMM's grid is one workgroup per CU for every shape, and d-vector runs follow)
        t_k2 = min(st for st, _ in durations("f32", "void lstm_step_fwd_v2_kernel", start=True))
        d = [us for st, us in durations("f32", "void gemm_f32_256p_kernel<256, 32>", start=True) if st < t_k2]
        line(f, "roofline_gemm: gemm_f32_256p_kernel<256,32> at the K1 shape, the 5 isolated launches", d[-5:],
             rg["avg_launch_us"], 2.0 * T * B * 4 * H * H)
    for key, pre in (("roofline", "void lstm_persist3_bwd_bf16_kernel"),
                     ("roofline_fwd", "void lstm_persist")):
        r = pf["bf16"].get(key)  # the --dtype bf16 run: its headline is c3
        if not r:
            continue
        # the c3 run's timed steps: its first (1 warm-up + 3) x L layer launches, minus the warm-up's
        d = durations("bf16", pre) if key == "roofline" else sorted(
            durations("bf16", "void lstm_persist3_fwd_bf16_kernel", start=True) +
            durations("bf16", "void lstm_persist2_fwd_bf16_kernel", start=True))
        d = [x[1] if isinstance(x, tuple) else x for x in d][3:12]
        line(f, f"{key} of the c3 run: {pre[5:]}... per layer launch", d, r["avg_launch_us"], 2.0 * B * T * H * 4 * H)
print(open(os.path.join(prof, f"{tag}_roofline_check.txt")).read())
print(b["ms_per_step"], b.get("bf16", {}).get("ms_per_step"), b.get("f32_bf16x6", {}).get("ms_per_step"),
      b.get("vendor_baseline", {}).get("ms_per_step"), b.get("cpu_baseline", {}).get("sec_per_step"),
      b["roofline"]["frac"], b.get("roofline_gemm", {}).get("frac"), b.get("roofline_bf16", {}).get("frac"))

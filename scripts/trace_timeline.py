#!/usr/bin/env python3
"""Timeline analysis of a rocprofv3 kernel trace: splits the run into training steps (by the
clip_sgd kernel that ends each step), and for one step reports wall time, union-busy time,
per-kernel-class busy time and the concurrency profile.  Usage:
    python scripts/trace_timeline.py gpurun_out/prof/run_kernel_trace.csv [step_index]"""
import csv
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "")


def step_ends(ks):
    """End of each training step: its clip_sgd2_kernel (both parameter groups in one launch, ABI
    v8), or the second clip_sgd_kernel of each step (net group, then w/b group) in older traces."""
    two = [k[1] for k in ks if k[2].startswith("clip_sgd2")]
    return two if two else [k[1] for k in ks if k[2].startswith("clip_sgd")][1::2]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    which = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"])
                 for r in rows), key=lambda x: x[0])
    ends = step_ends(ks)
    starts = [ks[0][0]] + ends[:-1]
    s0, s1 = starts[which], ends[which]
    sel = [k for k in ks if k[0] >= s0 and k[1] <= s1]
    wall = s1 - s0
    ev = sorted([(a, 1) for a, _, _, _ in sel] + [(b, -1) for _, b, _, _ in sel])
    conc = defaultdict(int)
    cur, last = 0, s0
    for t, d in ev:
        conc[cur] += t - last
        cur += d
        last = t
    busy = defaultdict(int)
    cnt = defaultdict(int)
    for a, b, n, _ in sel:
        busy[n] += b - a
        cnt[n] += 1
    print(f"step {which}: wall {wall / 1e6:.3f} ms, kernels {len(sel)}")
    print("concurrency profile (ms at k kernels running):",
          {k: round(v / 1e6, 3) for k, v in sorted(conc.items())})
    for n, v in sorted(busy.items(), key=lambda x: -x[1])[:14]:
        print(f"  {n[:60]:60s} n={cnt[n]:5d} busy={v / 1e6:8.3f} ms avg={v / cnt[n] / 1e3:8.2f} us")
    # the step in launch order: each kernel's duration and the idle gap before it (the previous
    # kernel's end to this one's start, 0 when they overlap)
    print("in order (gap before, duration, us):")
    prev, gaps = s0, 0
    for a, b, n, _ in sel:
        g = max(0, a - prev)
        gaps += g
        print(f"  {g / 1e3:7.2f} {(b - a) / 1e3:9.2f}  {n[:70]}")
        prev = max(prev, b)
    print(f"idle gaps total {gaps / 1e3:.1f} us")


if __name__ == "__main__":
    main()


def phases(path, which=-1):
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows))
    ends = step_ends(ks)
    starts = [ks[0][0]] + ends[:-1]
    s0, s1 = starts[which], ends[which]
    sel = [k for k in ks if k[0] >= s0 and k[1] <= s1]
    fwd_end = max(b for a, b, n in sel if "step_fwd" in n)
    bwd_start = min(a for a, b, n in sel if "step_bwd" in n)
    last_bwd_step = max(b for a, b, n in sel if "step_bwd" in n)
    print(f"fwd phase {(fwd_end - s0) / 1e6:.3f} ms | fwd end -> first bwd step {(bwd_start - fwd_end) / 1e6:.3f} ms"
          f" | bwd steps span {(last_bwd_step - bwd_start) / 1e6:.3f} ms | tail {(s1 - last_bwd_step) / 1e6:.3f} ms")
    # per layer (grid signature not in tuple; use order: bwd steps come in 3 streams)

"""Per-rank step of every multi-GPU bench line, run alone on one GPU (world = 1).

The driver's 2/4/8-GPU scaling run executes these shapes on each rank; this script checks
on the one-GPU box that each of them runs (finite loss, no persistent-recurrence timeout) and
times it, for DESIGN §6's per-rank budgets:

  c2 / c3 (weak):   N = 64 per rank, T = 160            (the same shape at every world size)
  c4 (strong):      N = 64 / world per rank, T = 160, bf16
  c5 (strong):      N = 256 / world per rank, T = 180, bf16

Usage: python scripts/rank_shapes.py [--steps 5] [--warmup 2]
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = bench.Ctx(1, 0, dev)
    for world in (2, 4, 8):
        for name, Ng, T in (("c4", 64, 160), ("c5", 256, 180)):
            N = max(1, Ng // world)
            dt, loss, _, _, tr = bench.run_steps(ctx, N, 10, T, "bf16", args.steps, args.warmup, 2235)
            ms = dt / args.steps * 1e3
            ok = math.isfinite(loss)
            print(json.dumps({"line": name, "world": world, "N_per_rank": N, "M": 10, "T": T, "rows": N * 10,
                              "ms_per_step": round(ms, 3), "loss": round(loss, 5), "finite": ok,
                              "emb_per_s_if_linear": round(N * 10 * world / (ms * 1e-3), 1)}), flush=True)
            del tr
            torch.cuda.empty_cache()
            if not ok:
                sys.exit(1)


if __name__ == "__main__":
    main()

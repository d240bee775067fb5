"""Kernel timeline of one c5 rank's GE2E (N_local = 32 x M = 10 against N = 256 centroids, s0 = 224):
the fused sharded form (sv_ge2e_shard_prep / _rows / _finalize) and the split form, `--iters` calls
each, for rocprofv3 --kernel-trace --stats.  Usage: python scripts/ge2e_c5rank.py [--iters 20]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if "--lib" in sys.argv:  # an A/B build (Makefile `ab`) instead of the product library
    from pytorch_speaker_verification_amd import _lib  # noqa: E402
    _lib.use_library(sys.argv[sys.argv.index("--lib") + 1])
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--lib", default=None)
args = ap.parse_args()
dev = torch.device("cuda", 0)
print(bench.c5_rank_ge2e(dev, reps=args.iters))

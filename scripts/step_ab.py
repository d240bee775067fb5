"""Interleaved A/B of the fused training step (GE2ETrainer.step) between two complete trees --
this repo and another checkout holding its own package + built library (e.g. the previous
commit: `git worktree add ab_base HEAD~1 && make -C ab_base`) -- at the configs' per-GPU shapes,
in one process per tree and round (child processes: each imports its own package).
Usage: python scripts/step_ab.py --other ab_base [--rounds 3] [--shapes c4,c5,c3]
Prints one JSON line per (round, tree, shape): ms per step over `--steps` timed steps."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHAPES = {"c2": (64, 10, 160, "f32"), "c3": (64, 10, 160, "bf16"), "c4": (8, 10, 160, "bf16"),
          "c5": (32, 10, 180, "bf16")}
CHILD = r'''
import json, sys, time, torch
sys.path.insert(0, sys.argv[1])
from pytorch_speaker_verification_amd.speech_embedder_net import GE2ELoss, SpeechEmbedder
from pytorch_speaker_verification_amd.trainer import GE2ETrainer
N, M, T, prec, steps = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5], int(sys.argv[6])
dev = torch.device("cuda", 0)
torch.manual_seed(0)
net = SpeechEmbedder().to(dev)
net.precision = prec
tr = GE2ETrainer(net, GE2ELoss(dev), lr=0.01)
x = torch.randn(N * M, T, 40, generator=torch.Generator().manual_seed(7)).to(dev)
for _ in range(5):
    tr.step(x, N, M)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    loss = tr.step(x, N, M)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / steps
tr.check()
print("RES " + json.dumps({"ms": round(dt * 1e3, 4), "loss": float(loss)}))
'''

ap = argparse.ArgumentParser()
ap.add_argument("--other", required=True)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--shapes", default="c4,c5")
a = ap.parse_args()
trees = {"this": ROOT, "other": os.path.join(ROOT, a.other) if not os.path.isabs(a.other) else a.other}
for r in range(a.rounds):
    for name, path in trees.items():
        for sh in a.shapes.split(","):
            N, M, T, prec = SHAPES[sh]
            p = subprocess.run([sys.executable, "-c", CHILD, path, str(N), str(M), str(T), prec, str(a.steps)],
                               capture_output=True, text=True, timeout=300)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("RES ")]
            if p.returncode or not line:
                print(p.stderr[-2000:], file=sys.stderr)
                sys.exit(1)
            res = json.loads(line[0][4:])
            print(json.dumps({"round": r, "tree": name, "shape": sh, **res}), flush=True)

"""Bit-identity check of an A/B build against the product library: the bf16 stack forward +
backward at a rank shape (default c4: B = 80, T = 160) with fixed inputs; --out saves every output
tensor (torch.save of this script's own tensors), --compare A B reports the tensors that differ.
Usage: python scripts/bitident_ab.py [--lib L] --out f.pt ; python scripts/bitident_ab.py --compare a.pt b.pt"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--out", default=None)
ap.add_argument("--compare", nargs=2, default=None)
ap.add_argument("--B", type=int, default=80)
ap.add_argument("--T", type=int, default=160)
ap.add_argument("--reps", type=int, default=3)
args = ap.parse_args()
if args.compare:
    a, b = (torch.load(f, weights_only=True) for f in args.compare)
    bad = [k for k in a if not torch.equal(a[k], b[k])]
    print({"tensors": len(a), "differ": bad})
    sys.exit(1 if bad else 0)
from pytorch_speaker_verification_amd import _lib  # noqa: E402
if args.lib:
    _lib.use_library(args.lib)
from pytorch_speaker_verification_amd import ops  # noqa: E402
from pytorch_speaker_verification_amd._lib import PersistStatus  # noqa: E402
from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
net = SpeechEmbedder().to(dev)
x = torch.randn(args.B, args.T, 40, device=dev)
layers = net.LSTM_stack.layer_params()
wp, bp = net.projection.weight, net.projection.bias
ps = PersistStatus(dev)
out = {}
for r in range(args.reps):  # repeated: every launch must give the same bits
    emb, st = ops.embedder_forward_bf16(x, layers, wp, bp, save=True, status=ps)
    demb = torch.randn(emb.shape, generator=torch.Generator(device=dev).manual_seed(7), device=dev) * 0.1
    grads = ops.embedder_backward_bf16(st, demb, layers, wp, status=ps)
    torch.cuda.synchronize()
    flat = {"emb": emb}
    for i, g in enumerate(grads if isinstance(grads, (list, tuple)) else [grads]):
        if isinstance(g, torch.Tensor):
            flat[f"g{i}"] = g
        elif isinstance(g, (list, tuple)):
            for j, h in enumerate(g):
                if isinstance(h, torch.Tensor):
                    flat[f"g{i}_{j}"] = h
    flat = {k: v.detach().clone().cpu() for k, v in flat.items()}
    if r == 0:
        out = flat
    else:
        assert all(torch.equal(out[k], flat[k]) for k in out), "repeat differs"
print({"status": int(ps.block[0]), "tensors": len(out)})
if args.out:
    torch.save(out, args.out)

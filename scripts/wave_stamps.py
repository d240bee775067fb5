"""Per-phase cycles per step of the layer-wavefront kernels at the c4 rank shape (B = 80, T = 160,
bf16): a stamp build (`make ab NAME=wst FLAGS="-DSV_WAVE3_STAMP -DSV_WB_STAMP"`) records wave 0's
s_memtime cycle sums per phase per workgroup into the sync block; this prints the mean over the
workgroups of each layer, per step, for the forward (lstm_wave3_fwd_bf16_kernel) and the backward
(lstm_wave_bwd_bf16_kernel), and the launch times.
Usage: python scripts/wave_stamps.py --lib scripts/ab/libsv_ge2e_wst.so [--iters 5]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--B", type=int, default=80)
ap.add_argument("--T", type=int, default=160)
args = ap.parse_args()
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
emb, st = ops.embedder_forward_bf16(x, layers, wp, bp, save=True, status=ps)
demb = torch.randn_like(emb) * 0.1
fwd = lambda: ops.embedder_forward_bf16(x, layers, wp, bp, save=True, status=ps)  # noqa: E731
bwd = lambda: ops.embedder_backward_bf16(st, demb, layers, wp, status=ps)  # noqa: E731


def timed(f):
    for _ in range(2):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        f()
    e1.record()
    e1.synchronize()
    return round(e0.elapsed_time(e1) / args.iters, 4)


out = {"lib": args.lib or "libsv_ge2e.so", "B": args.B, "T": args.T, "fwd_ms": timed(fwd), "bwd_ms": timed(bwd),
       "status": int(ps.block[0])}
stamp0 = 32 + 4 * 64 * 32  # SV_SYNC_STAMP (words)
s64 = ps.block[stamp0:stamp0 + 2 * 1024 * 8].view(torch.int64).view(1024, 8).cpu().double()
for name, rows, names in (("fwd", s64[:512], ["wait", "h DMA issue", "x-part (wait + MFMA)", "h-part MFMA",
                                               "exchange + cell", "hand-off + arrival", "off-chain + next x DMA"]),
                          ("bwd", s64[512:], ["waits", "k-loop", "exchange + dx + cell", "hand-off + arrival",
                                              "dG^T + operand DMA"])):
    used = rows[:, :len(names)].sum(1) > 0
    if not used.any():
        continue
    per = {}
    for l in range(3):
        sel = used & (rows[:, 7 if name == "fwd" else 5] == l)
        if sel.any():
            m = rows[sel][:, :len(names)].mean(0) / (args.T - 1)
            per[f"layer{l}"] = {k: round(float(v), 1) for k, v in zip(names, m)}
            per[f"layer{l}"]["total"] = round(float(m.sum()), 1)
    out[name + "_cycles_per_step"] = per
print(json.dumps(out), flush=True)

"""A/B timing of the bf16 stack forward and backward at c3 (B = 640, T = 160, H = 768), HIP events
on the stream, for the product library or an A/B build (`make ab NAME=x FLAGS=...`, --lib).
With a stamp build (kPbwdDebug = 32 in sv_persist.hip, FLAGS=-DSV_PDBG=-1) it also prints the persistent backward's cycles per
step by phase (workgroup 0..N of the last backward layer launch: wait, A stream + MFMA + partial
exchange, cell epilogue, hand-off stores + arrival, post-arrival issue).
Usage: python scripts/persist_ab.py [--lib scripts/ab/libsv_ge2e_x.so] [--iters 5] [--B 640]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--B", type=int, default=640)
ap.add_argument("--T", type=int, default=160)
ap.add_argument("--schedule", default="auto")
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
ps = PersistStatus(dev)
wp, bp = net.projection.weight, net.projection.bias


def fwd():
    return ops.embedder_forward_bf16(x, layers, wp, bp, save=True, status=ps, schedule=args.schedule)


emb, st = fwd()
demb = torch.randn_like(emb) * 0.1


def bwd():
    ops.embedder_backward_bf16(st, demb, layers, wp, status=ps, schedule=args.schedule)


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
    return round(e0.elapsed_time(e1) / args.iters, 3)


out = {"lib": args.lib or "libsv_ge2e.so", "B": args.B, "T": args.T, "fwd_ms": timed(fwd), "bwd_ms": timed(bwd)}
out["status"] = int(ps.block[0])
# stamps: u64 [SV_NSTAMP_WG][SV_NSTAMP] at word SV_SYNC_STAMP = 32 + 4 * 64 * 32 of the sync block
stamp0 = 32 + 4 * 64 * 32
st64 = ps.block[stamp0:stamp0 + 2 * 1024 * 8].view(torch.int64).view(1024, 8)[:512, :5].cpu().double()
if st64.abs().sum() > 0:
    nwg = int((st64.sum(1) > 0).sum())
    per = st64[:nwg].mean(0) / (args.T - 1)
    names = ["wait", "A stream+MFMA+exchange", "cell epilogue", "hand-off+arrive", "post-arrival"]
    out["bwd_cycles_per_step"] = {k: round(float(v), 1) for k, v in zip(names, per)}
    out["bwd_cycles_total"] = round(float(per.sum()), 1)
    out["stamped_wgs"] = nwg
# forward stamps (the forward launcher's dbg = 32, FLAGS=-DSV_PDBG=-1): workgroup slots 512 .. of the same area, the last
# forward layer launch of the timed forwards
fw = ps.block[stamp0:stamp0 + 2 * 1024 * 8].view(torch.int64).view(1024, 8)[512:, :6].cpu().double()
if fw.abs().sum() > 0:
    nwg = int((fw.sum(1) > 0).sum())
    per = fw[:nwg].mean(0) / (args.T - 1)
    names = ["wait", "stage h + x-proj issue", "MFMA", "exchange+epilogue", "hand-off+arrive", "post-arrival"]
    out["fwd_cycles_per_step"] = {k: round(float(v), 1) for k, v in zip(names, per)}
    out["fwd_cycles_total"] = round(float(per.sum()), 1)
print(json.dumps(out), flush=True)

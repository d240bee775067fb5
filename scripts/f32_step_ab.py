"""A/B of the fp32 stack at c2 (B = 640, T = 160): forward and backward under the persistent
recurrences vs the layer-pipelined per-step kernels, HIP events on the stream, plus the per-layer
persistent launch times from the probes, and a full trainer step under each schedule.
Usage: python scripts/f32_step_ab.py [--iters 3] [--B 640] [--T 160]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if "--lib" in sys.argv:  # an A/B build (Makefile `ab`) instead of the product library
    from pytorch_speaker_verification_amd import _lib  # noqa: E402
    _lib.use_library(sys.argv[sys.argv.index("--lib") + 1])
from pytorch_speaker_verification_amd import ops  # noqa: E402
from pytorch_speaker_verification_amd._lib import PersistStatus  # noqa: E402
from pytorch_speaker_verification_amd.speech_embedder_net import GE2ELoss, SpeechEmbedder  # noqa: E402
from pytorch_speaker_verification_amd.trainer import GE2ETrainer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=3)
ap.add_argument("--B", type=int, default=640)
ap.add_argument("--T", type=int, default=160)
ap.add_argument("--lib", default=None)
ap.add_argument("--only", default=None, help="one schedule only")
ap.add_argument("--wave-stamps", action="store_true", help="with --stamps: a -DSV_PF32_WAVE_STAMP build, "
                "the backward's phases of every wave (workgroups 0-127)")
ap.add_argument("--stamps", action="store_true", help="a -DSV_PF32_STAMP build: the persistent forward's "
                "cycles per step by phase (last forward layer launch, mean and max over workgroups)")
args = ap.parse_args()
dev = torch.device("cuda", 0)
torch.manual_seed(0)
net = SpeechEmbedder().to(dev)
x = torch.randn(args.B, args.T, 40, device=dev)
layers = net.LSTM_stack.layer_params()
wp, bp = net.projection.weight, net.projection.bias
L = len(layers)


def ev(n):
    e = [torch.cuda.Event(enable_timing=True) for _ in range(n)]
    for q in e:
        q.record()
    return e


def timed(f):
    for _ in range(1):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        f()
    e1.record()
    e1.synchronize()
    return round(e0.elapsed_time(e1) / args.iters, 3)


out = {"B": args.B, "T": args.T, "lib": args.lib or "libsv_ge2e.so"}
for sched in ((args.only,) if args.only else ("auto", "per_step")):
    ps = PersistStatus(dev)
    # (probe arrays: 2 L events under the persistent schedule; the per-step one takes 2 L nch)
    pers = sched != "per_step"
    pf, pb = (ev(2 * L), ev(2 * L)) if pers else (None, None)
    emb, st = ops.embedder_forward(x, layers, wp, bp, status=ps, schedule=sched, probe=pf)
    demb = torch.randn_like(emb) * 0.1
    ops.embedder_backward(st, demb, layers, wp, status=ps, schedule=sched, probe=pb)
    torch.cuda.synchronize()
    o = {"fwd_ms": timed(lambda: ops.embedder_forward(x, layers, wp, bp, status=ps, schedule=sched)),
         "bwd_ms": timed(lambda: ops.embedder_backward(st, demb, layers, wp, status=ps, schedule=sched))}
    if pers:
        o["fwd_layer_us"] = [round(pf[2 * l].elapsed_time(pf[2 * l + 1]) * 1e3, 1) for l in range(L)]
        o["bwd_layer_us"] = [round(pb[2 * l].elapsed_time(pb[2 * l + 1]) * 1e3, 1) for l in range(L)]
    net.schedule = sched
    tr = GE2ETrainer(net, GE2ELoss(dev), lr=0.01)
    M = 10 if args.B % 10 == 0 else 8
    o["step_ms"] = timed(lambda: tr.step(x, args.B // M, M))
    tr.check()
    o["status"] = int(ps.block[0])
    if args.stamps:
        # u64 [SV_NSTAMP_WG][SV_NSTAMP] at word 32 + 4 * 64 * 32 of the sync block, written by the
        # last forward launch: wait, first-chunk DMA, rest of k-loop, exchange + cell, hand-off, off-chain
        ops.embedder_forward(x, layers, wp, bp, status=ps, schedule=sched)
        torch.cuda.synchronize()
        stamp0 = 32 + 4 * 64 * 32
        nwg = 24 * ((args.B + 63) // 64)
        st = ps.block[stamp0:stamp0 + 2 * 1024 * 8].view(torch.int64).view(1024, 8)[:nwg, :6].cpu().double()
        st = st / (args.T - 1)
        names = ["wait", "dma0", "kloop", "cell", "handoff", "offchain"]
        o["fwd_stamps_per_step_mean"] = {k: round(float(v), 1) for k, v in zip(names, st.mean(0))}
        o["fwd_stamps_per_step_max"] = {k: round(float(v), 1) for k, v in zip(names, st.max(0).values)}
        # the backward's (slots 512 + workgroup, wave 0, summed over both halves of steps t < T - 1)
        st_ = ops.embedder_forward(x, layers, wp, bp, status=ps, schedule=sched)[1]
        ops.embedder_backward(st_, demb, layers, wp, status=ps, schedule=sched)
        torch.cuda.synchronize()
        sb = ps.block[stamp0:stamp0 + 2 * 1024 * 8].view(torch.int64).view(1024, 8)[512:512 + nwg, :6].cpu().double()
        sb = sb / (args.T - 1)
        nb = ["wait", "kloop", "exchange", "cell", "handoff", "offchain"]
        o["bwd_stamps_per_step_mean"] = {k: round(float(v), 1) for k, v in zip(nb, sb.mean(0))}
        o["bwd_stamps_per_step_max"] = {k: round(float(v), 1) for k, v in zip(nb, sb.max(0).values)}
        if args.wave_stamps:  # a -DSV_PF32_WAVE_STAMP build: slots 512 + 4 wg + wave, workgroups 0-127
            sw = ps.block[stamp0:stamp0 + 2 * 1024 * 8].view(torch.int64).view(1024, 8)[512:1024, :6]
            sw = sw.cpu().double().view(128, 4, 6) / (args.T - 1)
            o["bwd_stamps_per_wave_mean"] = {f"wave{w}": {k: round(float(v), 1) for k, v in zip(nb, sw[:, w].mean(0))}
                                             for w in range(4)}
    out[sched] = o
    print(json.dumps({sched: o}), flush=True)
print(json.dumps(out), flush=True)

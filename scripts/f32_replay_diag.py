"""Diagnostic for the fp32 persistent forward's graph-replay disagreement (r03: the second replay of
dvector.GraphedEmbedder with schedule 'persist' differed from the eager call by 3.8e-2).

Replays the failing sequence (tests/test_dvector.py graphed test: weights scale 2.0, seeds 20..23)
R times with the persistent schedule forced in both the graphed and the eager call, and compares
EACH side with the per-step schedule (bit-identical by construction), so the wrong side is named.
Phase B captures embedder_forward(save=True) so every layer's h_tm stays reachable and reports the
first diverging (replay, layer, step, row block, unit block) against per-step.
Usage: python scripts/f32_replay_diag.py [--lib scripts/ab/libsv_ge2e_x.so] [--reps 6]"""
import argparse
import functools
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--reps", type=int, default=6)
ap.add_argument("--phase", default="AB")
ap.add_argument("--precision", default="f32")
ap.add_argument("--between", default="persist", help="eager call between phase-B replays: persist|per_step|none")
args = ap.parse_args()
from pytorch_speaker_verification_amd import _lib  # noqa: E402

if args.lib:
    _lib.use_library(args.lib)
import recipe  # noqa: E402
from conftest import model_dims  # noqa: E402
from pytorch_speaker_verification_amd import dvector, ops  # noqa: E402
from pytorch_speaker_verification_amd._lib import PersistStatus  # noqa: E402
from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder  # noqa: E402

dev = torch.device("cuda", 0)
dims = (40, 768, 3, 256)
sd = recipe.make_weights(19, *dims, scale=2.0)
with model_dims(*dims):
    net = SpeechEmbedder()
with torch.no_grad():
    for k, v in net.state_dict().items():
        v.copy_(torch.as_tensor(sd[k]))
net = net.cuda()
layers = net.LSTM_stack.layer_params()
wp, bp = net.projection.weight, net.projection.bias
base_fwd = ops.embedder_forward


def ref(x):
    return base_fwd(x.to(dev), layers, wp, bp, save=False, schedule="per_step")[0]


def md(a, b):
    return float((a - b).abs().max())


if "A" in args.phase:
    # phase A: the r29 sequence, persistent schedule forced in both calls
    if args.precision == "bf16":
        base_bf = ops.embedder_forward_bf16
        dvector.embedder_forward_bf16 = functools.partial(base_bf, schedule="persist")

        def ref(x):  # noqa: F811  (bf16: persistent and per-step are bit-identical too)
            return base_bf(x.to(dev), layers, wp, bp, save=False, schedule="per_step")[0]
    else:
        dvector.embedder_forward = functools.partial(base_fwd, schedule="persist")
    ge = dvector.GraphedEmbedder(net, precision=args.precision)
    bad = 0
    for rep in range(args.reps):
        for seed, S in ((20, 128), (21, 128), (22, 100), (23, 37), (25, 640), (26, 640)):
            x = torch.as_tensor(recipe.make_frames(seed + 100 * rep, S, 24, 40))
            got = ge(x)
            eag = dvector.embed_windows(net, x, batch=S, precision=args.precision)
            r = ref(x)
            rec = {"rep": rep, "S": S, "graph_vs_per_step": md(got, r), "eager_vs_per_step": md(eag, r)}
            bad += rec["graph_vs_per_step"] > 0 or rec["eager_vs_per_step"] > 0
            print(json.dumps(rec), flush=True)
    dvector.embedder_forward = base_fwd
    print(json.dumps({"phase": "A", "mismatching_calls": bad}), flush=True)

if "B" in args.phase:
    # phase B: save=True captures keep every layer's h_tm; first divergence per replay
    for S in (128, 640):
        st_ = PersistStatus(dev)
        xs = torch.zeros((S, 24, 40), device=dev)

        def f():
            return base_fwd(xs, layers, wp, bp, save=True, schedule="persist", status=st_)

        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            f()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            emb, st = f()
        for rep in range(args.reps):
            x = torch.as_tensor(recipe.make_frames(300 + rep, S, 24, 40)).to(dev)
            xs.copy_(x)
            g.replay()
            # an eager call in between (the failing sequence had eager persistent calls)
            if args.between != "none":
                _ = base_fwd(x, layers, wp, bp, save=False, schedule=args.between)[0]
            re, rst = base_fwd(x, layers, wp, bp, save=True, schedule="per_step")
            torch.cuda.synchronize()
            first = None
            slot0 = [float(st.h_tm[l][0].abs().max()) for l in range(3)]
            slot0_ref = [float(rst.h_tm[l][0].abs().max()) for l in range(3)]
            for l in range(3):
                d = (st.h_tm[l][1:] - rst.h_tm[l][1:]).abs()  # [T, B, H]: h_0 .. h_{T-1}
                dg = (st.gates[l] - rst.gates[l]).abs()      # activations [T, B, 4H]
                dc = (st.c_tm[l] - rst.c_tm[l]).abs()
                if float(d.max()) > 0 and first is None:
                    t = int((d.amax(dim=(1, 2)) > 0).nonzero()[0])
                    rows = (d[t].amax(dim=1) > 0).nonzero().flatten()
                    cols = (d[t].amax(dim=0) > 0).nonzero().flatten()
                    gcols = (dg[t].amax(dim=0) > 0).nonzero().flatten()
                    first = {"layer": l, "t": t, "row_blocks": sorted(set((rows // 64).tolist())),
                             "unit_blocks": sorted(set((cols // 32).tolist())), "n_rows": int(rows.numel()),
                             "n_cols": int(cols.numel()), "max": float(d[t].max()),
                             "gates_first_t": int((dg.amax(dim=(1, 2)) > 0).nonzero()[0]),
                             "gate_cols_at_t": sorted(set((gcols // 768).tolist())),
                             "c_first_t": int((dc.amax(dim=(1, 2)) > 0).nonzero()[0])}
                    # which (row, unit) pairs: row-block x unit-block tiles hit at t
                    tiles = ((d[t] > 0).reshape(S // 64 if S % 64 == 0 else 1, -1, 24, 32).amax(dim=(1, 3))
                             if S % 64 == 0 else None)
                    if tiles is not None:
                        first["tiles"] = [[int(i), int(j)] for i, j in tiles.nonzero().tolist()][:40]
            print(json.dumps({"S": S, "rep": rep, "emb_vs_per_step": md(emb, re), "first": first,
                              "slot0_graph": slot0, "slot0_per_step": slot0_ref,
                              "status": int(st_.block[0]), "w1": int(st_.block[1])}), flush=True)

if "T" in args.phase:
    # phase T (run under rocprofv3 --kernel-trace): one graph at S = 128, three replays, nothing
    # in between, so the trace shows each replay's kernels back to back
    S = 128
    st_ = PersistStatus(dev)
    xs = torch.zeros((S, 24, 40), device=dev)

    def f():
        return base_fwd(xs, layers, wp, bp, save=False, schedule="persist", status=st_)[0]

    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        f()
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        emb = f()
    for rep in range(3):
        x = torch.as_tensor(recipe.make_frames(400 + rep, S, 24, 40)).to(dev)
        xs.copy_(x)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        print(json.dumps({"trace_rep": rep, "emb_vs_per_step": md(emb, ref(x))}), flush=True)

if "M" in args.phase:
    # phase M: does a hipMemsetAsync captured into a torch CUDA graph take effect on replay, in order
    # with the kernels around it?  buf := 7; graph: memset(buf[:n], 0) -> buf += 1; after each
    # replay buf[:n] must be 1 and buf[n:] must be 8 (then buf is refilled with 7)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    for nbytes in (256, 4096, 393216):
        n = nbytes // 4
        buf = torch.full((n + 1024,), 7, dtype=torch.int32, device=dev)
        s = torch.cuda.Stream(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            rc = hip.hipMemsetAsync(buf.data_ptr(), 0, nbytes, torch.cuda.current_stream(dev).cuda_stream)
            buf.add_(1)
        res = []
        for rep in range(4):
            buf.fill_(7)
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            res.append([int((buf[:n] == 1).sum()), int((buf[n:] == 8).sum())])
        print(json.dumps({"memset_bytes": nbytes, "rc": rc, "replays_ok_counts": res, "expect": [n, 1024]}),
              flush=True)

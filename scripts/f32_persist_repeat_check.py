"""Repeated eager fp32 persistent forwards with new inputs each call, against the per-step schedule
(bit-identical by construction), at B = 128 (48 workgroups) and B = 640 (c2's 240), T = 24 and 160;
then the same inside a HIP graph (replays with new inputs)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pytorch_speaker_verification_amd.ops import embedder_forward  # noqa: E402
from pytorch_speaker_verification_amd._lib import PersistStatus  # noqa: E402

dev = torch.device("cuda", 0)
net, _ = bench.build_model(bench.DIMS, dev)
layers = net.LSTM_stack.layer_params()
wp, bp = net.projection.weight, net.projection.bias
for B, T in ((128, 24), (640, 24), (640, 160)):
    diffs = []
    for k in range(4):
        x = torch.randn(B, T, 40, device=dev)
        a = embedder_forward(x, layers, wp, bp, save=False, schedule="persist")[0]
        r = embedder_forward(x, layers, wp, bp, save=False, schedule="per_step")[0]
        diffs.append(float((a - r).abs().max()))
    # graph replays
    st = PersistStatus(dev)
    xs = torch.randn(B, T, 40, device=dev)
    f = lambda: embedder_forward(xs, layers, wp, bp, save=False, schedule="persist", status=st)[0]  # noqa: E731
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        f()
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = f()
    gd = []
    for k in range(4):
        xs.copy_(torch.randn(B, T, 40, device=dev))
        g.replay()
        r = embedder_forward(xs, layers, wp, bp, save=False, schedule="per_step")[0]
        gd.append(float((out - r).abs().max()))
    print(json.dumps({"B": B, "T": T, "eager_persist_vs_per_step": diffs, "graph_replays_vs_per_step": gd,
                      "status": int(st.block[0])}), flush=True)

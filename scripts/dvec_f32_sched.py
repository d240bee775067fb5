"""fp32 per-file d-vector call (T = 24): the forward's auto schedule (per-step kernels below the
3/4-fill rule) vs the fp32 persistent recurrences (schedule 'persist'), S windows per call."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pytorch_speaker_verification_amd.ops import embedder_forward  # noqa: E402

dev = torch.device("cuda", 0)
net, _ = bench.build_model(bench.DIMS, dev)
layers = net.LSTM_stack.layer_params()
wp, bp = net.projection.weight, net.projection.bias
for S in (64, 128, 256, 640):
    x = torch.randn(S, 24, 40, device=dev)
    res = {"S": S}
    outs = {}
    for sched in ("auto", "persist", "per_step"):
        f = lambda: embedder_forward(x, layers, wp, bp, save=False, schedule=sched)[0]  # noqa: E731
        outs[sched] = f()
        res[sched + "_ms"] = round(bench._timed(f, dev, 20), 3)
    res["persist_vs_auto_maxabs"] = float((outs["persist"] - outs["auto"]).abs().max())
    print(json.dumps(res), flush=True)

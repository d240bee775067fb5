"""Times d-vector bf16 inference at 16384 windows x T = 24: the per-timestep GEMM path
(sv_dvector_embed_bf16) and the persistent-batch path, HIP events on the stream."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_speaker_verification_amd import dvector  # noqa: E402
from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
net = SpeechEmbedder().to(dev)
S, T = int(os.environ.get("DV_S", "16384")), 24
x = torch.randn(S, T, 40, device=dev)
flops = sum(2.0 * S * T * 4 * 768 * ((40 if l == 0 else 768) + 768) for l in range(3)) + 2.0 * S * 768 * 256


def timed(f, n=5):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n


with torch.no_grad():
    out = {"S": S}
    for path in ("dvec", "persist"):
        ms = timed(lambda: dvector.embed_windows(net, x, precision="bf16", path=path))
        out[path] = {"ms": round(ms, 3), "tflops": round(flops / ms / 1e9, 1), "frac": round(flops / ms / 1e9 / 2500, 4)}
    print(json.dumps(out), flush=True)

"""Times the bf16 stack backward (c3 dims, T=160) with HIP events on its stream; the schedule
comes from the environment (SV_PERSIST_BWD, SV_PBWD_*, read once by the library)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_speaker_verification_amd import ops  # noqa: E402
from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder  # noqa: E402
from pytorch_speaker_verification_amd._lib import PersistStatus  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
net = SpeechEmbedder().to(dev)
x = torch.randn(640, 160, 40, device=dev)
layers = net.LSTM_stack.layer_params()
ps = PersistStatus(dev)
emb, st = ops.embedder_forward_bf16(x, layers, net.projection.weight, net.projection.bias, save=True, status=ps)
demb = torch.randn_like(emb) * 0.1
for _ in range(2):
    ops.embedder_backward_bf16(st, demb, layers, net.projection.weight, status=ps)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
n = int(os.environ.get("PB_ITERS", "5"))
e0.record()
for _ in range(n):
    ops.embedder_backward_bf16(st, demb, layers, net.projection.weight, status=ps)
e1.record()
e1.synchronize()
print(json.dumps({"persist_bwd": os.environ.get("SV_PERSIST_BWD", "-"), "P": os.environ.get("SV_PBWD_P", "8"),
                  "bwd_ms": round(e0.elapsed_time(e1) / n, 3), "status": int(ps.block[0])}), flush=True)
if int(os.environ.get("SV_PBWD_DEBUG", "0")) & 32:
    n = 240
    a = ps.stamps(n).numpy()[:, :5].astype("float64")
    names = ["wait", "gemm+exchange", "cell epilogue", "hand-off+arrive", "post-arrival issue"]
    per = a.mean(0) / 159.0  # per step (the last layer's launch, T-1 = 159 GEMM steps)
    print(json.dumps({"cycles_per_step": {k: round(v, 1) for k, v in zip(names, per)},
                      "total": round(per.sum(), 1)}), flush=True)

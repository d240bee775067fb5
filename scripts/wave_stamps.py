"""Per-phase cycle split of the layer-wavefront forward (lstm_wave3_fwd_bf16_kernel) at the c4 rank
shape: run with SV_WAVE3_STAMP=1 (profiling only).  Prints per layer the average s_memtime cycles
per step of each phase (wave 0 of each workgroup)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_speaker_verification_amd import ops  # noqa: E402
from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder  # noqa: E402
from pytorch_speaker_verification_amd._lib import PersistStatus  # noqa: E402

B, T = int(os.environ.get("WS_B", "80")), int(os.environ.get("WS_T", "160"))
dev = torch.device("cuda", 0)
torch.manual_seed(0)
net = SpeechEmbedder().to(dev)
x = torch.randn(B, T, 40, device=dev)
layers = net.LSTM_stack.layer_params()
ps = PersistStatus(dev)
for _ in range(3):
    emb, st = ops.embedder_forward_bf16(x, layers, net.projection.weight, net.projection.bias, save=True, status=ps)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
emb, st = ops.embedder_forward_bf16(x, layers, net.projection.weight, net.projection.bias, save=True, status=ps)
e1.record()
e1.synchronize()
nub, nrb, L = 24, (B + 31) // 32, 3
n = L * nub * nrb
a = ps.stamps(n).numpy()[:, :7].astype("float64")
names = ["own wait", "h DMA issue", "x wait + x-part", "h wait + h-part", "cell", "hand-off + arrive",
         "post stores + below wait + x DMA"]
q, rr = n >> 3, n & 7
out = {"fwd_ms": round(e0.elapsed_time(e1), 3), "status": int(ps.block[0])}
for layer in range(L):
    rows = []
    for i in range(n):
        xx = i & 7
        lg = xx * q + min(xx, rr) + (i >> 3)
        if lg // (nub * nrb) == layer:
            rows.append(a[i])
    per = sum(rows) / len(rows) / T
    out[f"layer{layer}"] = {k: round(v, 1) for k, v in zip(names, per)}
    out[f"layer{layer}"]["total"] = round(per.sum(), 1)
print(json.dumps(out, indent=1), flush=True)

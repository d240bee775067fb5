"""Times one persistent bf16 forward recurrence (T=160, c3 dims) with HIP events; the
SV_PERSIST_DEBUG env (read by the library) selects the diagnostic variants."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_speaker_verification_amd.ops import embedder_forward_bf16  # noqa: E402
from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder  # noqa: E402
from pytorch_speaker_verification_amd._lib import PersistStatus  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
net = SpeechEmbedder().to(dev)
x = torch.randn(640, 160, 40, device=dev)
layers = net.LSTM_stack.layer_params()
ps = PersistStatus(dev)
for _ in range(2):
    embedder_forward_bf16(x, layers, net.projection.weight, net.projection.bias, save=True, status=ps)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    embedder_forward_bf16(x, layers, net.projection.weight, net.projection.bias, save=True, status=ps)
e1.record()
e1.synchronize()
print(json.dumps({"debug": os.environ.get("SV_PERSIST_DEBUG", "0"), "persist": os.environ.get("SV_PERSIST", "1"),
                  "fwd_ms": round(e0.elapsed_time(e1) / 5, 3), "status": int(ps.block[0])}), flush=True)

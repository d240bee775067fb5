"""GE2E fwd+bwd timing at the c2 / c4-rank / c5-rank shapes: the fused 3-launch kernel
(sv_ge2e_train) vs the split path, HIP events on the launch stream; per-kernel times come from
rocprofv3 over this script."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_speaker_verification_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
out = {}
for N, M in ((64, 10), (8, 10), (32, 10)):
    g = torch.Generator().manual_seed(N)
    E = torch.nn.functional.normalize(torch.randn(N, M, 256, generator=g), dim=2).to(dev)
    w = torch.tensor(10.0, device=dev)
    b = torch.tensor(-5.0, device=dev)

    def fused():
        ops.ge2e_train(E, w, b)

    def split():
        _, _, st = ops.ge2e_forward(E, w, b)
        ops.ge2e_backward(st, w, b)
    res = {}
    for name, f in (("fused", fused), ("split", split)):
        for _ in range(5):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            f()
        e1.record()
        e1.synchronize()
        res[name + "_us"] = round(e0.elapsed_time(e1) / 50 * 1e3, 2)
    out[f"N{N}xM{M}"] = res
print(json.dumps(out))

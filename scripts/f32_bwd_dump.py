"""Dump the c2 fp32 stack backward's gradients (B = 640, T = 160, persistent schedule) of one seeded
input with a given build of the library, for a bitwise comparison of two builds
(python scripts/f32_bwd_dump.py [--lib scripts/ab/x.so] out.pt; then --compare a.pt b.pt)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if sys.argv[1] == "--compare":
    a, b = torch.load(sys.argv[2], weights_only=True), torch.load(sys.argv[3], weights_only=True)
    diff = {k: float((a[k] - b[k]).abs().max()) for k in a}
    print({"bit_identical": all(torch.equal(a[k], b[k]) for k in a), "max_abs_diff": max(diff.values()),
           "per_tensor": {k: (v, float(a[k].abs().max())) for k, v in diff.items()}})
    sys.exit(0)
if sys.argv[1] == "--lib":
    from pytorch_speaker_verification_amd import _lib
    _lib.use_library(sys.argv[2])
    sys.argv = sys.argv[2:]
import bench  # noqa: E402
from pytorch_speaker_verification_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
net, _ = bench.build_model(bench.DIMS, dev)
layers = net.LSTM_stack.layer_params()
g = torch.Generator(device="cpu").manual_seed(7)
x = torch.randn(640, 160, 40, generator=g).to(dev)
emb, st = ops.embedder_forward(x, layers, net.projection.weight, net.projection.bias)
demb = torch.randn(emb.shape, generator=g).to(dev) * 0.1
grads = ops.embedder_backward(st, demb, layers, net.projection.weight)
ops.check_persistent_status(wait=True)
torch.save({str(i): t.detach().cpu() for i, t in enumerate(grads)}, sys.argv[1])
print("dumped", sys.argv[1])

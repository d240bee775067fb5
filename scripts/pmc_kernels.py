"""Isolated launches of the dominant kernels for PMC collection (rocprofv3 --pmc)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_speaker_verification_amd._lib import call, lib, ptr  # noqa: E402

dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev).cuda_stream
B, T, H = 640, 160, 768
G = 4 * H
g = torch.Generator().manual_seed(0)
whh = (torch.randn(G, H, generator=g) * 0.03).to(dev)
hprev = torch.randn(B, H, generator=g).to(dev)
cprev = torch.randn(B, H, generator=g).to(dev)
gates = torch.randn(B, G, generator=g).to(dev)
c_t, h_t = torch.empty(B, H, device=dev), torch.empty(B, H, device=dev)
for _ in range(int(os.environ.get("REPS", "20"))):
    call("sv_lstm_step_fwd", ptr(hprev), ptr(whh), ptr(gates), ptr(cprev), ptr(c_t), ptr(h_t), B, H, s)
M, N, K = T * B, G, H
A = torch.randn(M, K, generator=g).to(dev)
Bm = torch.randn(N, K, generator=g).to(dev)
C = torch.empty(M, N, device=dev)
for _ in range(3):
    call("sv_gemm_f32", 1, 1, M, N, K, ptr(A), K, ptr(Bm), K, ptr(C), N, None, None, 0.0, None, 0, s)
torch.cuda.synchronize()
print("done")

# bf16 layer forward (K1 bf16 GEMM + 8 bf16 step kernels)
Tb = 8
x_bf = torch.randn(Tb, B, H, generator=g).bfloat16().to(dev)
wih_bf = (torch.randn(G, H, generator=g) * 0.03).bfloat16().to(dev)
whh_bf = (torch.randn(G, H, generator=g) * 0.03).bfloat16().to(dev)
bias = torch.zeros(G, device=dev)
gts = torch.empty(Tb, B, G, dtype=torch.bfloat16, device=dev)  # bf16 gates (ABI v3)
ctm = torch.empty(Tb, B, H, device=dev)
htm = torch.empty(Tb + 1, B, H, device=dev)
hbf = torch.empty(Tb + 1, B, H, dtype=torch.bfloat16, device=dev)
hT = torch.empty(H, (Tb + 1) * B, dtype=torch.bfloat16, device=dev)
for _ in range(2):
    call("sv_lstm_layer_fwd_bf16", ptr(x_bf), Tb, B, H, H, ptr(wih_bf), ptr(whh_bf), ptr(bias), ptr(bias), ptr(gts),
         ptr(ctm), ptr(htm), ptr(hbf), ptr(hT), s)
torch.cuda.synchronize()
print("done bf16")

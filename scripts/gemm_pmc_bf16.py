"""Isolated bf16 GEMM launches (the 256^2 kernel) at the c3 K1 / dx / dW shapes for rocprofv3
--pmc passes (MFMA busy, LDS waits and conflicts).  Usage under rocprofv3 --pmc ...."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_speaker_verification_amd._lib import call, lib, ptr  # noqa: E402

dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev).cuda_stream
B, T, H = 640, 160, 768
G = 4 * H
for (M, N, K) in ((T * B, G, H), (T * B, H, G), (G, H, T * B)):
    A = torch.randn(M, K, device=dev).bfloat16()
    Bm = torch.randn(N, K, device=dev).bfloat16()
    C = torch.empty(M, N, device=dev)
    w = torch.empty(lib().sv_gemm_bf16_workspace(M, N, K) // 4 + 1, device=dev)
    for _ in range(3):
        call("sv_gemm_bf16", M, N, K, ptr(A), K, ptr(Bm), K, ptr(C), N, None, None, 0.0, ptr(w), s)
    torch.cuda.synchronize()
    del A, Bm, C, w
print("done")

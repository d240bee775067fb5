"""Isolated fp32 GEMM launches at the K1 / dx shapes, ours and torch.matmul (hipBLASLt), for
rocprofv3 --pmc comparisons of clock and MFMA-busy (scripts/gpu_gemm_pmc.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_speaker_verification_amd._lib import call, ptr  # noqa: E402

dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev).cuda_stream
B, T, H = 640, 160, 768
G = 4 * H
for (M, N, K) in ((T * B, G, H), (T * B, H, G)):
    A = torch.randn(M, K, device=dev)
    Bm = torch.randn(N, K, device=dev)
    C = torch.empty(M, N, device=dev)
    for _ in range(3):
        call("sv_gemm_f32", 1, 1, M, N, K, ptr(A), K, ptr(Bm), K, ptr(C), N, None, None, 0.0, None, 0, s)
    if os.environ.get("WITH_TORCH", "1") == "1":
        for _ in range(3):
            torch.matmul(A, Bm.t(), out=C)
    torch.cuda.synchronize()
    del A, Bm, C
print("done")

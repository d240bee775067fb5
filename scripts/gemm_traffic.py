"""Isolated launches of the path's big NT GEMMs at the c2 / c3 shapes, for the HBM-traffic PMC
passes (scripts/gpu_gemm_traffic.sh -> scripts/pmc_traffic.py --gemm).  Each shape runs REPS
times after one warm-up call; the PMC fold tells the shapes apart by kernel name and grid.

  f32  K1 Gx = x . W_ih^T   M = T B = 102400, N = 4H = 3072, K = H = 768   gemm_f32_256_kernel<256,32,0>
  f32  dx    = dG . W_ih    M = 102400, N = 768, K = 3072                  gemm_f32_256_kernel<256,32,0>
  f32  dW    = dG^T . h     M = 3072, N = 768, K = 102400 (split-K slabs)  gemm_f32_256_kernel<256,32,1>
  bf16 K1 (bf16 output)                                                   gemm_bf16_8qp_kernel<2>
  bf16 dx (fp32 output)                                                   gemm_bf16_8q_kernel<0,1>
  bf16 dW (split-K slabs)                                                 gemm_bf16_8q_kernel<1,0>
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if "--lib" in sys.argv:  # an A/B build (Makefile `ab`)
    from pytorch_speaker_verification_amd import _lib  # noqa: E402
    _lib.use_library(sys.argv[sys.argv.index("--lib") + 1])
from pytorch_speaker_verification_amd._lib import call, lib, ptr  # noqa: E402

REPS = 3
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev).cuda_stream
B, T, H = 640, 160, 768
G = 4 * H
SHAPES = {"Gx": (T * B, G, H), "dx": (T * B, H, G), "dW": (G, H, T * B)}
for name, (M, N, K) in SHAPES.items():
    A = torch.randn(M, K, device=dev)
    Bm = torch.randn(N, K, device=dev)
    C = torch.empty(M, N, device=dev)
    w = torch.empty(lib().sv_gemm_f32_workspace(M, N, K) // 4 + 1, device=dev)
    for _ in range(1 + REPS):
        call("sv_gemm_f32", 1, 1, M, N, K, ptr(A), K, ptr(Bm), K, ptr(C), N, None, None, 0.0, ptr(w), 0, s)
    Ab, Bb = A.bfloat16(), Bm.bfloat16()
    del A, Bm
    if name == "Gx":
        Cb = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        for _ in range(1 + REPS):
            call("sv_gemm_bf16_bf", M, N, K, ptr(Ab), K, ptr(Bb), K, ptr(Cb), N, None, None, s)
        del Cb
    else:
        wb = torch.empty(lib().sv_gemm_bf16_workspace(M, N, K) // 4 + 1, device=dev)
        for _ in range(1 + REPS):
            call("sv_gemm_bf16", M, N, K, ptr(Ab), K, ptr(Bb), K, ptr(C), N, None, None, 0.0, ptr(wb), s)
        del wb
    torch.cuda.synchronize()
    del Ab, Bb, C, w
print("done", flush=True)

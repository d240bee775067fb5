"""fp32 GEMM accuracy / speed of the exact fp32 MFMA path vs the bf16x6 split (products mode 1; SV_F32_PRODUCTS selects it here):
errors against an fp64 reference on the same fp32 inputs, and the K1-shape throughput.
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_speaker_verification_amd._lib import call, lib, ptr  # noqa: E402

dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev).cuda_stream
MODE = int(os.environ.get("SV_F32_PRODUCTS", "0"))
out = {"products": MODE}
g = np.random.default_rng(5)
for name, (M, N, K, scale) in {"gx": (2048, 3072, 768, 1.0), "dw": (3072, 768, 20480, 1.0),
                               "mixed": (1024, 1024, 4096, 0.0)}.items():
    A = g.standard_normal((M, K)).astype(np.float32)
    B = g.standard_normal((N, K)).astype(np.float32)
    if name == "mixed":  # wide dynamic range: per-row / per-col scales over 2^-20 .. 2^20
        A *= np.exp2(g.uniform(-20, 20, (M, 1))).astype(np.float32)
        B *= np.exp2(g.uniform(-20, 20, (N, 1))).astype(np.float32)
    At, Bt = torch.tensor(A, device=dev), torch.tensor(B, device=dev)
    C = torch.empty(M, N, device=dev)
    ws = torch.empty(lib().sv_gemm_f32_workspace(M, N, K) // 4 + 1, device=dev)
    call("sv_gemm_f32", 1, 1, M, N, K, ptr(At), K, ptr(Bt), K, ptr(C), N, None, None, 0.0, ptr(ws), MODE, s)
    ref = A.astype(np.float64) @ B.astype(np.float64).T
    absref = np.abs(A).astype(np.float64) @ np.abs(B).astype(np.float64).T   # |A||B|^T: the error scale
    err = np.abs(C.cpu().numpy().astype(np.float64) - ref) / absref
    out[name] = {"max_rel_to_absprod": float(err.max()), "mean": float(err.mean())}
M, N, K = 102400, 3072, 768
A = torch.randn(M, K, device=dev)
Bm = torch.randn(N, K, device=dev) * 0.03
C = torch.empty(M, N, device=dev)
f = lambda: call("sv_gemm_f32", 1, 1, M, N, K, ptr(A), K, ptr(Bm), K, ptr(C), N, None, None, 0.0, None, MODE, s)  # noqa
f()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    f()
e1.record()
e1.synchronize()
us = e0.elapsed_time(e1) / 5 * 1e3
out["k1_us"] = round(us, 1)
out["k1_tflops_f32_equiv"] = round(2 * M * N * K / us / 1e6, 1)
print(json.dumps(out), flush=True)

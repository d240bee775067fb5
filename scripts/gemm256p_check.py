"""bf16 256-tile GEMM: result digest and timing at the c3 shapes, for an A/B of SV_GEMM256P
(run once per setting; equal digests = bit-identical results).  Prints one JSON line."""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_speaker_verification_amd._lib import call, lib, ptr  # noqa: E402

dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev).cuda_stream
SHAPES = {"K1": (102400, 3072, 768), "dW": (3072, 768, 102400), "dx": (102400, 768, 3072), "small": (512, 256, 4096)}
res = {"SV_GEMM256P": os.environ.get("SV_GEMM256P", "0")}
for name, (M, N, K) in SHAPES.items():
    g = torch.Generator(device=dev).manual_seed(1234)
    A = torch.randn(M, K, device=dev, generator=g).bfloat16()
    B = torch.randn(N, K, device=dev, generator=g).bfloat16()
    C = torch.empty(M, N, device=dev)
    w = torch.empty(lib().sv_gemm_bf16_workspace(M, N, K) // 4 + 1, device=dev)
    f = lambda: call("sv_gemm_bf16", M, N, K, ptr(A), K, ptr(B), K, ptr(C), N, None, None, 0.0, ptr(w), s)  # noqa: E731
    f()
    torch.cuda.synchronize()
    dig = hashlib.sha256(C.cpu().numpy().tobytes()).hexdigest()[:16]
    ref_err = None
    if name == "small":
        ref = A.float() @ B.float().t()
        ref_err = float((C - ref).abs().max() / ref.abs().max())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        f()
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) / 10 * 1e3
    res[name] = {"digest": dig, "us": round(us, 1), "tflops": round(2.0 * M * N * K / us / 1e6, 1), "rel_err": ref_err}
    del A, B, C, w
print(json.dumps(res), flush=True)

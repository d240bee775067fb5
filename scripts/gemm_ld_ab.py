"""GEMM time vs the operands' leading dimensions (row strides) at the c2 / c3 shapes: the product
kernels, operands allocated with padded rows -- a screen for L2-channel / DRAM concentration of
strides that are multiples of 2 KB.  HIP events on the stream; one JSON line per case.
Usage: python scripts/gemm_ld_ab.py [--reps 8] [--only bf16|f32]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_speaker_verification_amd._lib import call, lib, ptr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=8)
ap.add_argument("--only", default=None)
args = ap.parse_args()
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev).cuda_stream


def timeit(fn, reps, warm=2):
    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


torch.manual_seed(0)
T, B, H = 160, 640, 768
G, TB = 4 * H, T * B
# (name, M, N, K, [(lda, ldb), ...]); C = A . B^T, both K-contiguous
cases = [("dx", TB, H, G, [(G, G), (G, G + 8), (G, G + 64)]),
         ("K1", TB, G, H, [(H, H), (H + 64, H + 64), (H + 8, H + 8)]),
         ("dW", G, H, TB, [(TB, TB), (TB + 8, TB + 8), (TB + 64, TB + 64)])]
for dt in ("bf16", "f32"):
    if args.only and dt != args.only:
        continue
    for name, M, N, K, lds in cases:
        for lda, ldb in lds:
            mk = (lambda r, c: torch.randn(r, c, device=dev).bfloat16()) if dt == "bf16" else \
                (lambda r, c: torch.randn(r, c, device=dev))
            A, Bm = mk(M, lda), mk(N, ldb)
            C = torch.empty(M, N, device=dev)
            if dt == "bf16":
                w = torch.empty(lib().sv_gemm_bf16_workspace(M, N, K) // 4 + 1, device=dev)
                f = lambda: call("sv_gemm_bf16", M, N, K, ptr(A), lda, ptr(Bm), ldb, ptr(C), N, None, None, 0.0, ptr(w), s)  # noqa: E731
            else:
                w = torch.empty(lib().sv_gemm_f32_workspace(M, N, K) // 4 + 1, device=dev)
                f = lambda: call("sv_gemm_f32", 1, 1, M, N, K, ptr(A), lda, ptr(Bm), ldb, ptr(C), N, None, None, 0.0, ptr(w), 0, s)  # noqa: E731
            us = timeit(f, args.reps if dt == "bf16" else 3)
            print(json.dumps({"dtype": dt, "case": name, "M": M, "N": N, "K": K, "lda": lda, "ldb": ldb, "us": round(us, 1)}),
                  flush=True)
            del A, Bm, C, w

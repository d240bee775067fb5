"""fp32 / bf16 GEMM timing at the c2 shapes (ours via the C ABI, and torch.matmul =
hipBLASLt for comparison).  HIP events on the launch stream; prints one JSON line.
Usage: python scripts/gemm_bench.py [--torch] [--reps N]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_speaker_verification_amd._lib import call, lib, ptr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--torch", action="store_true")
ap.add_argument("--bf16", action="store_true")
ap.add_argument("--reps", type=int, default=8)
ap.add_argument("--check", action="store_true", help="bf16: error vs fp32 torch on the same bf16 inputs, "
                "and bitwise repeatability over --reps runs (a race screen)")
ap.add_argument("--shapes", default="Gx,dW,dx")
ap.add_argument("--lib", default=None, help="load this build of the library instead (A/B builds)")
ap.add_argument("--fill", default="randn", help="operand data: randn | zeros (power / clock upper bound)")
ap.add_argument("--bias", action="store_true", help="Gx with the two bias vectors, as K1 runs in the stack")
args = ap.parse_args()
if args.lib:
    from pytorch_speaker_verification_amd import _lib
    _lib.use_library(args.lib)
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev).cuda_stream
B, T, H = 640, 160, 768
G = 4 * H
SHAPES = {"Gx": (T * B, G, H), "dW": (G, H, T * B), "dx": (T * B, H, G)}


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


res = {"lib": args.lib or "libsv_ge2e.so"}
for name, (M, N, K) in SHAPES.items():
    if name not in args.shapes.split(","):
        continue
    A = torch.randn(M, K, device=dev) if args.fill == "randn" else torch.zeros(M, K, device=dev)
    Bm = torch.randn(N, K, device=dev) if args.fill == "randn" else torch.zeros(N, K, device=dev)
    C = torch.empty(M, N, device=dev)
    w = torch.empty(lib().sv_gemm_f32_workspace(M, N, K) // 4 + 1, device=dev)
    b0, b1 = (torch.randn(N, device=dev), torch.randn(N, device=dev)) if args.bias and name == "Gx" else (None, None)
    pb0, pb1 = (ptr(b0), ptr(b1)) if b0 is not None else (None, None)
    f = lambda: call("sv_gemm_f32", 1, 1, M, N, K, ptr(A), K, ptr(Bm), K, ptr(C), N, pb0, pb1, 0.0, ptr(w), 0, s)  # noqa: E731
    us = timeit(f, args.reps)
    res["sv_f32_" + name] = [round(us, 1), round(2.0 * M * N * K / us / 1e6, 1)]
    if args.torch:
        ref = torch.matmul(A.double(), Bm.double().t()) if name == "Gx" else None
        us = timeit(lambda: torch.matmul(A, Bm.t()), args.reps)
        res["torch_f32_" + name] = [round(us, 1), round(2.0 * M * N * K / us / 1e6, 1)]
        if ref is not None:
            f()
            torch.cuda.synchronize()
            sc = (A.abs().double() @ Bm.abs().double().t())
            res["sv_f32_Gx_err"] = float(((C.double() - ref).abs() / sc).max())
            res["torch_f32_Gx_err"] = float(((torch.matmul(A, Bm.t()).double() - ref).abs() / sc).max())
            del ref, sc
    if args.bf16:
        Ab, Bb = A.bfloat16(), Bm.bfloat16()
        wb = torch.empty(lib().sv_gemm_bf16_workspace(M, N, K) // 4 + 1, device=dev)
        us = timeit(lambda: call("sv_gemm_bf16", M, N, K, ptr(Ab), K, ptr(Bb), K, ptr(C), N, None, None, 0.0, ptr(wb), s),
                    args.reps)
        res["sv_bf16_" + name] = [round(us, 1), round(2.0 * M * N * K / us / 1e6, 1)]
        if name == "Gx":  # the bf16 path's K1: bf16 output incl. biases
            Cb = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            us = timeit(lambda: call("sv_gemm_bf16_bf", M, N, K, ptr(Ab), K, ptr(Bb), K, ptr(Cb), N, pb0, pb1, s),
                        args.reps)
            res["sv_bf16_bfout_Gx"] = [round(us, 1), round(2.0 * M * N * K / us / 1e6, 1)]
            if args.check:
                ref = torch.matmul(Ab.float(), Bb.float().t())
                sc = torch.matmul(Ab.float().abs(), Bb.float().abs().t())
                res["sv_bf16_bfout_err_Gx"] = float(((Cb.float() - ref).abs() / sc).max())
                del ref, sc
                Cbf = Cb
            del Cb
        if args.check:
            call("sv_gemm_bf16", M, N, K, ptr(Ab), K, ptr(Bb), K, ptr(C), N, None, None, 0.0, ptr(wb), s)
            torch.cuda.synchronize()
            first = C.clone()
            same = True
            for _ in range(max(args.reps, 8)):
                C.fill_(float("nan"))
                call("sv_gemm_bf16", M, N, K, ptr(Ab), K, ptr(Bb), K, ptr(C), N, None, None, 0.0, ptr(wb), s)
                torch.cuda.synchronize()
                same = same and bool(torch.equal(C, first))
            ref = torch.matmul(Ab.float(), Bb.float().t())
            sc = torch.matmul(Ab.float().abs(), Bb.float().abs().t())
            res["sv_bf16_err_" + name] = float(((first - ref).abs() / sc).max())
            res["sv_bf16_repeat_" + name] = same
            if name == "Gx":  # the bf16-output kernel rounds the same fp32 sums once (RNE)
                res["sv_bf16_bfout_is_rne_of_f32out"] = bool(torch.equal(Cbf, first.bfloat16()))
                del Cbf
            del ref, sc, first
        if args.torch:
            us = timeit(lambda: torch.matmul(Ab, Bb.t()), args.reps)
            res["torch_bf16_" + name] = [round(us, 1), round(2.0 * M * N * K / us / 1e6, 1)]
            try:  # bf16 operands, fp32 output (what our K1/dx/dW write)
                us = timeit(lambda: torch.mm(Ab, Bb.t(), out_dtype=torch.float32), args.reps)
                res["torch_bf16_f32out_" + name] = [round(us, 1), round(2.0 * M * N * K / us / 1e6, 1)]
            except (TypeError, RuntimeError) as e:
                res["torch_bf16_f32out_" + name] = str(e)[:80]
    del A, Bm, C, w
print(json.dumps(res), flush=True)

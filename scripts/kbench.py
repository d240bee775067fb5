"""Per-kernel timing at the c2 shapes (HIP events on the launch stream).  Used for A/B of
kernel variants; prints one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_speaker_verification_amd._lib import call, lib, ptr  # noqa: E402

dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev).cuda_stream
B, T, H, F = 640, 160, 768, 768
G = 4 * H
g = torch.Generator().manual_seed(0)
res = {"variant": os.environ.get("SV_STEP_VARIANT", "default")}


def timeit(fn, reps=50, warm=5):
    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


whh = (torch.randn(G, H, generator=g) * 0.03).to(dev)
hprev = torch.randn(B, H, generator=g).to(dev)
cprev = torch.randn(B, H, generator=g).to(dev)
gates = torch.randn(B, G, generator=g).to(dev)
c_t = torch.empty(B, H, device=dev)
h_t = torch.empty(B, H, device=dev)
us = timeit(lambda: call("sv_lstm_step_fwd", ptr(hprev), ptr(whh), ptr(gates), ptr(cprev), ptr(c_t), ptr(h_t), B, H, s))
res["fwd_step_us"] = round(us, 2)
res["fwd_step_tflops"] = round(2 * B * H * G / us / 1e6, 1)

res["fwd_step_nogemm_us"] = round(timeit(lambda: call("sv_lstm_step_fwd", None, ptr(whh), ptr(gates), ptr(cprev),
                                                       ptr(c_t), ptr(h_t), B, H, s)), 2)
whhT = whh.t().contiguous()
dgn = torch.randn(B, G, generator=g).to(dev) * 0.01
acts = torch.rand(B, G, generator=g).to(dev)
dgo = torch.empty(B, G, device=dev)
dcf0, dcf1 = torch.randn(B, H, generator=g).to(dev), torch.empty(B, H, device=dev)
bw = lambda: call("sv_lstm_step_bwd", ptr(dgn), ptr(whhT), ptr(hprev), ptr(dcf0), ptr(acts), ptr(cprev), ptr(cprev),  # noqa: E731
                  ptr(dgo), ptr(dcf1), B, H, s)
us = timeit(bw)
res["bwd_step_us"] = round(us, 2)
res["bwd_step_tflops"] = round(2 * B * H * G / us / 1e6, 1)
res["bwd_step_nogemm_us"] = round(timeit(lambda: call("sv_lstm_step_bwd", None, ptr(whhT), ptr(hprev), ptr(dcf0),
                                                       ptr(acts), ptr(cprev), ptr(cprev), ptr(dgo), ptr(dcf1), B, H, s)), 2)
# one layer fwd + bwd at T=16 to time the bwd step kernel in place
Ts = 16
x_tm = torch.randn(Ts, B, F, generator=g).to(dev)
w_ih = (torch.randn(G, F, generator=g) * 0.03).to(dev)
b = torch.zeros(G, device=dev)
gts = torch.empty(Ts, B, G, device=dev)
c_tm = torch.empty(Ts, B, H, device=dev)
h_tm = torch.empty(Ts + 1, B, H, device=dev)
hT = torch.empty(H, (Ts + 1) * B, device=dev)
xT = torch.empty(F, Ts * B, device=dev)
call("sv_transpose", ptr(x_tm), F, Ts * B, F, ptr(xT), Ts * B, s)
fwd = lambda: call("sv_lstm_layer_fwd", ptr(x_tm), Ts, B, F, H, ptr(w_ih), ptr(whh), ptr(b), ptr(b), ptr(gts),  # noqa: E731
                   ptr(c_tm), ptr(h_tm), ptr(hT), s)
res["layer_fwd_T16_us"] = round(timeit(fwd, reps=5, warm=1), 1)
dh = torch.randn(Ts, B, H, generator=g).to(dev) * 0.01
dg = torch.empty(Ts, B, G, device=dev)
dgT = torch.empty(G, Ts * B, device=dev)
dx = torch.empty(Ts, B, F, device=dev)
dw_ih, dw_hh = torch.empty(G, F, device=dev), torch.empty(G, H, device=dev)
db1, db2 = torch.empty(G, device=dev), torch.empty(G, device=dev)
ws = torch.empty(lib().sv_lstm_layer_bwd_workspace(Ts, B, F, H) // 4 + 1, device=dev)
bwd = lambda: call("sv_lstm_layer_bwd", Ts, B, F, H, ptr(xT), Ts * B, ptr(w_ih), ptr(whh), ptr(gts), ptr(c_tm),  # noqa: E731
                   ptr(hT), ptr(dh), 1, ptr(dg), ptr(dgT), ptr(dx), ptr(dw_ih), ptr(dw_hh), ptr(db1), ptr(db2), ptr(ws), s)
res["layer_bwd_T16_us"] = round(timeit(bwd, reps=5, warm=1), 1)


def gemm(ak, bk, M, N, K):
    A = torch.randn((M, K) if ak else (K, M), generator=g).to(dev)
    Bm = torch.randn((N, K) if bk else (K, N), generator=g).to(dev)
    C = torch.empty(M, N, device=dev)
    wsz = lib().sv_gemm_f32_workspace(M, N, K)
    w = torch.empty(wsz // 4 + 1, device=dev)
    f = lambda: call("sv_gemm_f32", ak, bk, M, N, K, ptr(A), A.shape[1], ptr(Bm), Bm.shape[1], ptr(C), N, None, None,  # noqa: E731
                     0.0, ptr(w), int(os.environ.get("SV_F32_PRODUCTS", "0")), s)
    us = timeit(f, reps=5, warm=1)
    return round(us, 1), round(2.0 * M * N * K / us / 1e6, 1)


res["gemm_Gx_us_tf"] = gemm(1, 1, T * B, G, H)
res["gemm_dW_us_tf"] = gemm(1, 1, G, H, T * B)
res["gemm_dx_us_tf"] = gemm(1, 1, T * B, H, G)
print(json.dumps(res), flush=True)


def torch_mm(M, N, K, dt):
    A = torch.randn(M, K, device=dev).to(dt)
    Bm = torch.randn(N, K, device=dev).to(dt)
    us = timeit(lambda: torch.matmul(A, Bm.t()), reps=5, warm=2)
    return round(us, 1), round(2.0 * M * N * K / us / 1e6, 1)


ref = {}
for name, (M, N, K) in {"Gx": (T * B, G, H), "dW": (G, H, T * B), "dx": (T * B, H, G)}.items():
    ref["torch_f32_" + name] = torch_mm(M, N, K, torch.float32)
    ref["torch_bf16_" + name] = torch_mm(M, N, K, torch.bfloat16)


def gemm_bf(M, N, K):
    A = torch.randn(M, K, generator=g).bfloat16().to(dev)
    Bm = torch.randn(N, K, generator=g).bfloat16().to(dev)
    C = torch.empty(M, N, device=dev)
    w = torch.empty(lib().sv_gemm_bf16_workspace(M, N, K) // 4 + 1, device=dev)
    f = lambda: call("sv_gemm_bf16", M, N, K, ptr(A), K, ptr(Bm), K, ptr(C), N, None, None, 0.0, ptr(w), s)  # noqa: E731
    us = timeit(f, reps=5, warm=1)
    return round(us, 1), round(2.0 * M * N * K / us / 1e6, 1)


for name, (M, N, K) in {"Gx": (T * B, G, H), "dW": (G, H, T * B), "dx": (T * B, H, G)}.items():
    ref["sv_bf16_" + name] = gemm_bf(M, N, K)
print(json.dumps(ref), flush=True)

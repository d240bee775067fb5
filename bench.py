#!/usr/bin/env python3
"""GE2E training-step benchmark (BASELINE.json metric: embeddings/sec + GE2E steps/sec at
N=64 x M=10, T=160, 40 mels, 3-layer LSTM 768 -> 256).

One "step" = SpeechEmbedder forward + GE2E loss + backward + clip_grad_norm_ (3.0 / 1.0)
+ SGD on one N x M batch per GPU (GE2ETrainer.step, all HIP kernels).  Multi-GPU: one
process per GPU (torchrun), speakers sharded across ranks (global batch = world * N
speakers, exact single-batch semantics via ShardedGE2E), SUM all-reduce of gradients over
RCCL; per-GPU work is fixed, so scaling is weak.

Prints ONE JSON line on rank 0.  value = training embeddings/s of the whole job
(world * N * M * steps / max-over-ranks time).  Extra fields: steps_per_sec,
fwd_embeddings_per_sec (no-grad forward), roofline (dominant kernel, live HIP-event
timing on the kernel's stream), cpu_baseline (the reference path on host cores,
oracle/torch_port.py, rank 0 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MI355X_FP32_MFMA_TFLOPS = 157.3   # /opt/skills/guides/MI355X_MICROARCH.md, chip-level table
MI355X_HBM_GBPS = 8000.0
MI355X_BF16_MFMA_TFLOPS = 2500.0  # dense bf16 MFMA (no sparsity)


def step_flops(B, T, F, H, P, L):
    """Algorithmic FLOPs: fwd = 2BTG[(F+H) + 2(2H)] ... as stated there:
    fwd = sum over layers of 2*B*T*4H*(F_l + H) + 2*B*H*P; step = 3*fwd - 2*B*T*4H*F."""
    G = 4 * H
    fwd = sum(2 * B * T * G * ((F if l == 0 else H) + H) for l in range(L)) + 2 * B * H * P
    return fwd, 3 * fwd - 2 * B * T * G * F


def build_model(dims, dev, seed=0):
    from pytorch_speaker_verification_amd.hparam import hparam as hp
    from pytorch_speaker_verification_amd.speech_embedder_net import GE2ELoss, SpeechEmbedder
    old = (hp.data.nmels, hp.model.hidden, hp.model.num_layer, hp.model.proj)
    hp.data.nmels, hp.model.hidden, hp.model.num_layer, hp.model.proj = dims
    try:
        torch.manual_seed(seed)  # reference init (xavier_normal_ / zero bias / Linear default)
        net = SpeechEmbedder()
    finally:
        hp.data.nmels, hp.model.hidden, hp.model.num_layer, hp.model.proj = old
    return net.to(dev), GE2ELoss(dev)


def time_step_kernel(B, H, dev, reps=64):
    """Average duration of the forward recurrent-step kernel (K2), HIP events on the
    stream it is launched on.  Returns (ms per launch, FLOPs per launch)."""
    from pytorch_speaker_verification_amd._lib import call, ptr, stream_of
    g = torch.Generator(device="cpu").manual_seed(7)
    whh = (torch.randn(4 * H, H, generator=g) * 0.02).to(dev)
    hprev = torch.randn(B, H, generator=g).to(dev)
    cprev = torch.randn(B, H, generator=g).to(dev)
    gates0 = torch.randn(B, 4 * H, generator=g).to(dev)
    gates = gates0.clone()
    c_t = torch.empty(B, H, device=dev)
    h_t = torch.empty(B, H, device=dev)
    s = torch.cuda.current_stream(dev)
    for _ in range(8):
        call("sv_lstm_step_fwd", ptr(hprev), ptr(whh), ptr(gates), ptr(cprev), ptr(c_t), ptr(h_t), B, H, stream_of(gates))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        call("sv_lstm_step_fwd", ptr(hprev), ptr(whh), ptr(gates), ptr(cprev), ptr(c_t), ptr(h_t), B, H, stream_of(gates))
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps, 2.0 * B * H * 4 * H


def time_gemm_kernel(M, N, K, dev, reps=5):
    """Average duration of the dominant kernel by total time, gemm_km_kernel<128,128> at the
    K1 shape of layers 1-2 (x W_ih^T: M = T*B, N = 4H, K = H), HIP events on its stream."""
    from pytorch_speaker_verification_amd._lib import call, ptr, stream_of
    g = torch.Generator(device="cpu").manual_seed(8)
    A = torch.randn(M, K, generator=g).to(dev)
    Bm = (torch.randn(N, K, generator=g) * 0.03).to(dev)
    C = torch.empty(M, N, device=dev)
    s = torch.cuda.current_stream(dev)
    f = lambda: call("sv_gemm_f32", 1, 1, M, N, K, ptr(A), K, ptr(Bm), K, ptr(C), N, None, None, 0.0, None,  # noqa: E731
                     stream_of(C))
    f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        f()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps, 2.0 * M * N * K, 4.0 * (M * K + N * K + M * N)


def pmc_traffic(kernel):
    """HBM bytes per launch from the committed rocprofv3 PMC passes (profiles/), corrected as
    MI355X_MICROARCH.md prescribes: FETCH_SIZE x 2 (gfx950 halves wide streaming reads) +
    WRITE_SIZE, both in KiB."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d[kernel]["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def _timed(f, dev, reps):
    s = torch.cuda.current_stream(dev)
    f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        f()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def hbm_kernels(tr, N, M, D, dev, reps=50):
    """The HBM-bound kernels of the step, HIP events on their stream:
    GE2E fwd+bwd (algorithmic bytes 3*B*D*4: read E twice, write dE) and clip+SGD over the
    flat parameter buffer (read g, read p, write p)."""
    g = torch.Generator(device="cpu").manual_seed(9)
    E = torch.nn.functional.normalize(torch.randn(N, M, D, generator=g), dim=2).to(dev)
    w, b = tr.loss_mod.w, tr.loss_mod.b

    def ge2e():
        _, _, st = tr.ge2e.forward(E, w, b)
        tr.ge2e.backward(st, w, b)
    ms_ge = _timed(ge2e, dev, reps)
    by_ge = 3.0 * N * M * D * 4
    n = tr.n_pad
    pc, gc = tr.flat_p[:n].clone(), tr.flat_g[:n].clone().mul_(1e-3)
    from pytorch_speaker_verification_amd.ops import clip_sgd_step_
    ms_cl = _timed(lambda: clip_sgd_step_(pc, gc, 3.0, 0.0, False), dev, reps)
    by_cl = 3.0 * n * 4
    r = lambda by, ms: round(by / (ms * 1e-3) / 1e9, 1)  # noqa: E731
    return {"ge2e_fwd_bwd": {"avg_us": round(ms_ge * 1e3, 2), "algorithmic_bytes": by_ge,
                             "achieved_GBps": r(by_ge, ms_ge), "peak_GBps": MI355X_HBM_GBPS,
                             "note": "launch-latency bound at this size (SURVEY §8d)"},
            "clip_sgd": {"avg_us": round(ms_cl * 1e3, 2), "algorithmic_bytes": by_cl,
                         "achieved_GBps": r(by_cl, ms_cl), "peak_GBps": MI355X_HBM_GBPS}}


def _ge2e_torch(E, w, b):
    """Plain torch GE2E loss (vectorised, autograd) for the vendor-library baseline."""
    N, M, D = E.shape
    C = E.mean(1)
    U = (E.sum(1, keepdim=True) - E) / (M - 1)
    nrm = lambda v: v / v.norm(dim=-1, keepdim=True).clamp_min(1e-8)  # noqa: E731
    En = nrm(E)
    cos = torch.einsum("nmd,kd->nmk", En, nrm(C))
    diag = (En * nrm(U)).sum(2)
    eye = torch.eye(N, device=E.device, dtype=torch.bool).unsqueeze(1)
    cos = torch.where(eye, diag.unsqueeze(2), cos) + 1e-6
    S = w * cos + b
    pos = S.diagonal(dim1=0, dim2=2).transpose(0, 1)
    return (torch.log(torch.exp(S).sum(2) + 1e-6) - pos).sum()


def vendor_baseline(dims, N, M, T, dev, steps=3, dtype="f32"):
    """Stock torch-ROCm on the same GPU: nn.LSTM (MIOpen RNN) + Linear + torch GE2E, autograd,
    clip_grad_norm_ x2, SGD -- the reference's training step run by the vendor libraries.
    dtype bf16: the LSTM and projection run entirely in bf16 (weights, states and gradients;
    a lower precision than this repo's bf16 path, which keeps cell state and gradients fp32)."""
    F, H, L, P = dims
    try:
        torch.manual_seed(0)
        wdt = torch.bfloat16 if dtype == "bf16" else torch.float32
        lstm = torch.nn.LSTM(F, H, num_layers=L, batch_first=True).to(dev, wdt)
        proj = torch.nn.Linear(H, P).to(dev, wdt)
        w = torch.nn.Parameter(torch.tensor(10.0, device=dev))
        b = torch.nn.Parameter(torch.tensor(-5.0, device=dev))
        net_params = list(lstm.parameters()) + list(proj.parameters())
        opt = torch.optim.SGD([{"params": net_params}, {"params": [w, b]}], lr=0.01)
        g = torch.Generator(device="cpu").manual_seed(1235)
        x = torch.randn(N * M, T, F, generator=g).to(dev, wdt)

        def step():
            opt.zero_grad()
            y, _ = lstm(x)
            e = proj(y[:, -1]).float()
            e = e / e.norm(dim=1, keepdim=True)
            loss = _ge2e_torch(e.view(N, M, P), w, b)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(net_params, 3.0)
            torch.nn.utils.clip_grad_norm_([w, b], 1.0)
            opt.step()
            return loss
        step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        return {"value": round(N * M / dt, 3), "unit": "embeddings/s", "ms_per_step": round(dt * 1e3, 3),
                "kind": f"torch-rocm nn.LSTM (MIOpen) + autograd, {dtype}, same GPU",
                "torch": torch.__version__}
    except Exception as ex:  # report, never fail the bench on the vendor leg
        return {"error": f"{type(ex).__name__}: {ex}"[:300]}


def f32_product_accuracy(dev, M=512, N=1024, K=768):
    """Max error of one fp32 GEMM (K1 shape family) against fp64, per product mode, relative to
    |A||B|^T -- the accuracy evidence for the bf16x6 mode."""
    from pytorch_speaker_verification_amd._lib import call, ptr, stream_of
    from pytorch_speaker_verification_amd.ops import set_f32_products
    g = np.random.default_rng(11)
    A = g.standard_normal((M, K)).astype(np.float32)
    B = g.standard_normal((N, K)).astype(np.float32)
    ref = A.astype(np.float64) @ B.astype(np.float64).T
    scale = np.abs(A).astype(np.float64) @ np.abs(B).astype(np.float64).T
    At, Bt = torch.tensor(A, device=dev), torch.tensor(B, device=dev)
    out = {}
    for mode in ("mfma_f32", "bf16x6"):
        prev = set_f32_products(mode)
        C = torch.empty(M, N, device=dev)
        call("sv_gemm_f32", 1, 1, M, N, K, ptr(At), K, ptr(Bt), K, ptr(C), N, None, None, 0.0, None, 0, stream_of(C))
        err = np.abs(C.cpu().numpy().astype(np.float64) - ref) / scale
        out[mode] = {"max": float(err.max()), "mean": float(err.mean())}
        set_f32_products(prev)
    return out


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(dims, N, M, T, seconds_budget=25.0):
    """The reference's CPU path (stock PyTorch port, oracle/torch_port.py) on host cores,
    one full training step of the same workload (bounded sample)."""
    from oracle import torch_port
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    net = torch_port.SpeechEmbedderPort(*dims)
    w = torch.nn.Parameter(torch.tensor(10.0))
    b = torch.nn.Parameter(torch.tensor(-5.0))
    opt = torch.optim.SGD([{"params": net.parameters()}, {"params": [w, b]}], lr=0.01)
    g = torch.Generator().manual_seed(1235)
    # warm oneDNN on a small batch first
    xw = torch.randn(4 * 2, 16, dims[0], generator=g)
    torch_port.train_step(net, w, b, opt, xw, 4, 2)
    x = torch.randn(N * M, T, dims[0], generator=g)
    t0 = time.perf_counter()
    torch_port.train_step(net, w, b, opt, x, N, M)
    dt = time.perf_counter() - t0
    return {"value": round(N * M / dt, 3), "unit": "embeddings/s", "cores": threads, "kind": "port",
            "cpu_model": _cpu_model(),
            "steps_per_sec": round(1.0 / dt, 5), "sec_per_step": round(dt, 3),
            "sample": f"1 full training step (fwd+GE2E+bwd+clip+SGD) of N={N}xM={M}, T={T}, fp32, "
                      f"oracle/torch_port.py (nn.LSTM on oneDNN), {threads} threads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--N", type=int, default=64)
    ap.add_argument("--M", type=int, default=10)
    ap.add_argument("--T", type=int, default=160)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--fwd-steps", type=int, default=5)
    ap.add_argument("--no-bf16", action="store_true", help="skip the config-c3 (bf16 operands) side measurement")
    ap.add_argument("--no-f32x", action="store_true", help="skip the fp32-via-bf16x6 side measurement")
    ap.add_argument("--preset", choices=["c2", "c3", "c5"], default=None,
                    help="BASELINE config per GPU: c2 = N64 M10 T160 f32, c3 = the same in bf16, "
                         "c5 = N256/8 GPUs -> 32 speakers per GPU, M10, T180, bf16")
    ap.add_argument("--no-vendor", action="store_true", help="skip the nn.LSTM/MIOpen same-GPU baseline")
    ap.add_argument("--dtype", choices=["f32", "bf16"], default="f32",
                    help="precision of the headline line (default f32 = BASELINE configs[1]; bf16 = configs[2])")
    args = ap.parse_args()
    if args.preset == "c3":
        args.dtype = "bf16"
    elif args.preset == "c5":
        args.N, args.M, args.T, args.dtype = 32, 10, 180, "bf16"

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from pytorch_speaker_verification_amd.ops import embedder_forward, embedder_forward_bf16
    from pytorch_speaker_verification_amd.trainer import GE2ETrainer

    dims = (40, 768, 3, 256)
    N, M, T = args.N, args.M, args.T
    B = N * M
    net, ge2e = build_model(dims, dev)
    net.precision = args.dtype
    tr = GE2ETrainer(net, ge2e, lr=0.01)
    g = torch.Generator(device="cpu").manual_seed(1234 + 1 + rank)   # SURVEY §8d seed 1234 + config index
    x = torch.randn(B, T, dims[0], generator=g).to(dev)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        tr.step(x, N, M)
    barrier()
    t0 = time.perf_counter()
    host_s = 0.0
    for _ in range(args.steps):
        th = time.perf_counter()
        loss = tr.step(x, N, M)
        host_s += time.perf_counter() - th
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)
    final_loss = float(loss)

    # forward-only (inference) embeddings/s
    layers = net.LSTM_stack.layer_params()
    fwd_fn = embedder_forward_bf16 if args.dtype == "bf16" else embedder_forward
    with torch.no_grad():
        for _ in range(2):
            fwd_fn(x, layers, net.projection.weight, net.projection.bias, save=False)
        barrier()
        tf0 = time.perf_counter()
        for _ in range(args.fwd_steps):
            fwd_fn(x, layers, net.projection.weight, net.projection.bias, save=False)
        barrier()
        tf = (time.perf_counter() - tf0) / args.fwd_steps

    fwd_fl, st_fl = step_flops(B, T, dims[0], dims[1], dims[3], dims[2])
    ms_step = dt / args.steps * 1e3
    out = {
        "metric": "embeddings/sec + GE2E steps/sec at N=64×M=10, 1/2/4/8 MI355X",
        "value": round(world * B * args.steps / dt, 3),
        "unit": "embeddings/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic x~N(0,1) frames, reference init (torch.manual_seed(0))",
        "config": {"workload": f"GE2E train step N={N}xM={M} per GPU, T={T}, 40 mels, LSTM 3x768, proj 256",
                   "global_batch": world * B, "speakers_global": world * N, "seq_len": T,
                   "parallelism": f"dp{world} (speaker-sharded GE2E, RCCL grad all-reduce)"},
        "steps_per_sec": round(args.steps / dt, 4),
        "host_enqueue_ms_per_step": round(host_s / args.steps * 1e3, 3),
        "fwd_embeddings_per_sec": round(world * B / tf, 1),
        "loss": round(final_loss, 5),
        "step_tflops": round(st_fl / (ms_step * 1e-3) / 1e12, 2),
        "step_mfma_frac": round(st_fl / (ms_step * 1e-3) / 1e12 /
                                (MI355X_FP32_MFMA_TFLOPS if args.dtype == "f32" else MI355X_BF16_MFMA_TFLOPS), 4),
    }
    if not args.no_f32x and args.dtype == "f32":
        # the same fp32 step with bf16x6 products (opt-in mode; exact-fp32 MFMA is the headline)
        from pytorch_speaker_verification_amd.ops import set_f32_products
        prev = set_f32_products("bf16x6")
        try:
            netx, gex = build_model(dims, dev)
            trx = GE2ETrainer(netx, gex, lr=0.01)
            for _ in range(args.warmup):
                trx.step(x, N, M)
            barrier()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                lx = trx.step(x, N, M)
            barrier()
            dx_ = time.perf_counter() - t0
            if world > 1:
                t = torch.tensor([dx_], device=dev, dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                dx_ = float(t)
        finally:
            set_f32_products(prev)
        msx = dx_ / args.steps * 1e3
        out["f32_bf16x6"] = {"config": "same workload, fp32 products formed as six bf16 MFMA products of a three-way "
                                       "bf16 split (fp32 accumulation); opt-in via set_f32_products('bf16x6')",
                             "value": round(world * B * args.steps / dx_, 3), "unit": "embeddings/s",
                             "ms_per_step": round(msx, 3), "loss": round(float(lx), 5)}
        if rank == 0:
            out["f32_bf16x6"]["gemm_error_vs_fp64"] = f32_product_accuracy(dev)
    if not args.no_bf16 and args.dtype == "f32":
        # BASELINE config c3: same workload, bf16 GEMM operands (fp32 accumulate/state/loss)
        net16, ge16 = build_model(dims, dev)
        net16.precision = "bf16"
        tr16 = GE2ETrainer(net16, ge16, lr=0.01)
        for _ in range(args.warmup):
            tr16.step(x, N, M)
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            l16 = tr16.step(x, N, M)
        barrier()
        d16 = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([d16], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            d16 = float(t)
        ms16 = d16 / args.steps * 1e3
        out["bf16"] = {"config": "c3: same workload, bf16 GEMM operands, fp32 accumulate/state/loss",
                       "value": round(world * B * args.steps / d16, 3), "unit": "embeddings/s",
                       "ms_per_step": round(ms16, 3), "steps_per_sec": round(args.steps / d16, 4),
                       "loss": round(float(l16), 5),
                       "step_tflops": round(st_fl / (ms16 * 1e-3) / 1e12, 2),
                       "step_mfma_frac": round(st_fl / (ms16 * 1e-3) / 1e12 / MI355X_BF16_MFMA_TFLOPS, 4)}
    if rank == 0:
        H = dims[1]
        ms_g, fl_g, by_g = time_gemm_kernel(T * B, 4 * H, H, dev)
        ach = fl_g / (ms_g * 1e-3) / 1e12
        out["roofline"] = {"kernel": "gemm_km_kernel<128,128> (K1/dW/dx NT GEMM, fp32 MFMA 32x32x2), K1 shape "
                                     f"M={T * B} N={4 * H} K={H}",
                           "bound": "mfma", "achieved": round(ach, 2), "peak": MI355X_FP32_MFMA_TFLOPS,
                           "unit": "TFLOP/s", "frac": round(ach / MI355X_FP32_MFMA_TFLOPS, 4),
                           "traffic": pmc_traffic("gemm_km_kernel<128,128>"), "algorithmic_bytes": by_g,
                           "avg_launch_us": round(ms_g * 1e3, 2), "flops_per_launch": fl_g}
        ms_k, fl_k = time_step_kernel(B, H, dev)
        ach_k = fl_k / (ms_k * 1e-3) / 1e12
        out["roofline_step_kernel"] = {"kernel": "lstm_step_fwd_v2_kernel (K2, fp32 MFMA 32x32x2)", "bound": "mfma",
                                       "achieved": round(ach_k, 2), "peak": MI355X_FP32_MFMA_TFLOPS,
                                       "unit": "TFLOP/s", "frac": round(ach_k / MI355X_FP32_MFMA_TFLOPS, 4),
                                       "traffic": pmc_traffic("lstm_step_fwd_v2_kernel"),
                                       "avg_launch_us": round(ms_k * 1e3, 2), "flops_per_launch": fl_k}
        if world == 1:  # (the GE2E leg would issue collectives on rank 0 alone otherwise)
            out["hbm_kernels"] = hbm_kernels(tr, N, M, dims[3], dev)
        if not args.no_vendor and world == 1:
            out["vendor_baseline"] = vendor_baseline(dims, N, M, T, dev, dtype=args.dtype)
            if "bf16" in out:
                out["bf16"]["vendor_baseline"] = vendor_baseline(dims, N, M, T, dev, dtype="bf16")
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(dims, N, M, T)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

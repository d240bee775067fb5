#!/usr/bin/env python3
"""GE2E training-step benchmark (BASELINE.json metric: embeddings/sec + GE2E steps/sec at
N=64 x M=10, T=160, 40 mels, 3-layer LSTM 768 -> 256, at 1/2/4/8 MI355X).

One "step" = SpeechEmbedder forward + GE2E loss + backward + clip_grad_norm_ (3.0 / 1.0)
+ SGD on one N x M batch (GE2ETrainer.step, all HIP kernels), inputs already in HBM.

Multi-GPU: one process per GPU.  ``python bench.py --gpus N`` launches the N ranks itself
(torch.distributed.run, 127.0.0.1) before this process touches the GPU; under an external
launcher (WORLD_SIZE set) it runs as one rank.  Speakers are sharded across ranks (exact
single-batch semantics via ShardedGE2E), gradients SUM-all-reduced over RCCL.

Headline line (rank 0 prints ONE JSON line): config c2 (fp32, the reference's precision) with
N = 64 speakers PER GPU -> weak scaling; value = world * N * M * steps / max-over-ranks time.
Side measurements in the same line:
  bf16            c3: the same per-GPU workload with bf16 GEMM operands (weak scaling)
  c4              (world > 1) c3's global batch N = 64 x M = 10 split over the ranks, bf16:
                  strong scaling, value = 640 * steps / time
  c5              (world > 1) N = 256 x M = 10, T = 180 split over the ranks, bf16 (strong)
  c4_rank_shape / c5_rank_shape   (world = 1) one rank's share of c4 / c5 at 8 GPUs, alone
  roofline        the worst-fraction in-step kernel of the headline step: at c2 the persistent
                  fp32 backward recurrence (lstm_persist_bwd_f32_h2_kernel; the per-step
                  schedule: K3), timed by HIP event pairs on its stream INSIDE the timed steps
  roofline_bf16   the same for c3's dominant kernels, the persistent bf16 recurrences
  roofline_gemm / roofline_step_kernel   secondary: the K1-shape fp32 GEMM and K2 in isolation
  roofline_dw_gemm  the fp32 dW GEMM (the c2 step's largest kernel by busy time) in isolation
  dropin_loop     the reference's own loop body (train_speech_embedder.py:46-65) run unchanged on
                  the dropin/ modules (autograd + torch clip + torch SGD), beside the fused trainer
  cpu_baseline    the reference's CPU path (oracle/torch_port.py, nn.LSTM on oneDNN) on every
                  host CPU this process may use, median of 3 steps at c2, plus c1
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
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
METRIC = "embeddings/sec + GE2E steps/sec at N=64×M=10, 1/2/4/8 MI355X"
SIDE_STEPS = 40  # timed steps of each side line at least (the headline times exactly --steps)
DIMS = (40, 768, 3, 256)          # nmels, hidden, layers, proj (config/config.yaml)


def step_flops(B, T, F, H, P, L):
    """Algorithmic FLOPs: fwd = sum over layers of 2*B*T*4H*(F_l + H) + 2*B*H*P;
    step = 3*fwd - 2*B*T*4H*F."""
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


class Ctx:
    def __init__(self, world, rank, dev):
        self.world, self.rank, self.dev = world, rank, dev

    def barrier(self):
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(self, v):
        if self.world == 1:
            return v
        t = torch.tensor([v], device=self.dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t)


_T0 = time.perf_counter()


def log(msg):
    """Progress to stderr (rank 0), so a long run is visibly alive."""
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench {time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def _events(n):
    """Timing events with their native HIP event materialised (torch creates it lazily, at the
    first record; the C ABI records them itself)."""
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(n)]
    for e in evs:
        e.record()
    return evs


def run_steps(ctx, N, M, T, precision, steps, warmup, seed, probe=None, products="mfma_f32"):
    """Time `steps` fused training steps of this rank's N x M batch.  probe = None, "fwd_bwd"
    (bf16: events around each layer's persistent recurrences) or "bwd_chunks" (fp32: events
    around one K3 launch per chunk).  Returns (max-over-ranks seconds, loss, host enqueue s,
    per-step probe event lists, trainer)."""
    from pytorch_speaker_verification_amd.ops import PIPELINE_CHUNK
    from pytorch_speaker_verification_amd.trainer import GE2ETrainer
    log(f"run N={N} M={M} T={T} {precision} {products} steps={steps} warmup={warmup}")
    net, ge2e = build_model(DIMS, ctx.dev)
    net.precision = precision
    net.f32_products = products
    tr = GE2ETrainer(net, ge2e, lr=0.01)
    g = torch.Generator(device="cpu").manual_seed(seed + ctx.rank)
    x = torch.randn(N * M, T, DIMS[0], generator=g).to(ctx.dev)
    for _ in range(warmup):
        tr.step(x, N, M)
    L = DIMS[2]
    nch = (T + PIPELINE_CHUNK - 1) // PIPELINE_CHUNK
    probes = []
    for _ in range(steps if probe else 0):
        if probe == "fwd_bwd":
            probes.append({"fwd": _events(2 * L), "bwd": _events(2 * L)})
        else:  # fp32: events + the kernel's own real-time stamps around one K3 launch per chunk
            ks = torch.zeros(2 * L * T, dtype=torch.int64, device=ctx.dev)
            ks[0::2] = -1  # (UINT64_MAX, 0) pairs: atomic min / max targets
            probes.append({"bwd": _events(2 * L * nch), "kstamp": ks})
    ctx.barrier()
    t0 = time.perf_counter()
    host = 0.0
    for k in range(steps):
        th = time.perf_counter()
        loss = tr.step(x, N, M, probe=probes[k] if probe else None)
        host += time.perf_counter() - th
    ctx.barrier()
    dt = ctx.max_over_ranks(time.perf_counter() - t0)
    tr.check()  # raises if a persistent recurrence timed out during the timed steps
    log(f"  {dt / steps * 1e3:.3f} ms/step")
    return dt, float(loss), host, probes, tr


def kstamp_us(probes):
    """Average execution span (us) of the timed steps' K3 launches from the kernels' own real-time
    stamps (100 MHz GPU clock, first-workgroup start to last-workgroup end)."""
    spans = []
    for p in probes:
        ks = p["kstamp"].cpu().view(-1, 2)
        spans += [int(e - s_) / 100.0 for s_, e in ks.tolist() if e > 0]
    return sum(spans) / max(1, len(spans)), len(spans)


def probe_ms(probes, key):
    """Sum over the (before, after) event pairs of one step's probe list, averaged over steps."""
    tot = 0.0
    for p in probes:
        ev = p[key]
        for i in range(len(ev) // 2):
            try:   # a schedule that runs all layers in one launch records only the first pair
                tot += ev[2 * i].elapsed_time(ev[2 * i + 1])
            except RuntimeError:
                pass
    return tot / max(1, len(probes))


def persist_kernels(B, H=768, cus=256):
    """(bwd, fwd) names of the per-layer persistent bf16 recurrence kernels the library picks for
    the upper layers at batch B (sv_persist.hip: the wide 32 x 64 tile where the 32-unit tile would
    need 64-row blocks)."""
    wide = H == 768 and (B + 31) // 32 * (H // 32) > cus and (B + 31) // 32 * (H // 64) <= cus
    bwd = "lstm_persist3_bwd_bf16_kernel" if wide else "lstm_persist2_bwd_bf16_kernel"
    fwd = "lstm_persist3_fwd_bf16_kernel" if wide else "lstm_persist2_fwd_bf16_kernel"
    return bwd, fwd


def bf16_recurrences(B, T):
    """What the bf16 trainer step runs for its recurrences at batch B under schedule 'auto', and
    how its probe events must be read.  The trainer probes only the first row chunk
    (trainer.bf16_row_chunks: equal persistent chunks past 672 rows, two wavefront halves up to
    192), so the FLOPs are that chunk's.  Returns dict(kind, bwd, fwd, launches (per direction per
    step), fwd_flops / bwd_flops (per launch), rows)."""
    from pytorch_speaker_verification_amd._lib import lib
    from pytorch_speaker_verification_amd.trainer import bf16_row_chunks
    F, H, L, _ = DIMS
    r0, r1 = bf16_row_chunks(B, H, "auto", L, T, F)[0]
    b = r1 - r0
    G = 4 * H
    if lib().sv_wave_ok(L, T, b, F, H):
        # one launch for all layers: the forward contracts every layer's input and recurrent
        # operands, the backward every layer's dh_rec and the upper layers' dx
        return {"kind": "wave", "bwd": "lstm_wave_bwd_bf16_kernel", "fwd": "lstm_wave3_fwd_bf16_kernel",
                "launches": 1, "rows": b,
                "fwd_flops": float(sum(2 * b * T * G * ((F if l == 0 else H) + H) for l in range(L))),
                "bwd_flops": float(2 * b * T * G * H * (2 * L - 1))}
    kb, kf = persist_kernels(b, H)
    fl = float(2 * b * T * H * G)
    return {"kind": "persist", "bwd": kb, "fwd": kf, "launches": L, "rows": b, "fwd_flops": fl, "bwd_flops": fl}


def pmc_traffic(kernel):
    """HBM bytes per launch from the committed rocprofv3 PMC passes (bench_pmc_traffic.json at the
    repo root: profiles/ does not travel to the GPU box), corrected as MI355X_MICROARCH.md
    prescribes (FETCH_SIZE x 2 + WRITE_SIZE, both KiB)."""
    try:
        with open(os.path.join(ROOT, "bench_pmc_traffic.json")) as f:
            return json.load(f)[kernel]["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


def _timed(f, dev, reps, warm=3):
    """Average ms per call of f over `reps` calls, HIP events on the current stream, after `warm`
    untimed calls (first launches pay code-object load and cold caches)."""
    s = torch.cuda.current_stream(dev)
    for _ in range(warm):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        f()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def time_step_kernel(B, H, dev, reps=64):
    """K2 (fp32 forward recurrent step) in isolation, HIP events on its stream."""
    from pytorch_speaker_verification_amd._lib import call, ptr, stream_of
    g = torch.Generator(device="cpu").manual_seed(7)
    whh = (torch.randn(4 * H, H, generator=g) * 0.02).to(dev)
    hprev, cprev = torch.randn(B, H, generator=g).to(dev), torch.randn(B, H, generator=g).to(dev)
    gates = torch.randn(B, 4 * H, generator=g).to(dev)
    c_t, h_t = torch.empty(B, H, device=dev), torch.empty(B, H, device=dev)
    f = lambda: call("sv_lstm_step_fwd", ptr(hprev), ptr(whh), ptr(gates), ptr(cprev), ptr(c_t), ptr(h_t), B, H,  # noqa
                     stream_of(gates))
    return _timed(f, dev, reps), 2.0 * B * H * 4 * H


def time_gemm_kernel(M, N, K, dev, reps=5):
    """The fp32 NT GEMM (sv_gemm_f32: gemm_f32_256_kernel, the 256 x 256 LDS-DMA tile, at this shape)
    at the K1 shape of layers 1-2 in isolation, HIP events on its stream."""
    from pytorch_speaker_verification_amd._lib import call, ptr, stream_of
    g = torch.Generator(device="cpu").manual_seed(8)
    A = torch.randn(M, K, generator=g).to(dev)
    Bm = (torch.randn(N, K, generator=g) * 0.03).to(dev)
    C = torch.empty(M, N, device=dev)
    f = lambda: call("sv_gemm_f32", 1, 1, M, N, K, ptr(A), K, ptr(Bm), K, ptr(C), N, None, None, 0.0, None, 0,  # noqa
                     stream_of(C))
    return _timed(f, dev, reps), 2.0 * M * N * K, 4.0 * (M * K + N * K + M * N)


def time_dw_gemm(T, B, H, dev, reps=5):
    """The fp32 weight-gradient GEMM of the persistent backward (dW_hh = dG^T h: M = 4H, N = H,
    K = T * B, split-K slabs; gemm_f32_256_kernel through sv_gemm_f32 with both operands
    k-contiguous, as sv_lstm_stack_bwd calls it) in isolation: by busy time the c2 step's largest
    kernel (3 launches of it and 3 of dW_ih per step)."""
    from pytorch_speaker_verification_amd._lib import call, lib, ptr, stream_of
    g = torch.Generator(device="cpu").manual_seed(10)
    K = T * B
    A = (torch.randn(4 * H, K, generator=g) * 0.01).to(dev)
    Bm = torch.randn(H, K, generator=g).to(dev)
    C = torch.empty(4 * H, H, device=dev)
    ws = torch.empty(int(lib().sv_gemm_f32_workspace(4 * H, H, K)) // 4 + 1, device=dev)
    f = lambda: call("sv_gemm_f32", 1, 1, 4 * H, H, K, ptr(A), K, ptr(Bm), K, ptr(C), H, None, None, 0.0,  # noqa
                     ptr(ws), 0, stream_of(C))
    return _timed(f, dev, reps), 2.0 * 4 * H * H * K, 4.0 * (4 * H * K + H * K + 4 * H * H)


def user_train_step(net, loss_fn, opt, frames, n_spk, n_utt, gen=None):
    """One step of a user-written GE2E loop over nn.Module objects, the shape of the loop
    train_speech_embedder.py:46-65 runs (there: reshape, a shuffled row order around the forward,
    zero_grad, forward, GE2E loss, backward, clip_grad_norm_ 3.0 / 1.0, SGD step).  Written here
    with torch primitives: the row shuffle is ``torch.randperm`` and its inverse ``argsort``.
    Whatever modules it is handed (this package's through dropin/, or the stock-PyTorch port) run
    through autograd, torch's clip_grad_norm_ and the optimizer, nothing fused."""
    rows = n_spk * n_utt
    flat = frames.flatten(0, 1)                                   # [N*M, T, F]
    order = torch.randperm(rows, generator=gen).to(flat.device)
    back = torch.argsort(order)                                   # order[back] == arange
    opt.zero_grad()
    emb = net(flat.index_select(0, order)).index_select(0, back)
    loss = loss_fn(emb.view(n_spk, n_utt, -1))
    loss.backward()
    for group, max_norm in zip(opt.param_groups, (3.0, 1.0)):
        torch.nn.utils.clip_grad_norm_(group["params"], max_norm)
    opt.step()
    return loss


def dropin_loop(ctx, N, M, T, steps, warmup, precision="f32"):
    """ms per step of a user-written loop (user_train_step) on this package's
    modules imported the reference's way (dropin/: `from speech_embedder_net import ...`), the
    same synthetic batch as the headline, beside the fused GE2ETrainer."""
    if os.path.join(ROOT, "dropin") not in sys.path:
        sys.path.append(os.path.join(ROOT, "dropin"))
    from speech_embedder_net import GE2ELoss, SpeechEmbedder  # noqa: E402  (dropin/ shim)
    torch.manual_seed(0)
    net = SpeechEmbedder().to(ctx.dev)
    net.precision = precision
    ge2e = GE2ELoss(ctx.dev)
    opt = torch.optim.SGD([{"params": net.parameters()}, {"params": ge2e.parameters()}], lr=0.01)
    g = torch.Generator(device="cpu").manual_seed(1235 + ctx.rank)
    x = torch.randn(N, M, T, DIMS[0], generator=g).to(ctx.dev)
    gen = torch.Generator().manual_seed(0)
    for _ in range(warmup):
        user_train_step(net, ge2e, opt, x, N, M, gen)
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = user_train_step(net, ge2e, opt, x, N, M, gen)
    ctx.barrier()
    dt = ctx.max_over_ranks(time.perf_counter() - t0)
    return {"config": f"user-written loop of train_speech_embedder.py:46-65's shape on dropin/ modules (autograd forward / "
                      f"backward, torch clip_grad_norm_ x2, torch SGD), N={N}xM={M}, T={T}, {precision}",
            "ms_per_step": round(dt / steps * 1e3, 3), "value": round(N * M * ctx.world * steps / dt, 3),
            "unit": "embeddings/s", "loss": round(float(loss.detach()), 5)}


def hbm_kernels(tr, N, M, D, dev, reps=50):
    """The HBM-bound kernels of the step: GE2E fwd+bwd (algorithmic bytes 3*B*D*4)
    and clip+SGD over the flat parameter buffer (read g, read p, write p)."""
    from pytorch_speaker_verification_amd.ops import clip_sgd_step_
    g = torch.Generator(device="cpu").manual_seed(9)
    E = torch.nn.functional.normalize(torch.randn(N, M, D, generator=g), dim=2).to(dev)
    w, b = tr.loss_mod.w, tr.loss_mod.b

    def ge2e():  # the trainer's GE2E (fused 3-launch kernel on one GPU)
        tr.ge2e.train(E, w, b)

    def ge2e_split():
        _, _, st = tr.ge2e.forward(E, w, b)
        tr.ge2e.backward(st, w, b)
    ms_ge = _timed(ge2e, dev, reps)
    ms_split = _timed(ge2e_split, dev, reps)
    # the same 3 launches captured once in a HIP graph and replayed: the device-side time
    # without the per-call host path (ctypes + argument marshalling) that bounds the eager loop
    graph_us = None
    try:
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            ge2e()
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize(dev)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            ge2e()
        graph_us = round(_timed(gr.replay, dev, reps) * 1e3, 2)
    except Exception as ex:  # capture is a measurement aid only: report why it is absent
        graph_us = f"capture failed: {type(ex).__name__}"
    by_ge = 3.0 * N * M * D * 4
    n = tr.n_pad
    pc, gc = tr.flat_p[:n].clone(), tr.flat_g[:n].clone().mul_(1e-3)
    ms_cl = _timed(lambda: clip_sgd_step_(pc, gc, 3.0, 0.0, False), dev, reps)
    by_cl = 3.0 * n * 4
    r = lambda by, ms: round(by / (ms * 1e-3) / 1e9, 1)  # noqa: E731
    return {"ge2e_fwd_bwd": {"avg_us": round(ms_ge * 1e3, 2), "algorithmic_bytes": by_ge,
                             "achieved_GBps": r(by_ge, ms_ge), "peak_GBps": MI355X_HBM_GBPS,
                             "split_path_us": round(ms_split * 1e3, 2), "hip_graph_replay_us": graph_us,
                             "note": "fused 3-launch kernel (sv_ge2e_train); avg_us: the trainer's eager per-call loop, "
                                     "hip_graph_replay_us: the same launches replayed from a HIP graph (adds the "
                                     "graph launch); launch- and L2-latency bound at this size"},
            "clip_sgd": {"avg_us": round(ms_cl * 1e3, 2), "algorithmic_bytes": by_cl,
                         "achieved_GBps": r(by_cl, ms_cl), "peak_GBps": MI355X_HBM_GBPS}}


def c5_rank_ge2e(dev, world=8, reps=50):
    """The GE2E of one c5 rank at 8 GPUs as ShardedGE2E.train runs it (sharded_ge2e.py): this
    rank's N_local = 32 speakers x M = 10 against all N = 256 centroids, the last rank (speaker
    offset s0 = 224), the fused sharded kernels (sv_ge2e_shard_prep / _rows / _finalize) with the
    two exchanges left out (the all-gathered sums and the all-reduced buffer are synthetic); the
    split kernels of the same shard beside it."""
    from pytorch_speaker_verification_amd.sharded_ge2e import HipFusedShard, HipShardKernels
    N, M, D = 256, 10, 256
    Nl = N // world
    s0 = N - Nl
    g = torch.Generator(device="cpu").manual_seed(25)
    E = torch.nn.functional.normalize(torch.randn(Nl, M, D, generator=g), dim=2).to(dev)
    others = torch.nn.functional.normalize(torch.randn(N, M, D, generator=g), dim=2).sum(1).to(dev)
    w = torch.tensor(10.0, device=dev)
    b = torch.tensor(-5.0, device=dev)
    f = HipFusedShard()
    assert f.ok(N, M, D)
    ssum_local, ws = f.prep(E, N)
    ssum_all = others.clone()
    ssum_all[s0:] = ssum_local

    def fused():
        sl, wsp = f.prep(E, N)
        _, _, red, _ = f.rows(E, s0, N, ssum_all, w, b, wsp)
        f.finalize(E, s0, N, red, wsp)
    k = HipShardKernels()

    def split():
        k.speaker_sums(E)
        _, _, st = k.fwd_rows(E, s0, N, ssum_all, w, b)
        red, _ = k.bwd_rows(st, w, b, None)
        k.finalize(st, red)
    ms_f = _timed(fused, dev, reps)
    ms_s = _timed(split, dev, reps)

    def replay_us(f):  # the same launches captured once in a HIP graph: device time without the host path
        try:
            st = torch.cuda.Stream(dev)
            st.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(st):
                f()
            torch.cuda.current_stream(dev).wait_stream(st)
            torch.cuda.synchronize(dev)
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                f()
            return round(_timed(gr.replay, dev, reps) * 1e3, 2)
        except Exception as ex:  # a measurement aid only: report why it is absent
            return f"capture failed: {type(ex).__name__}"
    by = 3.0 * Nl * M * D * 4
    return {"workload": f"one c5 rank's GE2E at {world} GPUs: N_local={Nl}xM={M} rows against N={N} centroids, "
                        f"s0={s0}, D={D} (exchanges excluded)",
            "fused_us": round(ms_f * 1e3, 2), "split_us": round(ms_s * 1e3, 2),
            "fused_graph_replay_us": replay_us(fused), "split_graph_replay_us": replay_us(split),
            "algorithmic_bytes": by,
            "note": "fused: sv_ge2e_shard_prep + _rows (centroids of all 256 speakers in two fp32 LDS tiles) + "
                    "_finalize; split: the sv_ge2e_speaker_sums / fwd_rows / bwd_rows / bwd_finalize kernels; "
                    "*_us: eager per-call loop (host path included: tensor allocation and ctypes calls), "
                    "*_graph_replay_us: the same launches replayed from a HIP graph"}


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



def dvector_inference(net, dev, S=16384, T=24, reps=3):
    """d-vector extraction (dvector_create.py:96-101): S windows of T = 24 frames
    (240 ms at a 10 ms hop) embedded by the trained net, no autograd state (dvector.embed_windows,
    fp32 MFMA path), windows already in HBM; MIOpen nn.LSTM + Linear on the same windows beside it."""
    from pytorch_speaker_verification_amd.dvector import GraphedEmbedder, embed_windows
    F, H, L, P = DIMS
    g = torch.Generator(device="cpu").manual_seed(24)
    xw = torch.randn(S, T, F, generator=g).to(dev)
    flops = sum(2.0 * S * T * 4 * H * ((F if l == 0 else H) + H) for l in range(L)) + 2.0 * S * H * P

    def ours():
        return embed_windows(net, xw, batch=S)
    res = {"workload": f"{S} windows x T={T} x {F} mel, fp32 (dvector_create.py:96-101)"}
    with torch.no_grad():
        ms = _timed(ours, dev, reps)
        res.update(ms_per_batch=round(ms, 3), windows_per_sec=round(S / (ms * 1e-3), 1),
                   tflops=round(flops / (ms * 1e-3) / 1e12, 2),
                   mfma_frac=round(flops / (ms * 1e-3) / 1e12 / MI355X_FP32_MFMA_TFLOPS, 4))
        # the c3 mixed-precision forward on the same windows (bf16 operands, fp32 state): the default
        # large-batch path (sv_dvector_embed_bf16: one 256 x 256 GEMM launch per timestep and layer
        # with the cell in its epilogue) and, beside it, calls of the largest co-resident persistent
        # batch (dvector.bf16_batch)
        from pytorch_speaker_verification_amd.dvector import bf16_batch
        bb = bf16_batch(H)
        ms16 = _timed(lambda: embed_windows(net, xw, precision="bf16"), dev, reps)
        ms16p = _timed(lambda: embed_windows(net, xw, precision="bf16", path="persist"), dev, reps)
        res["bf16"] = {"ms_per_batch": round(ms16, 3), "windows_per_sec": round(S / (ms16 * 1e-3), 1),
                       "path": "per-timestep 256x256 GEMM + fused cell (sv_dvector_embed_bf16)",
                       "tflops": round(flops / (ms16 * 1e-3) / 1e12, 2),
                       "mfma_frac": round(flops / (ms16 * 1e-3) / 1e12 / MI355X_BF16_MFMA_TFLOPS, 4),
                       "persistent_batches": {"ms_per_batch": round(ms16p, 3), "windows_per_call": bb,
                                              "mfma_frac": round(flops / (ms16p * 1e-3) / 1e12 /
                                                                 MI355X_BF16_MFMA_TFLOPS, 4)}}
        # the reference's call shape: one file's windows per call (dvector_create.py:96-100, tens
        # to hundreds of windows); 128 windows, per call (kernels + host), fp32 and bf16
        Sf = 128
        xf = xw[:Sf].contiguous()
        flops_f = flops * Sf / S
        per_file = {"windows": Sf}
        for prec in ("f32", "bf16"):
            msf = _timed(lambda: embed_windows(net, xf, precision=prec), dev, max(reps, 10))
            peak = MI355X_BF16_MFMA_TFLOPS if prec == "bf16" else MI355X_FP32_MFMA_TFLOPS
            per_file[prec] = {"ms_per_call": round(msf, 3), "windows_per_sec": round(Sf / (msf * 1e-3), 1),
                              "mfma_frac": round(flops_f / (msf * 1e-3) / 1e12 / peak, 4)}
            # the same call replayed from a HIP graph (dvector.GraphedEmbedder: one launch per call)
            ge = GraphedEmbedder(net, precision=prec)
            msg = _timed(lambda: ge(xf), dev, max(reps, 10))
            per_file[prec]["graph"] = {"ms_per_call": round(msg, 3), "windows_per_sec": round(Sf / (msg * 1e-3), 1),
                                       "mfma_frac": round(flops_f / (msg * 1e-3) / 1e12 / peak, 4)}
        res["per_file_call"] = per_file
        try:
            lstm = torch.nn.LSTM(F, H, num_layers=L, batch_first=True).to(dev)
            proj = torch.nn.Linear(H, P).to(dev)

            def vendor():  # in chunks of 4096 windows: one 16384-window call fails inside MIOpen
                outs = []
                for i in range(0, S, 4096):
                    y, _ = lstm(xw[i:i + 4096])
                    e = proj(y[:, -1])
                    outs.append(e / e.norm(dim=1, keepdim=True))
                return torch.cat(outs)
            msv = _timed(vendor, dev, reps)
            res["vendor_miopen"] = {"ms_per_batch": round(msv, 3), "windows_per_sec": round(S / (msv * 1e-3), 1)}
        except Exception as ex:
            res["vendor_miopen"] = f"unavailable: {type(ex).__name__}: {str(ex)[:160]}"
    return res


def vendor_baseline(N, M, T, dev, steps=3, dtype="f32"):
    """Stock torch-ROCm on the same GPU: nn.LSTM (MIOpen RNN) + Linear + torch GE2E, autograd,
    clip_grad_norm_ x2, SGD -- the reference's training step run by the vendor libraries.
    dtype bf16: the LSTM and projection run entirely in bf16 (a lower precision than this
    repo's bf16 path, which keeps cell state and gradients fp32)."""
    F, H, L, P = DIMS
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
                "kind": f"torch-rocm nn.LSTM (MIOpen) + autograd, {dtype}, same GPU", "torch": torch.__version__}
    except Exception as ex:  # report, never fail the bench on the vendor leg
        return {"error": f"{type(ex).__name__}: {ex}"[:300]}


def f32_product_accuracy(dev, M=512, N=1024, K=768):
    """Max error of one fp32 GEMM (K1 shape family) against fp64, per product mode, relative to
    |A||B|^T -- the accuracy evidence for the bf16x6 mode."""
    from pytorch_speaker_verification_amd._lib import call, ptr, stream_of
    from pytorch_speaker_verification_amd.ops import F32_PRODUCT_MODES
    g = np.random.default_rng(11)
    A = g.standard_normal((M, K)).astype(np.float32)
    B = g.standard_normal((N, K)).astype(np.float32)
    ref = A.astype(np.float64) @ B.astype(np.float64).T
    scale = np.abs(A).astype(np.float64) @ np.abs(B).astype(np.float64).T
    At, Bt = torch.tensor(A, device=dev), torch.tensor(B, device=dev)
    out = {}
    for mode, code in F32_PRODUCT_MODES.items():
        C = torch.empty(M, N, device=dev)
        call("sv_gemm_f32", 1, 1, M, N, K, ptr(At), K, ptr(Bt), K, ptr(C), N, None, None, 0.0, None, code, stream_of(C))
        err = np.abs(C.cpu().numpy().astype(np.float64) - ref) / scale
        out[mode] = {"max": float(err.max()), "mean": float(err.mean())}
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


def cpu_share():
    """CPUs this job may actually use: the cgroup CPU quota (cpu.max) when one is set -- on the
    GPU box the host grants each GPU job a share of its cores this way, while the affinity mask
    and os.cpu_count() show the whole machine -- else the affinity mask."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return (min(aff, quota) if quota else aff), aff, quota


def cpu_baseline(N, M, T, reps=3):
    """The reference's CPU path (stock PyTorch port, oracle/torch_port.py) on every host CPU this
    job may use (cpu_share: the cgroup quota the host grants it), median of `reps` full training
    steps of the same workload, plus the c1 config (N=4 x M=5)."""
    from oracle import torch_port
    threads, aff, quota = cpu_share()
    torch.set_num_threads(threads)

    def one(Nc, Mc, Tc, r):
        torch.manual_seed(0)
        net = torch_port.SpeechEmbedderPort(*DIMS)
        w = torch.nn.Parameter(torch.tensor(10.0))
        b = torch.nn.Parameter(torch.tensor(-5.0))
        opt = torch.optim.SGD([{"params": net.parameters()}, {"params": [w, b]}], lr=0.01)
        g = torch.Generator().manual_seed(1235)
        torch_port.train_step(net, w, b, opt, torch.randn(8, 16, DIMS[0], generator=g), 4, 2)  # warm oneDNN
        x = torch.randn(Nc * Mc, Tc, DIMS[0], generator=g)
        ts = []
        for _ in range(r):
            t0 = time.perf_counter()
            torch_port.train_step(net, w, b, opt, x, Nc, Mc)
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)), ts
    log(f"cpu baseline on {threads} threads")
    dt, ts = one(N, M, T, reps)
    dt1, _ = one(4, 5, 160, 5)
    log(f"  cpu {dt:.2f} s/step, c1 {dt1:.3f} s/step")
    return {"value": round(N * M / dt, 3), "unit": "embeddings/s", "cores": threads, "kind": "port",
            "host_cpus": os.cpu_count(), "affinity_cpus": aff, "cgroup_quota_cpus": quota,
            "torch_threads": torch.get_num_threads(), "cpu_model": _cpu_model(),
            "steps_per_sec": round(1.0 / dt, 5), "sec_per_step": round(dt, 3),
            "sec_per_step_samples": [round(t, 3) for t in ts],
            "c1": {"workload": "N=4xM=5, T=160, fp32 (BASELINE configs[0])", "sec_per_step": round(dt1, 4),
                   "value": round(20 / dt1, 2), "unit": "embeddings/s"},
            "sample": f"median of {reps} full training steps (fwd+GE2E+bwd+clip+SGD) of N={N}xM={M}, T={T}, fp32, "
                      f"oracle/torch_port.py (nn.LSTM on oneDNN) on {threads} threads = every CPU this job may use "
                      f"(cgroup quota {quota}, affinity {aff}, host {os.cpu_count()}); c1: median of 5"}


def _launch_ranks(args):
    """--gpus N without an external launcher: start N ranks (torch.distributed.run) as a child
    process before this process initialises the GPU, and return its exit code."""
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def bf16_roofline(probes, B, T, steps, where):
    """(backward, forward) roofline entries of the bf16 step's recurrences from its probe events:
    per-layer persistent launches (one event pair per layer) or the one-launch layer wavefront (its
    first pair spans the whole launch)."""
    r = bf16_recurrences(B, T)
    n = r["launches"]
    if r["kind"] == "wave":
        what = ("one launch for all {L} layers (layer wavefront, sv_wave.hip / sv_persist3.hip); FLOPs = every "
                "layer's {part} at {rows} rows").format(L=DIMS[2], rows=r["rows"], part="{part}")
        nb = what.format(part="dh_rec and the upper layers' dx contractions")
        nf = what.format(part="input and recurrent gate contractions")
    else:
        nb = f"persistent backward recurrence, one launch per layer, {r['rows']} rows per launch"
        nf = (f"persistent forward recurrence, one launch per layer, {r['rows']} rows; layer 0: "
              "lstm_persist2_fwd_bf16_kernel with the fused input projection")
    chunk = "" if r["rows"] == B else f" (the first of the step's row chunks: {r['rows']} of {B} rows)"
    note = f"in-step: HIP events around each launch inside the {where}{chunk}"
    bwd = roofline_entry(f"{r['bwd']} ({nb})", r["bwd_flops"], probe_ms(probes, "bwd") / n, MI355X_BF16_MFMA_TFLOPS,
                         pmc_traffic(r["bwd"]), n * steps, note)
    fwd = roofline_entry(f"{r['fwd']} ({nf})", r["fwd_flops"], probe_ms(probes, "fwd") / n, MI355X_BF16_MFMA_TFLOPS,
                         pmc_traffic(r["fwd"]), n * steps, note + " (average over the launches)")
    return bwd, fwd


def roofline_entry(kernel, flops, ms, peak, traffic, launches, note):
    ach = flops / (ms * 1e-3) / 1e12
    return {"kernel": kernel, "bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(ach / peak, 4), "traffic": traffic, "avg_launch_us": round(ms * 1e3, 2),
            "flops_per_launch": flops, "launches_timed": launches, "timing": note}


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
    ap.add_argument("--no-bf16", action="store_true", help="skip the bf16 side measurements (c3/c4/c5)")
    ap.add_argument("--no-f32x", action="store_true", help="skip the fp32-via-bf16x6 side measurement")
    ap.add_argument("--no-vendor", action="store_true", help="skip the nn.LSTM/MIOpen same-GPU baseline")
    ap.add_argument("--no-extras", action="store_true", help="skip the isolated-kernel, HBM-kernel and d-vector "
                    "lines (profiling runs that want only the training steps)")
    ap.add_argument("--preset", choices=["c2", "c3", "c4", "c5"], default=None,
                    help="headline config: c2 = N64 M10 T160 f32 per GPU (default), c3 = the same in bf16, "
                         "c4 = N64 M10 T160 bf16 split over the GPUs (strong scaling), c5 = N256 M10 T180 bf16 "
                         "split over the GPUs")
    ap.add_argument("--dtype", choices=["f32", "bf16"], default="f32")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    ctx = Ctx(world, rank, dev)
    F, H, L, P = DIMS

    # ---- headline -------------------------------------------------------------------------
    strong = args.preset in ("c4", "c5")
    dtype = "bf16" if args.preset in ("c3", "c4", "c5") else args.dtype
    if args.preset == "c5":
        Ng, M, T = 256, 10, 180
    else:
        Ng, M, T = args.N, args.M, args.T
    N = max(1, Ng // world) if strong else Ng
    B = N * M
    from pytorch_speaker_verification_amd._lib import lib as _svlib
    # fp32: the persistent recurrences where the library picks them (c2: 240 of 256 CUs), else
    # the per-step kernels with their in-kernel stamps
    f32_persist = dtype == "f32" and bool(_svlib().sv_lstm_f32_persist_ok(B, H, 0))
    # the step time without timing probes (each probe event record idles the GPU ~6 us between two
    # kernels: 12 records per c2 step), then the same steps again with the probes for the roofline
    dt, loss, host, _, tr = run_steps(ctx, N, M, T, dtype, args.steps, args.warmup, 1235)
    dt_probed, _, _, probes, _ = run_steps(ctx, N, M, T, dtype, args.steps, 1, 1235,
                                           probe="bwd_chunks" if dtype == "f32" and not f32_persist else "fwd_bwd")
    ms_step = dt / args.steps * 1e3
    fwd_fl, st_fl = step_flops(B, T, F, H, P, L)
    peak = MI355X_FP32_MFMA_TFLOPS if dtype == "f32" else MI355X_BF16_MFMA_TFLOPS
    emb_total = world * B
    out = {
        "metric": METRIC,
        "value": round(emb_total * args.steps / dt, 3),
        "unit": "embeddings/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": dtype,
        "data": "synthetic x~N(0,1) frames, reference init (torch.manual_seed(0))",
        "config": {"workload": (f"GE2E train step, global N={N * world}xM={M} split over {world} GPU(s)" if strong else
                                f"GE2E train step N={N}xM={M} per GPU") + f", T={T}, 40 mels, LSTM 3x768, proj 256",
                   "preset": args.preset or ("c3" if dtype == "bf16" else "c2"),
                   "global_batch": emb_total, "speakers_global": N * world, "per_gpu_batch": B, "seq_len": T,
                   "parallelism": f"dp{world} (speaker-sharded GE2E, RCCL grad all-reduce)"},
        "steps_per_sec": round(args.steps / dt, 4),
        "host_enqueue_ms_per_step": round(host / args.steps * 1e3, 3),
        "probed_ms_per_step": round(dt_probed / args.steps * 1e3, 3),
        "loss": round(loss, 5),
        "step_tflops_per_gpu": round(st_fl / (ms_step * 1e-3) / 1e12, 2),
        "step_mfma_frac": round(st_fl / (ms_step * 1e-3) / 1e12 / peak, 4),
    }
    if f32_persist:
        fl = 2.0 * B * T * H * 4 * H
        out["roofline"] = roofline_entry(
            "lstm_persist_bwd_f32_h2_kernel (the c2 step's worst-fraction in-step kernel, not its largest by busy time "
            "-- that is the dW GEMM, roofline_dw_gemm: persistent fp32 backward recurrence, one launch per layer, two "
            "32-row chains, W_hh in registers, fp32 MFMA 32x32x2)", fl, probe_ms(probes, "bwd") / L, MI355X_FP32_MFMA_TFLOPS,
            pmc_traffic("lstm_persist_bwd_f32_h2_kernel"), L * args.steps,
            "in-step: HIP events around each layer's launch inside the timed steps (on its stream, main)")
        out["roofline_fwd"] = roofline_entry(
            "lstm_persist_fwd_f32_kernel (persistent fp32 forward recurrence)", fl, probe_ms(probes, "fwd") / L,
            MI355X_FP32_MFMA_TFLOPS, pmc_traffic("lstm_persist_fwd_f32_kernel"), L * args.steps,
            "in-step, as roofline (average over the L layers' launches)")
    elif dtype == "f32":
        # K3, the headline step's dominant kernel: per-chunk HIP-event spans on its own stream over
        # the timed steps / its L*T launches per step
        from pytorch_speaker_verification_amd.ops import PIPELINE_CHUNK
        us_k3, n_k3 = kstamp_us(probes)
        ms_ev = probe_ms(probes, "bwd") / (L * ((T + PIPELINE_CHUNK - 1) // PIPELINE_CHUNK))
        out["roofline"] = roofline_entry(
            "lstm_step_bwd_v2_kernel (K3, fp32 MFMA 32x32x2, backward recurrent step)", 2.0 * B * H * 4 * H,
            us_k3 * 1e-3, MI355X_FP32_MFMA_TFLOPS, pmc_traffic("lstm_step_bwd_v2_kernel"), n_k3,
            "in-step: every K3 launch of the timed steps, timed by the kernel's own start / end stamps on the GPU's "
            "100 MHz real-time clock (execution span, as rocprofv3 measures it; HIP event pairs on the stream also "
            "count the wait for CUs held by the concurrent GEMMs: stream_span_us, HIP events around one launch per "
            "32-step chunk)")
        out["roofline"]["stream_span_us"] = round(ms_ev * 1e3, 2)
    else:
        out["roofline"], out["roofline_fwd"] = bf16_roofline(probes, B, T, args.steps, "timed steps")

    # forward-only (inference) embeddings/s at the headline shape
    from pytorch_speaker_verification_amd.ops import embedder_forward, embedder_forward_bf16
    g = torch.Generator(device="cpu").manual_seed(1235 + rank)
    x = torch.randn(B, T, F, generator=g).to(dev)
    net = tr.net
    layers = net.LSTM_stack.layer_params()
    fwd_fn = embedder_forward_bf16 if dtype == "bf16" else embedder_forward
    with torch.no_grad():
        for _ in range(2):
            fwd_fn(x, layers, net.projection.weight, net.projection.bias, save=False)
        ctx.barrier()
        tf0 = time.perf_counter()
        for _ in range(args.fwd_steps):
            fwd_fn(x, layers, net.projection.weight, net.projection.bias, save=False)
        ctx.barrier()
        tf = ctx.max_over_ranks((time.perf_counter() - tf0) / args.fwd_steps)
    out["fwd_embeddings_per_sec"] = round(emb_total / tf, 1)
    # the two readings of the metric side by side, under explicit names: `value` stays the training
    # step's embeddings/s (the series every round reports); SURVEY §8d defines embeddings/s as
    # N*M / t(forward, no grad) and GE2E steps/s as 1 / t(full training step)
    out["metric_readings"] = {
        "train_step_embeddings_per_sec": out["value"],
        "forward_only_embeddings_per_sec": out["fwd_embeddings_per_sec"],
        "ge2e_steps_per_sec": out["steps_per_sec"],
        "value_is": "train_step_embeddings_per_sec (N*M*world / t(fwd + GE2E + bwd + clip + SGD))",
        "forward_only_is": "SURVEY 8d embeddings/s: N*M*world / t(forward, no grad, save=False)",
    }

    # ---- side measurements ----------------------------------------------------------------
    def side(name, Nl, Ml, Tl, prec, strong_, descr, probe=None, products="mfma_f32"):
        # the step time without timing probes (each probe event record idles the GPU ~6 us between
        # two kernels: 4 - 12 per step at these shapes), then, for the roofline entries, a second
        # run of the same steps with the probes (its time is reported beside, probed_ms_per_step)
        # at least SIDE_STEPS timed steps: a 2 ms step timed over K = 10 steps carried the timed region's
        # start-up (the first kernel is enqueued only after the barrier) as ~1 % of its step time
        ns, nw = max(args.steps, SIDE_STEPS), max(args.warmup, 5)
        d, l_, _, _, _ = run_steps(ctx, Nl, Ml, Tl, prec, ns, nw, 2235, products=products)
        pr, dp = None, None
        if probe:
            dp, _, _, pr, _ = run_steps(ctx, Nl, Ml, Tl, prec, ns, 1, 2235, probe=probe, products=products)
        ms = d / ns * 1e3
        _, fl = step_flops(Nl * Ml, Tl, F, H, P, L)
        tot = Nl * Ml * world
        o = {"config": descr, "value": round(tot * ns / d, 3), "unit": "embeddings/s", "steps": ns, "warmup": nw,
             "ms_per_step": round(ms, 3), "steps_per_sec": round(ns / d, 4), "loss": round(l_, 5),
             "scaling": "strong" if strong_ else "weak", "per_gpu_batch": Nl * Ml, "seq_len": Tl,
             "step_tflops_per_gpu": round(fl / (ms * 1e-3) / 1e12, 2),
             "step_mfma_frac": round(fl / (ms * 1e-3) / 1e12 /
                                     (MI355X_FP32_MFMA_TFLOPS if prec == "f32" else MI355X_BF16_MFMA_TFLOPS), 4)}
        if dp is not None:
            o["probed_ms_per_step"] = round(dp / ns * 1e3, 3)
        out[name] = o
        return o, pr

    if not args.no_bf16 and args.preset is None and dtype == "f32":
        o, pr = side("bf16", N, M, T, "bf16", False, "c3: the headline workload with bf16 GEMM operands, fp32 "
                     "accumulate/state/loss", probe="fwd_bwd")
        out["roofline_bf16"], out["roofline_bf16_fwd"] = bf16_roofline(pr, B, T, len(pr), "timed c3 steps")
        def side_rl(name, Nl, Tl, descr):
            o, pr = side(name, Nl, 10, Tl, "bf16", True, descr, probe="fwd_bwd")
            o["roofline"], o["roofline_fwd"] = bf16_roofline(pr, Nl * 10, Tl, len(pr), f"timed {name} steps")
        if world > 1:
            side_rl("c4", max(1, 64 // world), 160,
                    f"c4: N=64xM=10, T=160, bf16, split over {world} GPUs ({max(1, 64 // world)} speakers per rank); "
                    "value = 640 embeddings per step / time")
            side_rl("c5", max(1, 256 // world), 180,
                    f"c5: N=256xM=10, T=180, bf16, split over {world} GPUs ({max(1, 256 // world)} speakers per rank)")
        else:
            side_rl("c4_rank_shape", 8, 160,
                    "one rank's share of c4 at 8 GPUs (N=8xM=10, T=160, bf16) run alone on this GPU: the per-rank "
                    "step time of the 8-GPU strong-scaling config (value counts this GPU's 80 embeddings)")
            side_rl("c5_rank_shape", 32, 180,
                    "one rank's share of c5 at 8 GPUs (N=32xM=10, T=180, bf16) run alone on this GPU; its GE2E runs "
                    "the single-GPU fused kernel at N=32 (the real rank's sharded GE2E: c5_rank_ge2e)")
    if not args.no_f32x and dtype == "f32" and world == 1:
        o, _ = side("f32_bf16x6", N, M, T, "f32", False,
                    "same workload, fp32 products formed as six bf16 MFMA products of a three-way bf16 split (fp32 "
                    "accumulation); opt-in per module: net.f32_products = 'bf16x6'", products="bf16x6")
        o["gemm_error_vs_fp64"] = f32_product_accuracy(dev)
    if rank == 0 and not args.no_extras:
        ms_g, fl_g, by_g = time_gemm_kernel(160 * 640, 4 * H, H, dev)
        out["roofline_gemm"] = dict(roofline_entry(
            f"gemm_f32_256p_kernel<256,32> (K1/dx NT GEMM: persistent, one workgroup per CU walking 256x256 LDS-DMA "
            f"tiles, fp32 MFMA 32x32x2), K1 shape "
            f"M={160 * 640} N={4 * H} K={H}",
            fl_g, ms_g, MI355X_FP32_MFMA_TFLOPS, pmc_traffic("gemm_f32_256p_kernel<256,32>@K1"), 5,
            "isolated launches after 3 untimed ones, HIP events on its stream"), algorithmic_bytes=by_g)
        ms_w, fl_w, by_w = time_dw_gemm(T, B, H, dev)
        out["roofline_dw_gemm"] = dict(roofline_entry(
            f"gemm_f32_256_kernel<256,32,1,0> (dW_hh = dG^T h of the persistent fp32 backward: split-K slabs, the c2 "
            f"step's largest kernel by busy time), M={4 * H} N={H} K={T * B}", fl_w, ms_w, MI355X_FP32_MFMA_TFLOPS,
            pmc_traffic("gemm_f32_256_kernel<256,32,1,0>@dW.in_step"), 5,
            "isolated launches after 3 untimed ones, HIP events on its stream"), algorithmic_bytes=by_w)
        ms_k, fl_k = time_step_kernel(640, H, dev)
        out["roofline_step_kernel"] = roofline_entry(
            "lstm_step_fwd_v2_kernel (K2, fp32 forward recurrent step) at B=640", fl_k, ms_k,
            MI355X_FP32_MFMA_TFLOPS, pmc_traffic("lstm_step_fwd_v2_kernel"), 64, "isolated launches")
        if world == 1:
            log("hbm kernels / vendor baseline")
            out["hbm_kernels"] = hbm_kernels(tr, N, M, P, dev)
            out["c5_rank_ge2e"] = c5_rank_ge2e(dev)
            log("d-vector inference")
            out["dvector_inference"] = dvector_inference(tr.net, dev)
            if not args.no_vendor:
                out["vendor_baseline"] = vendor_baseline(N, M, T, dev, dtype=dtype)
                if "bf16" in out:
                    out["bf16"]["vendor_baseline"] = vendor_baseline(N, M, T, dev, dtype="bf16")
    if world == 1 and not args.no_extras and not strong:
        log("drop-in loop body")
        out["dropin_loop"] = dropin_loop(ctx, N, M, T, args.steps, args.warmup, dtype)
        out["dropin_loop"]["vs_fused_trainer"] = round(out["dropin_loop"]["ms_per_step"] / ms_step, 4)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(N, M, T)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

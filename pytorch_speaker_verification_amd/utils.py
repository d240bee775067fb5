"""Drop-in GE2E helpers (reference utils.py:27-132) on the HIP kernels.

``get_centroids``, ``get_cossim`` and ``calc_loss`` keep the reference's names, argument
meaning and output shapes, and they are differentiable like the reference's autograd ops: a loss
composed from them as ``GE2ELoss.forward`` does (speech_embedder_net.py:45-48) trains, with the
backward in HIP kernels (include/sv_ge2e.h, sv_ge2e_*_bwd).  They are also the stand-alone forms
used outside the training loss (the EER evaluation, train_speech_embedder.py:127-129).  Inputs
may live on the CPU (the reference's test() never moves its net, :100-102): CPU inputs make a
round trip to the current GPU, results and gradients come back to the CPU.
"""
from __future__ import annotations

import torch

from ._lib import call, compute_device, lib, ptr, stream_of


def _dev(t, dev):
    return t.detach().float().to(dev).contiguous()


def _pad_d(*ts):
    """Zero-pad the last dim to a multiple of 4 (the kernels' float4 rows); returns (tensors, D)."""
    D = ts[0].shape[-1]
    if D % 4 == 0:
        return ts, D
    Dp = (D + 3) // 4 * 4
    return tuple(torch.nn.functional.pad(t, (0, Dp - D)).contiguous() for t in ts), D


class _Centroids(torch.autograd.Function):
    """C = E.mean(1) (utils.py:27-29); backward dE = dC / M broadcast (sv_ge2e_centroids_bwd)."""

    @staticmethod
    def forward(ctx, E):
        home, dev = E.device, compute_device(E)
        Ed = _dev(E, dev)
        N, M, D = Ed.shape
        C = torch.empty((N, D), dtype=torch.float32, device=dev)
        call("sv_ge2e_centroids", ptr(Ed), N, M, D, ptr(C), stream_of(Ed))
        ctx.home, ctx.dev, ctx.shape = home, dev, (N, M, D)
        return C.to(home)

    @staticmethod
    def backward(ctx, dC):
        N, M, D = ctx.shape
        g = _dev(dC, ctx.dev)
        dE = torch.empty((N, M, D), dtype=torch.float32, device=ctx.dev)
        call("sv_ge2e_centroids_bwd", ptr(g), N, M, D, ptr(dE), stream_of(g))
        return dE.to(ctx.home)


class _Cossim(torch.autograd.Function):
    """cos [N,M,Nc] = get_cossim(E, C) (utils.py:72-115); backward through the cosines against C_k
    (k != j) and, on the diagonal, through E's own leave-one-out centroid (sv_ge2e_cossim_bwd)."""

    @staticmethod
    def forward(ctx, E, C):
        home, dev = E.device, compute_device(E)
        (Ed, Cd), D0 = _pad_d(_dev(E, dev), _dev(C, dev))
        N, M, D = Ed.shape
        Nc = Cd.shape[0]
        cos = torch.empty((N, M, Nc), dtype=torch.float32, device=dev)
        ws = torch.empty(max(1, lib().sv_ge2e_cossim_workspace(N, M, D, Nc) // 4 + 1), dtype=torch.float32, device=dev)
        call("sv_ge2e_cossim", ptr(Ed), N, M, D, ptr(Cd), Nc, ptr(cos), ptr(ws), stream_of(Ed))
        ctx.save_for_backward(Ed, Cd)
        ctx.home, ctx.c_home, ctx.dev, ctx.D0 = home, C.device, dev, D0
        return cos.to(home)

    @staticmethod
    def backward(ctx, dcos):
        Ed, Cd = ctx.saved_tensors
        N, M, D = Ed.shape
        Nc = Cd.shape[0]
        g = _dev(dcos, ctx.dev)
        dE = torch.empty_like(Ed)
        dC = torch.empty_like(Cd)
        ws = torch.empty(max(1, lib().sv_ge2e_cossim_bwd_workspace(N, M, D, Nc) // 4 + 1), dtype=torch.float32,
                         device=ctx.dev)
        call("sv_ge2e_cossim_bwd", ptr(Ed), N, M, D, ptr(Cd), Nc, ptr(g), ptr(dE), ptr(dC), ptr(ws), stream_of(g))
        D0 = ctx.D0
        return dE[..., :D0].contiguous().to(ctx.home), dC[..., :D0].contiguous().to(ctx.c_home)


class _CalcLoss(torch.autograd.Function):
    """(loss, per) = calc_loss(S) (utils.py:126-132); backward dS_jik = (gloss + gper_ji)
    (softmax_jik Z/(Z + 1e-6) - [k == j]) (sv_ge2e_calc_loss_bwd)."""

    @staticmethod
    def forward(ctx, S):
        home, dev = S.device, compute_device(S)
        Sd = _dev(S, dev)
        N, M, K = Sd.shape
        per = torch.empty((N, M), dtype=torch.float32, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        call("sv_ge2e_calc_loss", ptr(Sd), N, M, K, ptr(per), ptr(loss), stream_of(Sd))
        ctx.save_for_backward(Sd)
        ctx.home, ctx.dev = home, dev
        return loss.to(home), per.to(home)

    @staticmethod
    def backward(ctx, gloss, gper):
        (Sd,) = ctx.saved_tensors
        N, M, K = Sd.shape
        gl = None if gloss is None else _dev(gloss.reshape(1), ctx.dev)
        gp = None if gper is None else _dev(gper, ctx.dev)
        dS = torch.empty_like(Sd)
        call("sv_ge2e_calc_loss_bwd", ptr(Sd), N, M, K, ptr(gl), ptr(gp), ptr(dS), stream_of(Sd))
        return dS.to(ctx.home)


def get_centroids(embeddings):
    """C[j] = mean_i E[j, i]  (utils.py:27-29).  [N,M,D] -> [N,D]."""
    return _Centroids.apply(embeddings)


def get_cossim(embeddings, centroids):
    """cos[j,i,k] = cosine(E_ji, C_k) + 1e-6, the diagonal k = j taken against E's own
    leave-one-out centroid (utils.py:72-115).  [N,M,D], [Nc,D] -> [N,M,Nc]."""
    N, M, _ = embeddings.shape
    if M < 2:
        raise ValueError("get_cossim needs M >= 2 utterances per speaker (leave-one-out centroids)")
    if centroids.shape[0] < N:
        raise IndexError("get_cossim: fewer centroids than speakers (the reference indexes cos[j,:,j])")
    return _Cossim.apply(embeddings, centroids)


def calc_loss(sim_matrix):
    """(loss, per_embedding_loss[N,M]) with per = log(sum_k e^S + 1e-6) - S[j,i,j]
    (utils.py:126-132)."""
    return _CalcLoss.apply(sim_matrix)

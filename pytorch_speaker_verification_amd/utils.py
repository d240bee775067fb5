"""Drop-in GE2E helpers (reference utils.py:27-132) on the HIP kernels.

``get_centroids``, ``get_cossim`` and ``calc_loss`` keep the reference's names, argument
meaning and output shapes; they are the stand-alone forms used outside the training loss
(e.g. the EER evaluation, train_speech_embedder.py:127-129).  They compute forward values
only: training differentiates through ``GE2ELoss`` (fused kernels with a closed-form
backward), so their outputs carry a backward that raises instead of silently dropping
gradients.  Inputs may require grad (the reference's test() runs its net without no_grad) and
may live on the CPU (its net is never moved, :100-102): CPU inputs make a round trip to the
current GPU and the result comes back to the CPU.
"""
from __future__ import annotations

import torch

from ._lib import call, compute_device, lib, ptr, stream_of


class _ForwardOnly(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fn, *inputs):
        return fn(*inputs)

    @staticmethod
    def backward(ctx, *grads):
        raise RuntimeError("get_centroids/get_cossim/calc_loss are forward-only kernels; "
                           "train through GE2ELoss")


def _run(fn, *tensors):
    """fn (which moves its inputs to the compute GPU itself) on tensors; outputs return to the
    first input's device.  With grad-requiring inputs a backward through the outputs raises."""
    home = tensors[0].device
    if torch.is_grad_enabled() and any(t.requires_grad for t in tensors):
        outs = _ForwardOnly.apply(fn, *tensors)
    else:
        outs = fn(*tensors)
    if isinstance(outs, tuple):
        return tuple(o.to(home) for o in outs)
    return outs.to(home)


def _centroids(E):
    E = E.detach().float().to(compute_device(E)).contiguous()
    N, M, D = E.shape
    C = torch.empty((N, D), dtype=torch.float32, device=E.device)
    call("sv_ge2e_centroids", ptr(E), N, M, D, ptr(C), stream_of(E))
    return C


def _cossim(E, C):
    dev = compute_device(E)
    E = E.detach().float().to(dev).contiguous()
    C = C.detach().float().to(dev).contiguous()
    N, M, D = E.shape
    Nc = C.shape[0]
    if D % 4:
        Dp = (D + 3) // 4 * 4
        E = torch.nn.functional.pad(E, (0, Dp - D)).contiguous()
        C = torch.nn.functional.pad(C, (0, Dp - D)).contiguous()
        D = Dp
    cos = torch.empty((N, M, Nc), dtype=torch.float32, device=dev)
    ws = torch.empty(max(1, lib().sv_ge2e_cossim_workspace(N, M, D, Nc) // 4 + 1), dtype=torch.float32, device=dev)
    call("sv_ge2e_cossim", ptr(E), N, M, D, ptr(C), Nc, ptr(cos), ptr(ws), stream_of(E))
    return cos


def _calc_loss(S):
    S = S.detach().float().to(compute_device(S)).contiguous()
    N, M, K = S.shape
    per = torch.empty((N, M), dtype=torch.float32, device=S.device)
    loss = torch.empty((), dtype=torch.float32, device=S.device)
    call("sv_ge2e_calc_loss", ptr(S), N, M, K, ptr(per), ptr(loss), stream_of(S))
    return loss, per


def get_centroids(embeddings):
    """C[j] = mean_i E[j, i]  (utils.py:27-29).  [N,M,D] -> [N,D]."""
    return _run(_centroids, embeddings)


def get_cossim(embeddings, centroids):
    """cos[j,i,k] = cosine(E_ji, C_k) + 1e-6, the diagonal k = j taken against E's own
    leave-one-out centroid (utils.py:72-115).  [N,M,D], [Nc,D] -> [N,M,Nc]."""
    N, M, _ = embeddings.shape
    if M < 2:
        raise ValueError("get_cossim needs M >= 2 utterances per speaker (leave-one-out centroids)")
    if centroids.shape[0] < N:
        raise IndexError("get_cossim: fewer centroids than speakers (the reference indexes cos[j,:,j])")
    return _run(_cossim, embeddings, centroids)


def calc_loss(sim_matrix):
    """(loss, per_embedding_loss[N,M]) with per = log(sum_k e^S + 1e-6) - S[j,i,j]
    (utils.py:126-132)."""
    return _run(_calc_loss, sim_matrix)

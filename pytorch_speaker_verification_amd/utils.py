"""Drop-in GE2E helpers (reference utils.py:27-132) on the HIP kernels.

``get_centroids``, ``get_cossim`` and ``calc_loss`` keep the reference's names, argument
meaning and output shapes; they are the stand-alone forms used outside the training loss
(e.g. the EER evaluation, train_speech_embedder.py:127-129).  They are forward-only:
training differentiates through ``GE2ELoss`` (fused kernels with a closed-form backward),
so calling them on tensors that require grad raises instead of silently dropping grads.
"""
from __future__ import annotations

import torch

from ._lib import call, lib, ptr, require_device, stream_of


def _fwd_only(*ts):
    if torch.is_grad_enabled() and any(t.requires_grad for t in ts):
        raise RuntimeError("get_centroids/get_cossim/calc_loss are forward-only kernels; "
                           "train through GE2ELoss (or wrap the call in torch.no_grad())")


def get_centroids(embeddings):
    """C[j] = mean_i E[j, i]  (utils.py:27-29).  [N,M,D] -> [N,D]."""
    E = embeddings.float().contiguous()
    require_device(E)
    _fwd_only(embeddings)
    N, M, D = E.shape
    C = torch.empty((N, D), dtype=torch.float32, device=E.device)
    call("sv_ge2e_centroids", ptr(E), N, M, D, ptr(C), stream_of(E))
    return C


def get_cossim(embeddings, centroids):
    """cos[j,i,k] = cosine(E_ji, C_k) + 1e-6, the diagonal k = j taken against E's own
    leave-one-out centroid (utils.py:72-115).  [N,M,D], [Nc,D] -> [N,M,Nc]."""
    E = embeddings.float().contiguous()
    C = centroids.float().contiguous()
    require_device(E, C)
    _fwd_only(embeddings, centroids)
    N, M, D = E.shape
    Nc = C.shape[0]
    if M < 2:
        raise ValueError("get_cossim needs M >= 2 utterances per speaker (leave-one-out centroids)")
    if Nc < N:
        raise IndexError("get_cossim: fewer centroids than speakers (the reference indexes cos[j,:,j])")
    if D % 4:
        Dp = (D + 3) // 4 * 4
        E = torch.nn.functional.pad(E, (0, Dp - D)).contiguous()
        C = torch.nn.functional.pad(C, (0, Dp - D)).contiguous()
        D = Dp
    cos = torch.empty((N, M, Nc), dtype=torch.float32, device=E.device)
    ws = torch.empty(max(1, lib().sv_ge2e_cossim_workspace(N, M, D, Nc) // 4 + 1), dtype=torch.float32,
                     device=E.device)
    call("sv_ge2e_cossim", ptr(E), N, M, D, ptr(C), Nc, ptr(cos), ptr(ws), stream_of(E))
    return cos


def calc_loss(sim_matrix):
    """(loss, per_embedding_loss[N,M]) with per = log(sum_k e^S + 1e-6) - S[j,i,j]
    (utils.py:126-132)."""
    S = sim_matrix.float().contiguous()
    require_device(S)
    _fwd_only(sim_matrix)
    N, M, K = S.shape
    per = torch.empty((N, M), dtype=torch.float32, device=S.device)
    loss = torch.empty((), dtype=torch.float32, device=S.device)
    call("sv_ge2e_calc_loss", ptr(S), N, M, K, ptr(per), ptr(loss), stream_of(S))
    return loss, per

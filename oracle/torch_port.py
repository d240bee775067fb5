"""ORACLE (test infrastructure only) -- the reference's hot path restated on stock PyTorch.

A port of speech_embedder_net.py:15-49 + utils.py:27-132 + train_speech_embedder.py:54-65
onto plain torch ops (nn.LSTM = oneDNN on CPU, MIOpen on GPU).  Two uses:
  * bench.py's ``cpu_baseline`` leg: the reference's CPU execution path timed on the GPU
    box's host cores (the reference's own Python never travels there);
  * the full-size checker in tests (N=64 x M=10, T=160) where the numpy oracle is too slow.
It is pinned to the reference by tests/test_oracle_golden.py-style checks against the same
golden vectors (tests/test_torch_port.py).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class SpeechEmbedderPort(nn.Module):
    def __init__(self, nmels=40, hidden=768, num_layer=3, proj=256):
        super().__init__()
        self.LSTM_stack = nn.LSTM(nmels, hidden, num_layers=num_layer, batch_first=True)
        self.projection = nn.Linear(hidden, proj)

    def forward(self, x):
        x, _ = self.LSTM_stack(x.float())
        x = x[:, x.size(1) - 1]
        x = self.projection(x)
        return x / torch.norm(x, dim=1).unsqueeze(1)


def ge2e_loss(E, w, b):
    """GE2ELoss.forward restated: centroids, leave-one-out diagonal, w*cos+b, sum loss."""
    N, M, D = E.shape
    C = E.mean(dim=1)
    U = (E.sum(dim=1, keepdim=True) - E) / (M - 1)
    En = E / E.norm(dim=2, keepdim=True).clamp_min(1e-8)
    Cn = C / C.norm(dim=1, keepdim=True).clamp_min(1e-8)
    Un = U / U.norm(dim=2, keepdim=True).clamp_min(1e-8)
    cos = torch.einsum("jid,kd->jik", En, Cn)
    same = (En * Un).sum(-1)
    eye = torch.eye(N, dtype=torch.bool, device=E.device)[:, None, :]
    cos = torch.where(eye, same[:, :, None], cos) + 1e-6
    S = w * cos + b
    pos = (S * eye).sum(-1)
    neg = torch.log(torch.exp(S).sum(-1) + 1e-6)
    return (neg - pos).sum()


def load_recipe_weights(net, sd_np):
    with torch.no_grad():
        for k, v in net.state_dict().items():
            v.copy_(torch.as_tensor(sd_np[k]))


def train_step(net, w, b, opt, x, N, M):
    """One train_speech_embedder.py:54-65 step body; returns the loss (tensor)."""
    opt.zero_grad()
    emb = net(x).reshape(N, M, -1)
    loss = ge2e_loss(emb, w, b)
    loss.backward()
    torch.nn.utils.clip_grad_norm_(net.parameters(), 3.0)
    torch.nn.utils.clip_grad_norm_([w, b], 1.0)
    opt.step()
    return loss


class GE2ELossPort(nn.Module):
    """GE2ELoss (speech_embedder_net.py:35-49) as a module with learnable w = 10, b = -5, for the
    reference's own loop body (its optimizer takes ge2e_loss.parameters())."""

    def __init__(self, device):
        super().__init__()
        self.w = nn.Parameter(torch.tensor(10.0, device=device))
        self.b = nn.Parameter(torch.tensor(-5.0, device=device))

    def forward(self, embeddings):
        return ge2e_loss(embeddings, self.w, self.b)

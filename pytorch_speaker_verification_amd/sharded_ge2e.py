"""Speaker-sharded GE2E across ranks ("exact-parity partitioning").

Rank r owns speakers [r*N_local, (r+1)*N_local) with all their M utterances, so the
leave-one-out centroids stay local.  Per step:

  fwd  per-speaker sums (local)  --all_gather-->  Ssum [N, D]  --> local rows of S [N_local*M, N],
       local loss (the global loss is the SUM over ranks; all_reduce only for reporting)
  bwd  local rows give this shard's dC^ [Np, D] and beta [N] contributions --all_reduce(SUM)-->
       finalize the local dE; (dw, db) stay per-rank partials and are summed together with
       the network gradients by the caller.

With world size 1 this is exactly the single-GPU GE2ELoss.  The per-shard arithmetic is
a pluggable ``kernels`` object: the HIP kernels (``HipShardKernels``) in production; the
CPU tests plug in a numpy restatement so the exchange protocol runs under gloo.  For the
training step (``train``) with global N <= 256 the HIP kernels run in their fused sharded form
(``HipFusedShard``: prep, rows, finalize around the same two exchanges; c5's N = 256 stages the
centroids in two LDS tiles); larger N take the split kernels.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ._lib import call, lib, ptr, stream_of


class HipShardKernels:
    """Per-shard GE2E steps on the C ABI (sv_ge2e_speaker_sums / fwd_rows / bwd_rows / finalize)."""

    def speaker_sums(self, E):
        Nl, M, D = E.shape
        out = torch.empty((Nl, D), dtype=torch.float32, device=E.device)
        call("sv_ge2e_speaker_sums", ptr(E), Nl, M, D, ptr(out), stream_of(E))
        return out

    def fwd_rows(self, E, s0, N, ssum_all, w, b):
        Nl, M, D = E.shape
        ws = torch.empty(lib().sv_ge2e_workspace_size(Nl, M, D, N) // 4 + 1, dtype=torch.float32, device=E.device)
        per = torch.empty((Nl, M), dtype=torch.float32, device=E.device)
        loss = torch.empty((), dtype=torch.float32, device=E.device)
        call("sv_ge2e_fwd_rows", ptr(E), Nl, M, D, s0, N, ptr(ssum_all), ptr(w), ptr(b), ptr(per), ptr(loss), ptr(ws),
             stream_of(E))
        return loss, per, {"ws": ws, "shape": (Nl, M, D), "s0": s0, "N": N}

    def bwd_rows(self, st, w, b, gloss):
        Nl, M, D = st["shape"]
        N = st["N"]
        Np = (N + 3) // 4 * 4
        dev = st["ws"].device
        # one buffer so the caller can all_reduce dC^ and beta together
        red = torch.empty(Np * D + N, dtype=torch.float32, device=dev)
        dwdb = torch.empty(2, dtype=torch.float32, device=dev)
        call("sv_ge2e_bwd_rows", Nl, M, D, st["s0"], N, ptr(w), ptr(b), ptr(gloss), ptr(red), ptr(red[Np * D:]),
             ptr(dwdb), ptr(st["ws"]), stream_of(red))
        return red, dwdb

    def finalize(self, st, red):
        Nl, M, D = st["shape"]
        N = st["N"]
        Np = (N + 3) // 4 * 4
        dE = torch.empty((Nl, M, D), dtype=torch.float32, device=red.device)
        call("sv_ge2e_bwd_finalize", Nl, M, D, st["s0"], N, ptr(red), ptr(red[Np * D:]), ptr(dE), ptr(st["ws"]),
             stream_of(red))
        return dE


class HipFusedShard:
    """The fused GE2E kernels in the speaker-sharded form (sv_ge2e_shard_prep / _rows /
    _finalize): 3 launches + the centroid pass around the two exchanges, for global N <= 256
    (sv_ge2e_train_ok); the split kernels above for the rest."""

    @staticmethod
    def ok(N, M, D):
        return bool(lib().sv_ge2e_train_ok(N, M, D))

    def prep(self, E, N):
        Nl, M, D = E.shape
        ws = torch.empty(lib().sv_ge2e_workspace_size(Nl, M, D, N) // 4 + 64, dtype=torch.float32, device=E.device)
        ssum = torch.empty((Nl, D), dtype=torch.float32, device=E.device)
        call("sv_ge2e_shard_prep", ptr(E), Nl, M, D, ptr(ssum), ptr(ws), stream_of(E))
        return ssum, ws

    def rows(self, E, s0, N, ssum_all, w, b, ws):
        Nl, M, D = E.shape
        Np = (N + 3) // 4 * 4
        dev = E.device
        per = torch.empty((Nl, M), dtype=torch.float32, device=dev)
        red = torch.empty(Np * D + N, dtype=torch.float32, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        dwdb = torch.empty(2, dtype=torch.float32, device=dev)
        call("sv_ge2e_shard_rows", Nl, M, D, s0, N, ptr(ssum_all), ptr(w), ptr(b), ptr(per), ptr(red), ptr(loss),
             ptr(dwdb), ptr(ws), stream_of(E))
        return loss, per, red, dwdb

    def finalize(self, E, s0, N, red, ws):
        Nl, M, D = E.shape
        dE = torch.empty((Nl, M, D), dtype=torch.float32, device=E.device)
        call("sv_ge2e_shard_finalize", Nl, M, D, s0, N, ptr(red), ptr(dE), ptr(ws), stream_of(E))
        return dE


def all_gather_rows(x, rank, world, group=None):
    """Concatenate every rank's x [n, ...] along dim 0 with all_gather_into_tensor (RCCL; gloo
    for CPU tensors).  Gloo has no device all-gather for GPU tensors: there the equivalent SUM
    all-reduce of a zero-padded buffer."""
    n = x.shape[0]
    if dist.get_backend(group) == "nccl" or not x.is_cuda:
        out = x.new_empty((n * world,) + tuple(x.shape[1:]))
        dist.all_gather_into_tensor(out, x.contiguous(), group=group)
    else:
        out = x.new_zeros((n * world,) + tuple(x.shape[1:]))
        out[rank * n:(rank + 1) * n].copy_(x)
        dist.all_reduce(out, group=group)
    return out


class ShardedGE2E:
    def __init__(self, kernels=None, group=None):
        self.k = kernels if kernels is not None else HipShardKernels()
        self.group = group
        if dist.is_available() and dist.is_initialized():
            self.rank = dist.get_rank(group)
            self.world = dist.get_world_size(group)
        else:
            self.rank, self.world = 0, 1

    def forward(self, E_local, w, b, reduce_loss=True):
        """Returns (loss, per_local, state); loss is the global sum when reduce_loss."""
        Nl, M, D = E_local.shape
        N = Nl * self.world
        s0 = Nl * self.rank
        ssum_local = self.k.speaker_sums(E_local)
        if self.world > 1:
            ssum_all = all_gather_rows(ssum_local, self.rank, self.world, self.group)
        else:
            ssum_all = ssum_local
        loss, per, st = self.k.fwd_rows(E_local, s0, N, ssum_all, w, b)
        if self.world > 1 and reduce_loss:
            loss = loss.clone()
            dist.all_reduce(loss, group=self.group)
        return loss, per, st

    def train(self, E_local, w, b, reduce_loss=True, dwdb_out=None):
        """Forward + backward for the training step (gloss = 1): (loss, dE_local, dwdb_partial[2]);
        the loss is the global sum when reduce_loss, else this shard's partial (the trainer sums
        the partials inside its gradient all-reduce instead of a collective of its own).  One rank
        holding every speaker uses the fused 3-launch kernel (ops.ge2e_train), which writes dwdb
        straight into ``dwdb_out`` when given (the trainer's gradient slot); sharded runs take the
        exchange protocol above."""
        if self.world == 1 and isinstance(self.k, HipShardKernels):
            from .ops import ge2e_train
            loss, _, dE, dwdb = ge2e_train(E_local, w, b, dwdb_out=dwdb_out)
            return loss, dE, dwdb
        Nl, M, D = E_local.shape
        N = Nl * self.world
        if isinstance(self.k, HipShardKernels) and D % 4 == 0 and HipFusedShard.ok(N, M, D):
            # fused sharded form: prep -> all-gather sums -> rows -> all-reduce(dC^, beta) -> dE
            f = HipFusedShard()
            E = E_local.contiguous()
            s0 = Nl * self.rank
            ssum_local, ws = f.prep(E, N)
            ssum_all = all_gather_rows(ssum_local, self.rank, self.world, self.group)
            loss, _, red, dwdb = f.rows(E, s0, N, ssum_all, w.contiguous(), b.contiguous(), ws)
            dist.all_reduce(red, group=self.group)
            dE = f.finalize(E, s0, N, red, ws)
            if reduce_loss:
                loss = loss.clone()
                dist.all_reduce(loss, group=self.group)
            return loss, dE, dwdb
        loss, _, st = self.forward(E_local, w, b, reduce_loss=reduce_loss)
        dE, dwdb = self.backward(st, w, b)
        return loss, dE, dwdb

    def backward(self, st, w, b, gloss=None):
        """Returns (dE_local, dwdb_partial[2]).  dwdb must still be summed over ranks."""
        red, dwdb = self.k.bwd_rows(st, w, b, gloss)
        if self.world > 1:
            dist.all_reduce(red, group=self.group)
        return self.k.finalize(st, red), dwdb

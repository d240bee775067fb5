"""Fused GE2E training step (the body of train_speech_embedder.py:44-65) on the HIP kernels.

One ``GE2ETrainer.step(x)`` = SpeechEmbedder forward -> GE2E loss -> closed-form GE2E
backward -> LSTM/projection backward -> (data-parallel: SUM all-reduce of gradients over
RCCL) -> clip_grad_norm_(net, 3.0) + clip_grad_norm_([w, b], 1.0) + SGD(lr), with no
autograd graph and no host synchronisation.  Numerically the same step as the reference
loop body (the reference's random perm/unperm of rows is value-neutral: rows are
independent, SURVEY §8 a-J).

Parameters are flattened into one device buffer (the module's nn.Parameters become views
of it, so state_dict(), optimizers and checkpoints keep working) so that the gradient
all-reduce and the clip+SGD update each touch one contiguous buffer:

    flat_p = [ net params (n, padded to n_pad = 4k) | w | b | pad pad | 4 words ]   flat_g likewise;
    the last 4 words of flat_g ride along the head all-reduce bucket (data parallel): the two
    status flags of the persistent recurrences and this rank's loss partial (summed, the
    global loss), so neither needs a collective of its own.

Data parallel: one process per GPU; rank r holds speakers [r*N, (r+1)*N) of a global
batch of world*N speakers (ShardedGE2E), so the step is the single-GPU step of that
global batch.  The gradient SUM all-reduce is bucketed by readiness:
bucket L = projection + pad + {w, b}, then one bucket per LSTM layer, top layer first, each
launched on a communication stream as soon as the backward's per-layer completion event
fires; the clip + SGD kernel waits for all buckets.  Per-step schedules: bucket L goes before
the BPTT starts and RCCL traffic overlaps the lower layers' BPTT.  Persistent schedules (no
collective may run beside a persistent grid): bucket L and the upper layers' buckets go once
the last recurrence is done, overlapping layer 0's weight-gradient GEMMs.

Failure surfacing (the reference never steps on wrong gradients, train_speech_embedder.py:61-65):
the persistent recurrences (fp32 and bf16) synchronise through this trainer's own sync block
(``self.status``, include/sv_ge2e.h).  If a hand-off wait times out, the block's sticky status
is set, the clip + SGD kernels skip the update on the device, the returned loss is NaN, and the
next ``step()`` (or ``check()``) raises PersistentRecurrenceError -- read through an async
device-to-pinned copy, so the steady state never synchronises the host.  Data parallel: each
rank's status bits travel as flags in the head gradient bucket (SUM all-reduce) and are merged
back into every rank's status before clip + SGD, so a timeout on one rank skips the update on
all ranks and every rank raises.  After handling the error, ``reset_status()`` clears the block.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ._lib import PersistStatus, call, ptr, stream_of
from .ops import (clip_sgd_step2_, embedder_backward, embedder_backward_bf16, embedder_forward,
                  embedder_forward_bf16)
from .sharded_ge2e import ShardedGE2E


def bf16_row_chunks(B, H, schedule="auto", L=3, T=160, F=40):
    """Row ranges of the bf16 LSTM stack.  A batch too large for the co-resident persistent
    recurrences (sv_persist_fwd_ok / sv_persist_bwd_ok: B > 672 at H = 768, e.g. c5 split over 2
    GPUs = 1280 rows per rank) runs as k equal row chunks that each fit, one after another (every
    chunk's recurrences have the whole chip), instead of the per-step kernels (c5 at 2 GPUs: 48.3
    ms per step on those, profiles/r03_v6_rank_shapes.txt).  Rows are independent in the LSTM, so
    only the weight gradients change: their sums over rows split into k partial sums (bf16-level,
    tested against the bf16 oracle).  A batch up to twice what the one-launch layer wavefront takes
    (sv_wave_ok: 96 rows) runs as two wavefront halves: c4 over 4 GPUs, 160 rows, otherwise takes the
    per-layer persistent kernels on 120 of the 256 CUs.  Under schedule 'auto' only; [(0, B)] when B
    fits or no chunking helps."""
    from ._lib import lib
    if schedule != "auto" or B <= 0:
        return [(0, B)]
    lb = lib()
    wave = lambda b: bool(lb.sv_wave_ok(L, T, b, F, H))  # noqa: E731
    fits = lambda b: bool(lb.sv_persist_fwd_ok(b, H)) and bool(lb.sv_persist_bwd_ok(b, H))  # noqa: E731
    if wave(B):
        return [(0, B)]
    if wave((B + 1) // 2):
        return [(0, (B + 1) // 2), ((B + 1) // 2, B)]
    if fits(B):
        return [(0, B)]
    for k in range(2, 9):
        c = (B + k - 1) // k
        if fits(c):
            return [(i * c, min(B, (i + 1) * c)) for i in range(k) if i * c < B]
    return [(0, B)]


class GE2ETrainer:
    def __init__(self, embedder, ge2e_loss, lr=0.01, clip_net=3.0, clip_wb=1.0, group=None, write_grads=True):
        self.net = embedder
        self.loss_mod = ge2e_loss
        self.lr, self.clip_net, self.clip_wb = float(lr), float(clip_net), float(clip_wb)
        self.group = group
        self.write_grads = write_grads
        self.ge2e = ShardedGE2E(group=group)
        # the data-parallel machinery (comm stream, bucketed SUM all-reduce from the backward's
        # events, status flags): on whenever the group has more than one rank; a world-1 process
        # group may switch it on to run the collectives on one GPU (tests/test_gpu_rccl.py)
        self.dp = self.ge2e.world > 1
        self.status = None
        self._flatten()
        if self.ge2e.world > 1:
            # every rank starts from rank 0's parameters (as DDP does), so SUM-reduced gradients
            # update identical replicas even if the ranks' inits differed; only here, where every
            # rank takes part (a later re-flatten after a device move is rank-local)
            dist.broadcast(self.flat_p, src=dist.get_global_rank(self.group, 0) if self.group is not None else 0,
                           group=self.group)

    # -------------------------------------------------------------------------------------
    def _flatten(self):
        params = self.net.flat_params()
        dev = params[0].device
        n = sum(p.numel() for p in params)
        n_pad = (n + 3) // 4 * 4
        self.n, self.n_pad = n, n_pad
        flat_p = torch.zeros(n_pad + 8, dtype=torch.float32, device=dev)
        flat_g = torch.zeros(n_pad + 8, dtype=torch.float32, device=dev)
        off = 0
        self.grad_views = []
        with torch.no_grad():
            for p in params:
                k = p.numel()
                flat_p[off:off + k].copy_(p.reshape(-1))
                p.data = flat_p[off:off + k].view_as(p)
                g = flat_g[off:off + k].view_as(p)
                self.grad_views.append(g)
                if self.write_grads:
                    p.grad = g
                off += k
            w, b = self.loss_mod.w, self.loss_mod.b
            flat_p[n_pad] = w.detach()
            flat_p[n_pad + 1] = b.detach()
            w.data = flat_p[n_pad:n_pad + 1].view(())
            b.data = flat_p[n_pad + 1:n_pad + 2].view(())
            if self.write_grads:
                w.grad = flat_g[n_pad:n_pad + 1].view(())
                b.grad = flat_g[n_pad + 1:n_pad + 2].view(())
        self.flat_p, self.flat_g = flat_p, flat_g
        self.flags = flat_g[n_pad + 4:n_pad + 6]      # status flags (sv_status_to_flag / _merge)
        self.loss_word = flat_g[n_pad + 6:n_pad + 7]  # this rank's loss partial -> the global loss
        if self.status is None or self.status.block.device != dev:
            self.status = PersistStatus(dev)
        self._ptrs = [p.data_ptr() for p in params]
        # all-reduce buckets: [off(layer l), off(layer l+1)) per layer; the head bucket runs
        # from the projection weight to the end (proj w, proj b, pad, w, b, pad)
        offs = [0]
        for p in params:
            offs.append(offs[-1] + p.numel())
        L = len(params) // 4
        self.buckets = [(offs[4 * l], offs[4 * l + 4]) for l in range(L)] + [(offs[4 * L], n_pad + 8)]
        self._comm = None

    def _check_layout(self):
        if [p.data_ptr() for p in self.net.flat_params()] != self._ptrs:
            self._flatten()  # the module was moved / reloaded since

    # -------------------------------------------------------------------------------------
    def check(self):
        """Wait for every step enqueued so far and raise PersistentRecurrenceError if one of
        them had a persistent-recurrence timeout."""
        self.status.poll(wait=True)

    def reset_status(self):
        """After a PersistentRecurrenceError: wait for the device, then clear the sticky status so
        the next step() updates again (the skipped step is not replayed).  Data parallel: every
        rank calls it (each raised)."""
        torch.cuda.synchronize(self.flat_p.device)
        self.status.clear()

    def step(self, x, N, M, probe=None):
        """x: [N*M, T, nmels] float32 on this rank's GPU (this rank's N speakers x M
        utterances, speaker-major).  Returns the (global) loss as a 0-dim device tensor.
        probe (bench only): {"fwd": events, "bwd": events, "kstamp": tensor} timing probes handed
        to the stack forward / backward (include/sv_ge2e.h)."""
        probe = probe or {}
        self.status.poll()  # raises if an earlier step's recurrences timed out
        self._check_layout()
        net = self.net
        layers = net.LSTM_stack.layer_params()
        w_p, b_p = net.projection.weight, net.projection.bias
        w, b = self.loss_mod.w, self.loss_mod.b
        bf16 = getattr(net, "precision", "f32") == "bf16"
        products = getattr(net, "f32_products", "mfma_f32")
        schedule = getattr(net, "schedule", "auto")
        chunks = (bf16_row_chunks(x.shape[0], layers[0][1].shape[1], schedule, len(layers), x.shape[1], x.shape[2])
                  if bf16 else [(0, x.shape[0])])
        if bf16 and len(chunks) > 1:
            xf = x.float()
            outs = [embedder_forward_bf16(xf[r0:r1].contiguous(), layers, w_p, b_p, status=self.status,
                                          probe=probe.get("fwd") if i == 0 else None, schedule=schedule)
                    for i, (r0, r1) in enumerate(chunks)]
            emb = torch.cat([o[0] for o in outs])
            st = [o[1] for o in outs]
        elif bf16:
            emb, st = embedder_forward_bf16(x.float().contiguous(), layers, w_p, b_p, status=self.status,
                                            probe=probe.get("fwd"), schedule=schedule)
        else:
            emb, st = embedder_forward(x.float().contiguous(), layers, w_p, b_p, products=products,
                                       status=self.status, probe=probe.get("fwd"), schedule=schedule)
        E = emb.view(N, M, emb.shape[1])
        dp = self.dp
        # data parallel: the local loss partial goes to the head bucket's all-reduce (no collective)
        gslot = self.flat_g[self.n_pad:self.n_pad + 2]  # dL/dw, dL/db
        loss, dE, dwdb = self.ge2e.train(E, w, b, reduce_loss=not dp, dwdb_out=gslot)
        if dwdb.data_ptr() != gslot.data_ptr():  # (the split / sharded paths return their own)
            gslot.copy_(dwdb)
        works = []
        ready = None
        if dp:
            self.loss_word.copy_(loss.reshape(1))
            main = torch.cuda.current_stream(x.device)
            if self._comm is None:
                self._comm = torch.cuda.Stream(device=x.device)
            comm = self._comm

            def ready(k, event):
                lo, hi = self.buckets[k]
                if event is None:
                    comm.wait_stream(main)
                else:
                    comm.wait_event(event)
                with torch.cuda.stream(comm):  # SUM, never mean (SURVEY §7 hard part 4)
                    if k == len(self.buckets) - 1:
                        # the status bits go along as flags, converted on the comm stream behind the
                        # head bucket's event: under the persistent schedules that event follows the
                        # last recurrence, so the word is final (the per-step schedules never set it)
                        call("sv_status_to_flag", self.status.ptr(), ptr(self.flags), stream_of(self.flags))
                    works.append(dist.all_reduce(self.flat_g[lo:hi], group=self.group, async_op=True))
        if bf16 and len(chunks) > 1:
            # chunk 0 writes the gradient buffer, the others a scratch copy added into it; the
            # buckets go once the sum is complete
            dEf = dE.view(N * M, -1)
            if (getattr(self, "_gtmp", None) is None or self._gtmp.shape != self.flat_g.shape
                    or self._gtmp.device != self.flat_g.device):
                self._gtmp = torch.zeros_like(self.flat_g)
                off, self._gtmp_views = 0, []
                for g in self.grad_views:
                    self._gtmp_views.append(self._gtmp[off:off + g.numel()].view_as(g))
                    off += g.numel()
            for i, (r0, r1) in enumerate(chunks):
                embedder_backward_bf16(st[i], dEf[r0:r1], layers, w_p,
                                       grads=self.grad_views if i == 0 else self._gtmp_views,
                                       status=self.status, probe=probe.get("bwd") if i == 0 else None,
                                       schedule=schedule)
                if i > 0:
                    self.flat_g[:self.n].add_(self._gtmp[:self.n])
            if ready:
                for k in range(len(self.buckets) - 1, -1, -1):
                    ready(k, None)
        elif bf16:
            embedder_backward_bf16(st, dE.view(N * M, -1), layers, w_p, grads=self.grad_views, grad_ready=ready,
                                   status=self.status, probe=probe.get("bwd"), schedule=schedule)
        else:
            embedder_backward(st, dE.view(N * M, -1), layers, w_p, grads=self.grad_views, grad_ready=ready,
                              products=products, probe=probe.get("bwd"), kstamp=probe.get("kstamp"),
                              status=self.status, schedule=schedule)
        for wk in works:
            wk.wait()  # the current (main) stream waits for every bucket
        if dp:
            loss = self.loss_word.reshape(())  # the sum of every rank's partial
            # any rank's timeout -> this rank's status too: every rank skips the update
            call("sv_status_merge", self.status.ptr(), ptr(self.flags), stream_of(self.flags))
        n = self.n_pad
        # clip_grad_norm_ x2 + SGD (train_speech_embedder.py:63-65): both groups in one launch pair,
        # the second also the step's report -- NaN loss on a timeout, and the status word to a pinned
        # host slot (no copy, no event, no launch of its own)
        loss = loss.clone() if dp else loss  # (not a view of flat_g, which the next step reuses)
        clip_sgd_step2_(self.flat_p[:n], self.flat_g[:n], self.clip_net, self.flat_p[n:n + 4], self.flat_g[n:n + 4],
                        self.clip_wb, self.lr, self.write_grads, status=self.status, report=loss)
        return loss

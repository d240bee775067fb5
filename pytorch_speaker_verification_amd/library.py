"""``torch.library`` custom ops over the C ABI: the hot path's forward and
backward as dispatcher-visible operators, so that fake tensors, ``make_fx`` / ``torch.export``
tracing and ``torch.compile`` (dynamo + AOT autograd) see them as single ops with known output
shapes instead of opaque Python.

    sv::speech_embedder(x, params, precision, schedule) -> emb
        SpeechEmbedder.forward (speech_embedder_net.py:27-33): frames [B,T,F] -> unit-norm [B,P]
    sv::speech_embedder_backward(x, params, demb, precision, schedule, need_dx) -> [dx, *grads]
        its backward (train_speech_embedder.py:62); it runs the forward again with the activations
        saved, then the BPTT kernels -- activation recomputation, as torch.utils.checkpoint does,
        because a custom op's outputs must be tensors and the saved state is ~6 GB of them at c2
    sv::ge2e_loss(E, w, b) -> (loss, per)
        GE2ELoss.forward (speech_embedder_net.py:43-49, utils.py:27-132)
    sv::ge2e_loss_backward(E, w, b, gloss) -> (dE, dw, db)
        its closed-form backward (SURVEY §8 a-G); recomputes the GE2E forward (~20 us)

Autograd is registered on the forward ops (``register_autograd``), fake implementations on all
four (``register_fake``).  The module path (``SpeechEmbedder`` / ``GE2ELoss`` with their default
``dispatch = "function"``) keeps the torch.autograd.Function forms in ops.py, which hold the
forward's activations for the backward instead of recomputing them; ``dispatch = "library"``
routes a module through these ops.  Both run the same kernels: the embeddings are bit-identical
and the gradients agree to the GE2E / BPTT kernels' own determinism (tests/test_library*.py).
"""
from __future__ import annotations

from typing import List, Tuple

import torch
from torch import Tensor

from . import ops
from ._lib import PersistStatus, call, ptr, stream_of

_PRECISIONS = ("f32", "bf16")


def _layers(params: List[Tensor]):
    if len(params) < 6 or (len(params) - 2) % 4:
        raise ValueError("sv::speech_embedder: params = (w_ih, w_hh, b_ih, b_hh) per layer + (w_p, b_p)")
    L = (len(params) - 2) // 4
    return [tuple(params[4 * l:4 * l + 4]) for l in range(L)], params[4 * L], params[4 * L + 1]


def _forward(x, params, precision, schedule, save, status):
    if precision not in _PRECISIONS:
        raise ValueError(f"precision must be one of {_PRECISIONS}, got {precision!r}")
    layers, w_p, b_p = _layers(params)
    if precision == "bf16":
        return ops.embedder_forward_bf16(x.contiguous(), layers, w_p, b_p, save=save, status=status, schedule=schedule)
    return ops.embedder_forward(x.contiguous(), layers, w_p, b_p, save=save, status=status, schedule=schedule)


@torch.library.custom_op("sv::speech_embedder", mutates_args=(), device_types="cuda")
def speech_embedder(x: Tensor, params: List[Tensor], precision: str, schedule: str) -> Tensor:
    ops.check_persistent_status()  # earlier calls' completed checks (as EmbedderFunction.forward)
    status = PersistStatus(x.device)
    emb, _ = _forward(x.float(), params, precision, schedule, False, status)
    status.arm()
    ops._UNCHECKED.append(status)  # a hand-off timeout raises at the next check_persistent_status()
    return emb


@speech_embedder.register_fake
def _(x, params, precision, schedule):
    return x.new_empty((x.shape[0], params[-2].shape[0]), dtype=torch.float32)


@torch.library.custom_op("sv::speech_embedder_backward", mutates_args=(), device_types="cuda")
def speech_embedder_backward(x: Tensor, params: List[Tensor], demb: Tensor, precision: str, schedule: str,
                             need_dx: bool) -> List[Tensor]:
    status = PersistStatus(x.device)
    _, st = _forward(x.float(), params, precision, schedule, True, status)
    layers, w_p, _ = _layers(params)
    grads, flat = ops._flat_grads(params, demb.device)
    if precision == "bf16":
        out = ops.embedder_backward_bf16(st, demb.contiguous(), layers, w_p, grads=grads, status=status,
                                         schedule=schedule, need_dx=need_dx)
    else:
        out = ops.embedder_backward(st, demb.contiguous(), layers, w_p, grads=grads, need_dx=need_dx,
                                    status=status, schedule=schedule)
    call("sv_status_poison", status.ptr(), ptr(flat), flat.numel(), stream_of(flat))  # NaN on a timeout
    status.arm()
    ops._UNCHECKED.append(status)
    grads, dx = out if need_dx else (out, None)
    # outputs may not alias each other: the gradients are views of one flat buffer
    return [dx if dx is not None else x.new_empty((0,))] + [g.clone() for g in grads]


@speech_embedder_backward.register_fake
def _(x, params, demb, precision, schedule, need_dx):
    dx = x.new_empty(x.shape, dtype=torch.float32) if need_dx else x.new_empty((0,))
    return [dx] + [torch.empty_like(p) for p in params]


def _emb_setup(ctx, inputs, output):
    x, params, precision, schedule = inputs
    ctx.save_for_backward(x, *params)
    ctx.precision, ctx.schedule = precision, schedule


def _emb_backward(ctx, demb):
    x, *params = ctx.saved_tensors
    need_dx = ctx.needs_input_grad[0]
    out = speech_embedder_backward(x, params, demb, ctx.precision, ctx.schedule, need_dx)
    return (out[0] if need_dx else None), list(out[1:]), None, None


speech_embedder.register_autograd(_emb_backward, setup_context=_emb_setup)


@torch.library.custom_op("sv::ge2e_loss", mutates_args=(), device_types="cuda")
def ge2e_loss(E: Tensor, w: Tensor, b: Tensor) -> Tuple[Tensor, Tensor]:
    loss, per, _ = ops.ge2e_forward(E.contiguous(), w, b)
    return loss, per


@ge2e_loss.register_fake
def _(E, w, b):
    return E.new_empty((), dtype=torch.float32), E.new_empty(E.shape[:2], dtype=torch.float32)


@torch.library.custom_op("sv::ge2e_loss_backward", mutates_args=(), device_types="cuda")
def ge2e_loss_backward(E: Tensor, w: Tensor, b: Tensor, gloss: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    _, _, st = ops.ge2e_forward(E.contiguous(), w, b)
    dE, dw, db = ops.ge2e_backward(st, w, b, gloss.reshape(()).to(torch.float32))
    return dE, dw.reshape(w.shape).clone(), db.reshape(b.shape).clone()


@ge2e_loss_backward.register_fake
def _(E, w, b, gloss):
    return torch.empty_like(E, dtype=torch.float32), torch.empty_like(w), torch.empty_like(b)


def _ge2e_setup(ctx, inputs, output):
    ctx.save_for_backward(*inputs)


def _ge2e_backward(ctx, gloss, _gper):
    E, w, b = ctx.saved_tensors
    return ge2e_loss_backward(E, w, b, gloss)


ge2e_loss.register_autograd(_ge2e_backward, setup_context=_ge2e_setup)

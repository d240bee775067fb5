"""Drop-in ``speech_embedder_net`` module (reference: speech_embedder_net.py:1-49).

Same public surface -- ``SpeechEmbedder()``, ``GE2ELoss(device)``, and the re-exported
``get_centroids``, ``get_cossim``, ``calc_loss`` (:13) -- same parameter names, init and
state_dict keys, so checkpoints and the reference's train_speech_embedder.py work
unchanged.  The arithmetic runs in the gfx950 HIP kernels of libsv_ge2e.so
(pytorch_speaker_verification_amd.ops).  A module left on the CPU (the reference's test() never
moves its net, train_speech_embedder.py:100-102,120-121) still computes there: its inputs and
parameters make a differentiable round trip to the current GPU and the result comes back.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from ._lib import compute_device
from .hparam import hparam as hp
from .ops import EmbedderFunction, GE2EFunction
from .utils import calc_loss, get_centroids, get_cossim  # noqa: F401  (re-exports, as :13)


class LSTMStack(nn.Module):
    """Parameter container with nn.LSTM's names, shapes, registration order and default
    init (RNNBase.reset_parameters: U(-1/sqrt(H), 1/sqrt(H)) in registration order), so that
    under the same torch seed it holds exactly the reference's nn.LSTM weights.  Its
    forward is the HIP LSTM (batch_first, h0 = c0 = 0), returning the full output only
    through SpeechEmbedder; it is not an nn.LSTM replacement outside that use."""

    def __init__(self, input_size, hidden_size, num_layers=1, batch_first=True):
        super().__init__()
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        self.batch_first = batch_first
        for l in range(num_layers):
            inp = input_size if l == 0 else hidden_size
            setattr(self, f"weight_ih_l{l}", nn.Parameter(torch.empty(4 * hidden_size, inp)))
            setattr(self, f"weight_hh_l{l}", nn.Parameter(torch.empty(4 * hidden_size, hidden_size)))
            setattr(self, f"bias_ih_l{l}", nn.Parameter(torch.empty(4 * hidden_size)))
            setattr(self, f"bias_hh_l{l}", nn.Parameter(torch.empty(4 * hidden_size)))
        self.reset_parameters()

    def reset_parameters(self):
        stdv = 1.0 / math.sqrt(self.hidden_size)
        for w in self.parameters():
            nn.init.uniform_(w, -stdv, stdv)

    def layer_params(self):
        return [(getattr(self, f"weight_ih_l{l}"), getattr(self, f"weight_hh_l{l}"),
                 getattr(self, f"bias_ih_l{l}"), getattr(self, f"bias_hh_l{l}")) for l in range(self.num_layers)]


class SpeechEmbedder(nn.Module):
    """3-layer LSTM d-vector net (speech_embedder_net.py:15-33): frames [B,T,nmels] ->
    unit-norm embeddings [B,proj]."""

    def __init__(self):
        super().__init__()
        self.LSTM_stack = LSTMStack(hp.data.nmels, hp.model.hidden, num_layers=hp.model.num_layer, batch_first=True)
        for name, param in self.LSTM_stack.named_parameters():  # :20-24
            if "bias" in name:
                nn.init.constant_(param, 0.0)
            elif "weight" in name:
                nn.init.xavier_normal_(param)
        self.projection = nn.Linear(hp.model.hidden, hp.model.proj)  # :25
        # "f32" (exact fp32 MFMA, configs c1/c2) or "bf16" (bf16 GEMM operands, fp32
        # accumulation / state / loss, config c3).  Not part of the state_dict.
        self.precision = "f32"
        # fp32 product mode of the f32 path: "mfma_f32" (exact) or "bf16x6" (ops.F32_PRODUCT_MODES)
        self.f32_products = "mfma_f32"
        # bf16 stack schedule: "auto" (measured default), "per_layer", "per_step" or "persist"
        # (the SV_SCHED_* flags of include/sv_ge2e.h, passed on every call)
        self.schedule = "auto"
        # "function": ops.EmbedderFunction (the backward reads the forward's saved activations);
        # "library": the torch.library op sv::speech_embedder (library.py: visible to fake tensors,
        # make_fx and torch.compile; its backward recomputes the forward, fp32 exact products only)
        self.dispatch = "function"

    def flat_params(self):
        """Parameters in kernel order: (w_ih, w_hh, b_ih, b_hh) per layer, then w_p, b_p."""
        ps = [t for lp in self.LSTM_stack.layer_params() for t in lp]
        return ps + [self.projection.weight, self.projection.bias]

    def forward(self, x):
        # x.float() (:28) -> LSTM -> last frame (:30) -> projection (:31) -> x/|x| (:32)
        params = self.flat_params()
        dev = compute_device(params[0])
        host = None if params[0].is_cuda else params[0].device
        if host is not None:  # CPU-resident module: differentiable copies to the GPU and back
            params = [p.to(dev) for p in params]
        if self.dispatch == "library":
            from . import library
            out = library.speech_embedder(x.float().to(dev).contiguous(), params, self.precision, self.schedule)
        else:
            out = EmbedderFunction.apply(x.float().to(dev).contiguous(), self.LSTM_stack.num_layers, self.precision,
                                         self.f32_products, self.schedule, *params)
        return out if host is None else out.to(host)


class GE2ELoss(nn.Module):
    """GE2E softmax loss (speech_embedder_net.py:35-49) with learnable w=10, b=-5.

    The reference's ``torch.clamp(self.w, 1e-6)`` discards its result (:44),
    so it is a no-op and is not reproduced.  The loss is the SUM over all N*M rows."""

    def __init__(self, device):
        super().__init__()
        self.w = nn.Parameter(torch.tensor(10.0).to(device), requires_grad=True)
        self.b = nn.Parameter(torch.tensor(-5.0).to(device), requires_grad=True)
        self.device = device
        self.dispatch = "function"  # or "library": the torch.library op sv::ge2e_loss (library.py)

    def forward(self, embeddings):
        dev = compute_device(self.w)
        if self.dispatch == "library":
            from . import library
            fn = library.ge2e_loss
        else:
            fn = GE2EFunction.apply
        if self.w.is_cuda:
            loss, _ = fn(embeddings.to(dev).contiguous(), self.w, self.b)
            return loss
        loss, _ = fn(embeddings.to(dev).contiguous(), self.w.to(dev), self.b.to(dev))
        return loss.to(self.w.device)

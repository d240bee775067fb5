"""Torch-facing wrappers over the C ABI (include/sv_ge2e.h).

PyTorch supplies device memory (caching allocator), the current HIP stream and autograd
plumbing; every FLOP of the path runs in the HIP kernels of libsv_ge2e.so.

  embedder_forward / embedder_backward   SpeechEmbedder.forward (speech_embedder_net.py:27-33)
                                         and its backward: 3-layer LSTM + Linear + L2 norm
  ge2e_forward / ge2e_backward           GE2ELoss.forward (speech_embedder_net.py:43-49)
  EmbedderFunction, GE2EFunction         autograd.Function glue (loss.backward() works)
  clip_sgd_step_                         clip_grad_norm_ + SGD.step (train_speech_embedder.py:63-65)
  clip_sgd_step2_                        the same over both parameter groups in one launch pair
"""
from __future__ import annotations

import ctypes

import torch

from ._lib import (SV_DTYPE_BF16, SV_DTYPE_F32, SV_SCHED_CNT_READY, SV_SCHED_NO_EVENTS, SV_SCHED_WT_READY,
                   PersistStatus, call, lib, ptr, require_device, schedule_flags, stream_of)

# timesteps per chunk of the layer-pipelined schedules (measured at c2: 16 / 24 / 32 / 48 / 64 ->
# 69.3 / 69.7 / 69.1 / 69.5 / 69.6 ms per step)
PIPELINE_CHUNK = 32

# how the fp32 path forms its products (the `products` argument of the C ABI, include/sv_ge2e.h):
# "mfma_f32" (default, exact fp32 MFMA) or "bf16x6" (three-way bf16 split, six bf16 MFMA products
# per fp32 product, fp32 accumulation).  Per call, never process-wide.
F32_PRODUCT_MODES = {"mfma_f32": 0, "bf16x6": 1}


def _products(mode):
    try:
        return F32_PRODUCT_MODES[mode or "mfma_f32"]
    except KeyError:
        raise ValueError(f"unknown fp32 product mode {mode!r} (expected one of {sorted(F32_PRODUCT_MODES)})") from None


# sync blocks of bf16 calls made without a caller-owned one (autograd path): their status is
# checked (non-blocking) at the next call and by check_persistent_status()
_UNCHECKED = []


def _own_status(status, device):
    if status is not None:
        return status, False
    check_persistent_status()
    return PersistStatus(device), True


def _release_status(st, own):
    if own:
        st.arm()
        _UNCHECKED.append(st)


def check_persistent_status(wait=False):
    """Raise PersistentRecurrenceError if a persistent recurrence of an earlier call (made
    without a caller-owned sync block) timed out; wait=True waits for all of them first."""
    global _UNCHECKED
    pending = _UNCHECKED
    _UNCHECKED = []
    err = None
    for st in pending:
        try:
            st.poll(wait=wait)
        except RuntimeError as e:
            err = err or e
        if st._pending:
            _UNCHECKED.append(st)
    if err:
        raise err


class _StreamPool:
    """Side streams + events for the layer-pipelined schedules, one set per (device, role): the
    forward and the backward of a step keep separate sets, and a set only ever grows -- an event
    a call recorded is never destroyed while later work on `main` may still wait on it."""
    _pools = {}

    @classmethod
    def get(cls, device, role, n_streams, n_events):
        key = (device.index, role, n_streams)
        p = cls._pools.get(key)
        if p is None:
            p = ([torch.cuda.Stream(device=device) for _ in range(n_streams)], [])
            cls._pools[key] = p
        streams, events = p
        if len(events) < n_events:
            with torch.cuda.device(device):
                for _ in range(n_events - len(events)):
                    e = torch.cuda.Event()
                    e.record()  # materialise the native event
                    events.append(e)
        return p


def _parr(ts):
    return (ctypes.c_void_p * len(ts))(*[ptr(t) if t is not None else None for t in ts])


def _evarr(events):
    """Host array of native HIP events (timing probes), or NULL."""
    if not events:
        return None
    return (ctypes.c_void_p * len(events))(*[e.cuda_event for e in events])


def _ws(nbytes, device):
    """Workspace of at least nbytes (fp32 storage, 256-byte aligned by the allocator)."""
    n = max(1, (int(nbytes) + 3) // 4)
    return torch.empty(n, dtype=torch.float32, device=device)


# ----------------------------------------------------------------------------- LSTM stack
class EmbedderState:
    """Activations saved by the forward for the backward (all time-major, fp32)."""

    def __init__(self):
        self.x_tm = []      # per layer input [T,B,F_l]
        self.gates = []     # per layer [T,B,4H] activated i,f,g,o
        self.c_tm = []      # per layer [T,B,H]
        self.h_tm = []      # per layer [T+1,B,H]
        self.hT = []        # per layer [H,(T+1)B]  (h^T, column block t+1 = h_t, block 0 = 0)
        self.xT0 = None     # layer-0 input transposed [F, T*B]
        self.y = self.emb = self.ynorm = self.h_last = None
        self.T = self.B = self.H = self.P = 0
        self.bf16 = False
        self.bws = None     # bf16: the stacked backward's workspace, its weight transposes already in


def embedder_forward(x, layers, w_p, b_p, save=True, products="mfma_f32", status=None, probe=None, schedule="auto"):
    """x [B,T,F] float32 (batch_first); layers = [(w_ih, w_hh, b_ih, b_hh)] * L.
    Returns (emb [B,P], state).  products: fp32 product mode of the stack (F32_PRODUCT_MODES).
    schedule: 'auto' (the persistent recurrences where they fill the device, sv_lstm_f32_persist_ok),
    'per_step' (layer-pipelined K2 steps) or 'persist'; status: the caller's PersistStatus (sync
    block of the persistent recurrences; None = a fresh one, checked at the next call / by
    check_persistent_status()); probe: 2*L events around the layers' persistent launches."""
    prod = _products(products)
    sched = schedule_flags(schedule)
    require_device(x, w_p, b_p, *[t for l in layers for t in l])
    B, T, F = x.shape
    H = layers[0][1].shape[1]
    P = w_p.shape[0]
    dev = x.device
    s = stream_of(x)
    st = EmbedderState()
    st.T, st.B, st.H, st.P = T, B, H, P
    x_tm = torch.empty((T, B, F), dtype=torch.float32, device=dev)
    call("sv_frames_to_time_major", ptr(x), ptr(x_tm), B, T, F, s)
    Bp = (B + 3) // 4 * 4
    if save:  # layer-0 input transposed, [F, T*Bp] (column block t = x_t^T, padding columns zero)
        if Bp == B:
            st.xT0 = torch.empty((F, T * B), dtype=torch.float32, device=dev)
            call("sv_transpose", ptr(x_tm), F, T * B, F, ptr(st.xT0), T * B, s)
        else:
            st.xT0 = torch.zeros((F, T * Bp), dtype=torch.float32, device=dev)
            for t in range(T):
                call("sv_transpose", ptr(x_tm[t]), F, B, F, ptr(st.xT0) + 4 * t * Bp, T * Bp, s)
    inp = x_tm
    L = len(layers)
    if PIPELINE_CHUNK > 0 and L > 1:
        gs = [torch.empty((T, B, 4 * H), dtype=torch.float32, device=dev) for _ in range(L)]
        cs = [torch.empty((T, B, H), dtype=torch.float32, device=dev) for _ in range(L)]
        hs = [torch.empty((T + 1, B, H), dtype=torch.float32, device=dev) for _ in range(L)]
        hTs = [torch.empty((H, (T + 1) * Bp), dtype=torch.float32, device=dev) if save else None for _ in range(L)]
        nch = (T + PIPELINE_CHUNK - 1) // PIPELINE_CHUNK
        streams, events = _StreamPool.get(dev, "fwd", L, L * nch + 1)
        sp = (ctypes.c_void_p * L)(*[st_.cuda_stream for st_ in streams])
        ep = (ctypes.c_void_p * (L * nch + 1))(*[e.cuda_event for e in events[:L * nch + 1]])
        ps, own = _own_status(status, dev)
        call("sv_lstm_fwd", SV_DTYPE_F32, L, T, B, F, H, ptr(x_tm), _parr([l[0] for l in layers]),
             _parr([l[1] for l in layers]), _parr([l[2] for l in layers]), _parr([l[3] for l in layers]),
             _parr(gs), _parr(cs), _parr(hs), None, _parr(hTs), PIPELINE_CHUNK, s, sp, ep, prod, sched, ps.ptr(),
             _evarr(probe))
        _release_status(ps, own)
        if save:
            st.x_tm = [x_tm] + [h[1:] for h in hs[:-1]]
            st.gates, st.c_tm, st.h_tm, st.hT = gs, cs, hs, hTs
        layers_done = True
        inp = hs[-1][1:]
    else:
        layers_done = False
    if not layers_done and prod:
        raise ValueError("the bf16x6 product mode runs on the layer-pipelined stack only (SV_PIPELINE_CHUNK > 0, L > 1)")
    for (w_ih, w_hh, b_ih, b_hh) in ([] if layers_done else layers):
        Fl = inp.shape[2]
        gates = torch.empty((T, B, 4 * H), dtype=torch.float32, device=dev)
        c_tm = torch.empty((T, B, H), dtype=torch.float32, device=dev)
        h_tm = torch.empty((T + 1, B, H), dtype=torch.float32, device=dev)
        hT = torch.empty((H, (T + 1) * Bp), dtype=torch.float32, device=dev) if save else None
        call("sv_lstm_layer_fwd", ptr(inp), T, B, Fl, H, ptr(w_ih), ptr(w_hh), ptr(b_ih), ptr(b_hh), ptr(gates),
             ptr(c_tm), ptr(h_tm), ptr(hT), s)
        if save:
            st.x_tm.append(inp)
            st.gates.append(gates)
            st.c_tm.append(c_tm)
            st.h_tm.append(h_tm)
            st.hT.append(hT)
        inp = h_tm[1:]
    h_last = inp[T - 1]
    y = torch.empty((B, P), dtype=torch.float32, device=dev)
    emb = torch.empty((B, P), dtype=torch.float32, device=dev)
    ynorm = torch.empty((B,), dtype=torch.float32, device=dev)
    ws = _ws(lib().sv_proj_norm_workspace(B, H, P), dev)
    call("sv_proj_norm_fwd", ptr(h_last), B, H, P, ptr(w_p), ptr(b_p), ptr(y), ptr(emb), ptr(ynorm), ptr(ws), s)
    st.y, st.emb, st.ynorm, st.h_last = y, emb, ynorm, h_last
    return emb, st


def embedder_backward(st, demb, layers, w_p, grads=None, need_dx=False, grad_ready=None, products="mfma_f32",
                      probe=None, kstamp=None, status=None, schedule="auto"):
    """Backward of embedder_forward.  ``grads`` (optional) is a list of preallocated
    output tensors in parameter order [w_ih, w_hh, b_ih, b_hh]*L + [w_p, b_p]; returns it
    (and dx [B,T,F] if need_dx).

    ``grad_ready(k, event)`` (optional) is called as soon as a gradient group is enqueued:
    k = L for the projection, then k = L-1 .. 0 for the LSTM layers; ``event`` is the HIP
    event that completes it (None: the current stream).  The data-parallel trainer hangs its
    per-layer all-reduce buckets on it so communication overlaps the rest of the BPTT.

    ``probe`` (optional): 2*L*ceil(T/chunk) timing events recorded around one recurrent-step
    launch per chunk; ``kstamp`` (optional): int64 device tensor of 2*L*T slots, pairs preset
    to (-1, 0), set by every recurrent-step launch (l, t) to its start / end on the GPU's 100 MHz
    real-time clock (include/sv_ge2e.h, sv_lstm_stack_bwd).  Under the persistent schedule
    (``schedule``, ``status`` as embedder_forward) probe[2l] / [2l+1] bracket layer l's launch and
    kstamp is not written."""
    prod = _products(products)
    # no grad_ready: nothing waits on the per-layer completion events, so the persistent
    # schedule records none (include/sv_ge2e.h SV_SCHED_NO_EVENTS)
    sched = schedule_flags(schedule) | (0 if grad_ready else SV_SCHED_NO_EVENTS)
    demb = demb.contiguous()
    require_device(demb)
    T, B, H, P = st.T, st.B, st.H, st.P
    dev = demb.device
    s = stream_of(demb)
    L = len(layers)
    if grads is None:
        grads = []
        for (w_ih, w_hh, b_ih, b_hh) in layers:
            grads += [torch.empty_like(w_ih), torch.empty_like(w_hh), torch.empty_like(b_ih), torch.empty_like(b_hh)]
        grads += [torch.empty_like(w_p), torch.empty((P,), dtype=torch.float32, device=dev)]
    dh_last = torch.empty((B, H), dtype=torch.float32, device=dev)
    ws = _ws(lib().sv_proj_norm_workspace(B, H, P), dev)
    call("sv_proj_norm_bwd", ptr(demb), ptr(st.emb), ptr(st.ynorm), ptr(st.h_last), B, H, P, ptr(w_p),
         ptr(grads[4 * L]), ptr(grads[4 * L + 1]), ptr(dh_last), ptr(ws), s)
    stacked = PIPELINE_CHUNK > 0 and L > 1 and not need_dx
    # under the persistent schedule the projection bucket is enqueued behind the stack backward
    # (a collective must not run beside a persistent launch); else it overlaps the BPTT
    with torch.cuda.device(dev):  # (the library answers for the current device)
        late_head = stacked and bool(lib().sv_lstm_f32_persist_ok(B, H, sched))
    if grad_ready and not late_head:
        grad_ready(L, None)
    if prod and not stacked:
        raise ValueError("the bf16x6 product mode runs on the layer-pipelined stack only")
    Fmax = max(st.x_tm[l].shape[2] for l in range(L))
    Bp = (B + 3) // 4 * 4
    if stacked:
        F0 = st.x_tm[0].shape[2]
        ws = _ws(lib().sv_lstm_bwd_workspace(SV_DTYPE_F32, L, T, B, F0, H), dev)
        dgs = [torch.empty((T, B, 4 * H), dtype=torch.float32, device=dev) for _ in range(L)]
        dgTs = [torch.empty((4 * H, T * Bp), dtype=torch.float32, device=dev) for _ in range(L)]
        dxs = [None] + [torch.empty((T, B, H), dtype=torch.float32, device=dev) for _ in range(L - 1)]
        xT = [ptr(st.xT0)] + [ptr(st.hT[l - 1]) + Bp * 4 for l in range(1, L)]
        ld = [T * Bp] + [(T + 1) * Bp] * (L - 1)
        nch = (T + PIPELINE_CHUNK - 1) // PIPELINE_CHUNK
        nev = L * nch + L + 1
        streams, events = _StreamPool.get(dev, "bwd", L, nev)
        ps, own = _own_status(status, dev)
        sp = (ctypes.c_void_p * L)(*[st_.cuda_stream for st_ in streams])
        ep = (ctypes.c_void_p * nev)(*[e.cuda_event for e in events[:nev]])
        call("sv_lstm_bwd", SV_DTYPE_F32, L, T, B, F0, H, (ctypes.c_void_p * L)(*xT), (ctypes.c_long * L)(*ld),
             _parr([l[0] for l in layers]), _parr([l[1] for l in layers]), _parr(st.gates), _parr(st.c_tm),
             _parr(st.hT), ptr(dh_last), _parr(dgs), _parr(dgTs), _parr(dxs),
             _parr([grads[4 * l] for l in range(L)]), _parr([grads[4 * l + 1] for l in range(L)]),
             _parr([grads[4 * l + 2] for l in range(L)]), _parr([grads[4 * l + 3] for l in range(L)]), ptr(ws),
             PIPELINE_CHUNK, s, sp, ep, prod, _evarr(probe), ptr(kstamp) if kstamp is not None else None, sched,
             ps.ptr())
        _release_status(ps, own)
        if grad_ready:
            if late_head:
                # behind the event the library records right after the last recurrence (the status
                # word is final there), not behind all of main: the buckets then overlap layer 0's
                # dx / dW GEMMs
                grad_ready(L, events[L * nch + L - 1] if L > 1 else None)
            for l in range(L - 1, -1, -1):
                grad_ready(l, events[L * nch + l])
        return grads
    ws = _ws(lib().sv_lstm_layer_bwd_workspace(T, B, Fmax, H), dev)
    dgates = torch.empty((T, B, 4 * H), dtype=torch.float32, device=dev)
    dgT = torch.empty((4 * H, T * Bp), dtype=torch.float32, device=dev)
    dh_up, full = dh_last, 0
    dx_out = None
    for l in range(L - 1, -1, -1):
        w_ih, w_hh, _, _ = layers[l]
        Fl = st.x_tm[l].shape[2]
        want_dx = l > 0 or need_dx
        dx = torch.empty((T, B, Fl), dtype=torch.float32, device=dev) if want_dx else None
        if l == 0:
            xT, ld_xT = ptr(st.xT0), T * Bp
        else:  # previous layer's h^T, column blocks 1..T (= h_0 .. h_{T-1})
            xT, ld_xT = ptr(st.hT[l - 1]) + Bp * 4, (T + 1) * Bp
        call("sv_lstm_layer_bwd", T, B, Fl, H, xT, ld_xT, ptr(w_ih), ptr(w_hh), ptr(st.gates[l]),
             ptr(st.c_tm[l]), ptr(st.hT[l]), ptr(dh_up), full, ptr(dgates), ptr(dgT), ptr(dx), ptr(grads[4 * l]),
             ptr(grads[4 * l + 1]), ptr(grads[4 * l + 2]), ptr(grads[4 * l + 3]), ptr(ws), s)
        if grad_ready:
            grad_ready(l, None)
        dh_up, full = dx, 1
        if l == 0:
            dx_out = dx
    if need_dx:
        dxb = torch.empty((B, T, dx_out.shape[2]), dtype=torch.float32, device=dev)
        call("sv_frames_to_time_major", ptr(dx_out), ptr(dxb), T, B, dx_out.shape[2], s)  # [T,B,F] -> [B,T,F]
        return grads, dxb
    return grads


# ----------------------------------------------------------------------------- bf16 operands
def _bf(shape, dev):
    return torch.empty(shape, dtype=torch.bfloat16, device=dev)


def embedder_forward_bf16(x, layers, w_p, b_p, save=True, status=None, probe=None, schedule="auto"):
    """Mixed-precision forward (BASELINE config c3): bf16 GEMM operands, fp32 accumulation,
    bf16 storage of the x-projection and of the activated gates saved for the backward, fp32
    cell state / projection / norm.  Same outputs as embedder_forward.
    status: the caller's PersistStatus (sync block of the persistent recurrences); None = a
    fresh one, checked at the next call / check_persistent_status().  probe: 2*L timing events
    around the layers' persistent recurrences (include/sv_ge2e.h).  schedule: 'auto' (default),
    'per_layer', 'per_step' or 'persist' (the SV_SCHED_* flags of include/sv_ge2e.h)."""
    sched = schedule_flags(schedule)
    require_device(x, w_p, b_p, *[t for l in layers for t in l])
    B, T, F = x.shape
    H = layers[0][1].shape[1]
    P = w_p.shape[0]
    dev = x.device
    s = stream_of(x)
    Bp = (B + 7) // 8 * 8
    st = EmbedderState()
    st.T, st.B, st.H, st.P, st.bf16 = T, B, H, P, True
    x_bf = _bf((T, B, F), dev)
    L = len(layers)
    fused_x = F <= 64
    if save:  # layer 0's dW_ih operand x^T [F][T Bp] (padding columns zero)
        st.xT0 = (torch.empty if fused_x or Bp == B else torch.zeros)((F, T * Bp), dtype=torch.bfloat16, device=dev)
    if fused_x:  # x -> time-major bf16 and x^T: in the weights' launch below (sv_lstm_prep_bf16)
        srcs, dsts = [], []
    else:
        x_tm = torch.empty((T, B, F), dtype=torch.float32, device=dev)
        call("sv_frames_to_time_major", ptr(x), ptr(x_tm), B, T, F, s)
        srcs, dsts = [x_tm], [x_bf]
        if save:
            if Bp == B:
                call("sv_transpose_cast_bf16", ptr(x_tm), F, T * B, F, ptr(st.xT0), T * B, s)
            else:
                for t in range(T):
                    call("sv_transpose_cast_bf16", ptr(x_tm[t]), F, B, F, ptr(st.xT0) + 2 * t * Bp, T * Bp, s)
    if srcs:  # the time-major frames' cast (F > 64)
        call("sv_cast_bf16", ptr(srcs[0]), ptr(dsts[0]), srcs[0].numel(), s)
    # every layer's bf16 weights in one launch (sv_lstm_weights_bf16); when the stacked backward
    # follows, also its weight transposes, into the backward workspace it will be handed
    # (SV_SCHED_WT_READY: the backward launches no transposes)
    wbf = [(_bf(w_ih.shape, dev), _bf(w_hh.shape, dev)) for (w_ih, w_hh, _, _) in layers]
    if save and PIPELINE_CHUNK > 0 and L > 1:
        st.bws = _ws(lib().sv_lstm_bwd_workspace(SV_DTYPE_BF16, L, T, B, F, H), dev)
    wargs = (_parr([l[0] for l in layers]), _parr([l[1] for l in layers]), _parr([w[0] for w in wbf]),
             _parr([w[1] for w in wbf]), ptr(st.bws) if st.bws is not None else None, s)
    if fused_x:  # the frames' part in the same launch (sv_lstm_prep_bf16)
        call("sv_lstm_prep_bf16", L, T, B, F, H, ptr(x), ptr(x_bf), ptr(st.xT0) if save else None, Bp, *wargs)
    else:
        call("sv_lstm_weights_bf16", L, T, B, F, H, *wargs)
    inp = x_bf
    gs = [_bf((T, B, 4 * H), dev) for _ in range(L)]  # bf16 x-projection in, bf16 activations out
    cs = [torch.empty((T, B, H), dtype=torch.float32, device=dev) for _ in range(L)]
    hs = [torch.empty((T + 1, B, H), dtype=torch.float32, device=dev) for _ in range(L)]
    hbs = [_bf((T + 1, B, H), dev) for _ in range(L)]
    hTs = [_bf((H, (T + 1) * Bp), dev) if save else None for _ in range(L)]
    if PIPELINE_CHUNK > 0 and L > 1:
        nch = (T + PIPELINE_CHUNK - 1) // PIPELINE_CHUNK
        streams, events = _StreamPool.get(dev, "fwd", L, L * nch + 1)
        sp = (ctypes.c_void_p * L)(*[st_.cuda_stream for st_ in streams])
        ep = (ctypes.c_void_p * (L * nch + 1))(*[e.cuda_event for e in events[:L * nch + 1]])
        sync, own = _own_status(status, dev)
        call("sv_lstm_fwd", SV_DTYPE_BF16, L, T, B, F, H, ptr(x_bf), _parr([w[0] for w in wbf]),
             _parr([w[1] for w in wbf]), _parr([l[2] for l in layers]), _parr([l[3] for l in layers]),
             _parr(gs), _parr(cs), _parr(hs), _parr(hbs), _parr(hTs), PIPELINE_CHUNK, s, sp, ep, 0, sched,
             sync.ptr(), _evarr(probe))
        sync.bwd_counters_clean = True  # (the stack forward zeroes the backward's channels, every schedule)
        _release_status(sync, own)
    else:
        for l, (w_ih, w_hh, b_ih, b_hh) in enumerate(layers):
            Fl = inp.shape[2]
            call("sv_lstm_layer_fwd_bf16", ptr(inp), T, B, Fl, H, ptr(wbf[l][0]), ptr(wbf[l][1]), ptr(b_ih),
                 ptr(b_hh), ptr(gs[l]), ptr(cs[l]), ptr(hs[l]), ptr(hbs[l]), ptr(hTs[l]), s)
            inp = hbs[l][1:]
    if save:
        st.x_tm = [x_bf] + [h[1:] for h in hbs[:-1]]
        st.gates, st.c_tm, st.h_tm, st.hT = gs, cs, hs, hTs
    h_tm = hs[-1]
    h_last = st.h_tm[-1][T] if save else h_tm[T]
    y = torch.empty((B, P), dtype=torch.float32, device=dev)
    emb = torch.empty((B, P), dtype=torch.float32, device=dev)
    ynorm = torch.empty((B,), dtype=torch.float32, device=dev)
    ws = _ws(lib().sv_proj_norm_workspace(B, H, P), dev)
    call("sv_proj_norm_fwd", ptr(h_last), B, H, P, ptr(w_p), ptr(b_p), ptr(y), ptr(emb), ptr(ynorm), ptr(ws), s)
    st.y, st.emb, st.ynorm, st.h_last = y, emb, ynorm, h_last
    return emb, st


def embedder_forward_dvec_bf16(x, layers, w_p, b_p):
    """Embeddings [B, P] of B windows x [B, T, F] (fp32, batch-first) by sv_dvector_embed_bf16:
    the c3 forward's numerics (bf16 GEMM operands, bf16 input projection with its biases, fp32
    accumulation / state / projection) as one 256 x 256 GEMM launch per timestep and layer with the
    LSTM cell in its epilogue -- the large-batch d-vector path (dvector_create.py:96-101), no
    activations saved and no co-residency requirement."""
    require_device(x, w_p, *[t for l in layers for t in l if t is not None])
    B, T, F = x.shape
    H = layers[0][1].shape[1]
    P = w_p.shape[0]
    L = len(layers)
    x = x.contiguous()
    emb = torch.empty((B, P), dtype=torch.float32, device=x.device)
    ws = _ws(lib().sv_dvector_bf16_workspace(B, T, F, H, L, P), x.device)
    ts = [[l[i].contiguous() if l[i] is not None else None for l in layers] for i in range(4)]  # kept alive
    wih, whh, bih, bhh = (_parr(t) for t in ts)
    call("sv_dvector_embed_bf16", B, T, F, H, L, ptr(x), wih, whh, bih, bhh, ptr(w_p.contiguous()),
         ptr(b_p) if b_p is not None else None, P, ptr(emb), ptr(ws), stream_of(x))
    return emb


def embedder_backward_bf16(st, demb, layers, w_p, grads=None, grad_ready=None, status=None, probe=None,
                           schedule="auto", need_dx=False):
    """Backward of embedder_forward_bf16 (same ``grads`` / ``grad_ready`` contract as
    embedder_backward; ``status`` and ``schedule`` as embedder_forward_bf16).  need_dx: also the
    input gradient dx [B,T,F] (returns (grads, dx)), formed by the per-layer kernels, whose layer-0
    step adds the dx = dG W_ih GEMM (bf16 operands, fp32 accumulation) the stacked schedules skip;
    the per-layer per-step kernels are bit-identical to the persistent ones."""
    sched = schedule_flags(schedule) | (0 if grad_ready else SV_SCHED_NO_EVENTS)  # (as embedder_backward)
    demb = demb.contiguous()
    require_device(demb)
    T, B, H, P = st.T, st.B, st.H, st.P
    dev = demb.device
    s = stream_of(demb)
    L = len(layers)
    Bp = (B + 7) // 8 * 8
    if grads is None:
        grads = []
        for (w_ih, w_hh, b_ih, b_hh) in layers:
            grads += [torch.empty_like(w_ih), torch.empty_like(w_hh), torch.empty_like(b_ih), torch.empty_like(b_hh)]
        grads += [torch.empty_like(w_p), torch.empty((P,), dtype=torch.float32, device=dev)]
    dh_last = torch.empty((B, H), dtype=torch.float32, device=dev)
    ws = _ws(lib().sv_proj_norm_workspace(B, H, P), dev)
    call("sv_proj_norm_bwd", ptr(demb), ptr(st.emb), ptr(st.ynorm), ptr(st.h_last), B, H, P, ptr(w_p),
         ptr(grads[4 * L]), ptr(grads[4 * L + 1]), ptr(dh_last), ptr(ws), s)
    Fmax = max(st.x_tm[l].shape[2] for l in range(L))
    if PIPELINE_CHUNK > 0 and L > 1 and not need_dx:
        F0 = st.x_tm[0].shape[2]
        if st.bws is not None:  # the forward wrote the weight transposes into it (sv_lstm_weights_bf16)
            ws, sched = st.bws, sched | SV_SCHED_WT_READY
        else:
            ws = _ws(lib().sv_lstm_bwd_workspace(SV_DTYPE_BF16, L, T, B, F0, H), dev)
        dgs = [_bf((T, B, 4 * H), dev) for _ in range(L)]
        dgTs = [_bf((4 * H, T * Bp), dev) for _ in range(L)]
        dxs = [None] + [torch.empty((T, B, H), dtype=torch.float32, device=dev) for _ in range(L - 1)]
        xT = [ptr(st.xT0)] + [ptr(st.hT[l - 1]) + Bp * 2 for l in range(1, L)]
        ld = [T * Bp] + [(T + 1) * Bp] * (L - 1)
        nch = (T + PIPELINE_CHUNK - 1) // PIPELINE_CHUNK
        nev = L * nch + L + 1
        streams, events = _StreamPool.get(dev, "bwd", L, nev)
        sp = (ctypes.c_void_p * L)(*[st_.cuda_stream for st_ in streams])
        ep = (ctypes.c_void_p * nev)(*[e.cuda_event for e in events[:nev]])
        sync, own = _own_status(status, dev)
        if sync.bwd_counters_clean:  # the forward zeroed the backward's counters, none used since
            sched |= SV_SCHED_CNT_READY
        sync.bwd_counters_clean = False
        call("sv_lstm_bwd", SV_DTYPE_BF16, L, T, B, F0, H, (ctypes.c_void_p * L)(*xT), (ctypes.c_long * L)(*ld),
             _parr([l[0] for l in layers]), _parr([l[1] for l in layers]), _parr(st.gates), _parr(st.c_tm),
             _parr(st.hT), ptr(dh_last), _parr(dgs), _parr(dgTs), _parr(dxs),
             _parr([grads[4 * l] for l in range(L)]), _parr([grads[4 * l + 1] for l in range(L)]),
             _parr([grads[4 * l + 2] for l in range(L)]), _parr([grads[4 * l + 3] for l in range(L)]), ptr(ws),
             PIPELINE_CHUNK, s, sp, ep, 0, _evarr(probe), None, sched, sync.ptr())
        _release_status(sync, own)
        st.dgT = dgTs  # the weight-gradient GEMMs' A operands (tests check dW against them)
        if grad_ready:
            # the projection bucket is enqueued behind the stack backward: with the persistent
            # recurrences a collective must not run beside them (sv_lstm_stack_bwd_bf16): behind the
            # event recorded once every recurrence (and layer L-1's gradients) is done
            grad_ready(L, events[L * nch + L - 1] if L > 1 else None)
            for l in range(L - 1, -1, -1):
                grad_ready(l, events[L * nch + l])
        return grads
    if grad_ready:
        grad_ready(L, None)
    ws = _ws(lib().sv_lstm_layer_bwd_bf16_workspace(T, B, Fmax, H), dev)
    dg = _bf((T, B, 4 * H), dev)
    dgT = _bf((4 * H, T * Bp), dev)
    whhT = _bf((H, 4 * H), dev)
    dh_up, full = dh_last, 0
    for l in range(L - 1, -1, -1):
        w_ih, w_hh, _, _ = layers[l]
        Fl = st.x_tm[l].shape[2]
        wihT = _bf((Fl, 4 * H), dev)
        call("sv_transpose_cast_bf16", ptr(w_ih), Fl, 4 * H, Fl, ptr(wihT), 4 * H, s)
        call("sv_transpose_cast_bf16", ptr(w_hh), H, 4 * H, H, ptr(whhT), 4 * H, s)
        dx = torch.empty((T, B, Fl), dtype=torch.float32, device=dev) if (l > 0 or need_dx) else None
        if l == 0:
            xT, ld_xT = ptr(st.xT0), T * Bp
        else:
            xT, ld_xT = ptr(st.hT[l - 1]) + 2 * Bp, (T + 1) * Bp
        call("sv_lstm_layer_bwd_bf16", T, B, Fl, H, xT, ld_xT, ptr(wihT), ptr(whhT), ptr(st.gates[l]),
             ptr(st.c_tm[l]), ptr(st.hT[l]), ptr(dh_up), full, ptr(dg), ptr(dgT), ptr(dx), ptr(grads[4 * l]),
             ptr(grads[4 * l + 1]), ptr(grads[4 * l + 2]), ptr(grads[4 * l + 3]), ptr(ws), s)
        if grad_ready:
            grad_ready(l, None)
        dh_up, full = dx, 1
    if need_dx:
        dxb = torch.empty((B, T, dh_up.shape[2]), dtype=torch.float32, device=dev)
        call("sv_frames_to_time_major", ptr(dh_up), ptr(dxb), T, B, dh_up.shape[2], s)  # [T,B,F] -> [B,T,F]
        return grads, dxb
    return grads


def _flat_grads(params, dev):
    """Gradient tensors shaped like params, as views of one flat buffer (returned last)."""
    n = sum(p.numel() for p in params)
    flat = torch.empty(n, dtype=torch.float32, device=dev)
    out, off = [], 0
    for p in params:
        out.append(flat[off:off + p.numel()].view(p.shape))
        off += p.numel()
    return out, flat


class EmbedderFunction(torch.autograd.Function):
    """emb = SpeechEmbedder.forward(x) with params (w_ih, w_hh, b_ih, b_hh)*L, w_p, b_p.

    The forward and backward share one sync block; if a persistent recurrence of either timed
    out, every returned gradient is NaN (sv_status_poison), so an optimizer step on them
    cannot pass unnoticed, and check_persistent_status() raises."""

    @staticmethod
    def forward(ctx, x, num_layers, precision, products, schedule, *params):
        L = num_layers
        layers = [tuple(params[4 * l:4 * l + 4]) for l in range(L)]
        w_p, b_p = params[4 * L], params[4 * L + 1]
        # earlier calls' completed checks: raise on a timeout there, drop the finished entries (so
        # a forward-only loop keeps _UNCHECKED bounded)
        check_persistent_status()
        ctx.status = PersistStatus(x.device)
        if precision == "bf16":
            emb, st = embedder_forward_bf16(x.contiguous(), layers, w_p, b_p, save=True, status=ctx.status,
                                            schedule=schedule)
        else:
            emb, st = embedder_forward(x.contiguous(), layers, w_p, b_p, save=True, products=products,
                                       status=ctx.status, schedule=schedule)
        # checked even if no backward follows (eval, d-vectors, anything under no_grad): a hand-off
        # timeout in this forward raises at the next call / check_persistent_status()
        ctx.status.arm()
        _UNCHECKED.append(ctx.status)
        ctx.precision, ctx.products, ctx.schedule = precision, products, schedule
        ctx.st = st
        ctx.L = L
        ctx.save_for_backward(*params)
        return emb

    @staticmethod
    def backward(ctx, demb):
        params = ctx.saved_tensors
        L = ctx.L
        layers = [tuple(params[4 * l:4 * l + 4]) for l in range(L)]
        need_dx = ctx.needs_input_grad[0]
        grads, flat = _flat_grads(params, demb.device)
        if ctx.precision == "bf16":
            out = embedder_backward_bf16(ctx.st, demb, layers, params[4 * L], grads=grads, status=ctx.status,
                                         schedule=ctx.schedule, need_dx=need_dx)
        else:
            out = embedder_backward(ctx.st, demb, layers, params[4 * L], grads=grads, need_dx=need_dx,
                                    products=ctx.products, status=ctx.status, schedule=ctx.schedule)
        call("sv_status_poison", ctx.status.ptr(), ptr(flat), flat.numel(), stream_of(flat))
        ctx.status.arm()
        if ctx.status not in _UNCHECKED:
            _UNCHECKED.append(ctx.status)
        ctx.status = None
        ctx.st = None
        if need_dx:
            grads, dx = out
        else:
            grads, dx = out, None
        return (dx, None, None, None, None, *grads)


# ----------------------------------------------------------------------------- GE2E
class Ge2eState:
    pass


def _pad_d(E):
    D = E.shape[-1]
    if D % 4 == 0:
        return E.contiguous(), D
    Dp = (D + 3) // 4 * 4
    Ep = torch.zeros(E.shape[:-1] + (Dp,), dtype=E.dtype, device=E.device)
    Ep[..., :D] = E
    return Ep, D


def ge2e_forward(E, w, b):
    """GE2E loss of E [N,M,D] with device scalars w, b.  Returns (loss 0-dim, per [N,M], state)."""
    require_device(E, w, b)
    if E.dim() != 3 or E.shape[1] < 2:
        raise ValueError("GE2E expects embeddings [N, M, D] with M >= 2 (leave-one-out centroids)")
    Ep, D0 = _pad_d(E)
    N, M, D = Ep.shape
    dev = E.device
    s = stream_of(E)
    st = Ge2eState()
    st.ws = _ws(lib().sv_ge2e_workspace_size(N, M, D, N), dev)
    st.ssum = torch.empty((N, D), dtype=torch.float32, device=dev)
    st.N, st.M, st.D, st.D0 = N, M, D, D0
    loss = torch.empty((), dtype=torch.float32, device=dev)
    per = torch.empty((N, M), dtype=torch.float32, device=dev)
    call("sv_ge2e_fwd", ptr(Ep), N, M, D, ptr(w.contiguous()), ptr(b.contiguous()), ptr(loss), ptr(per), ptr(st.ws),
         ptr(st.ssum), s)
    return loss, per, st


def ge2e_backward(st, w, b, gloss=None):
    """Returns (dE [N,M,D0], dw 0-dim, db 0-dim)."""
    N, M, D = st.N, st.M, st.D
    dev = st.ws.device
    s = stream_of(st.ws)
    Np = (N + 3) // 4 * 4
    dE = torch.empty((N, M, D), dtype=torch.float32, device=dev)
    dwdb = torch.empty((2,), dtype=torch.float32, device=dev)
    dchat = torch.empty((Np, D), dtype=torch.float32, device=dev)
    beta = torch.empty((N,), dtype=torch.float32, device=dev)
    g = None if gloss is None else gloss.contiguous()
    call("sv_ge2e_bwd", N, M, D, ptr(w.contiguous()), ptr(b.contiguous()), ptr(g), ptr(dE), ptr(dwdb), ptr(dchat),
         ptr(beta), ptr(st.ws), s)
    if st.D0 != D:
        dE = dE[..., :st.D0].contiguous()
    return dE, dwdb[0], dwdb[1]


def ge2e_train(E, w, b, dwdb_out=None):
    """Fused GE2E forward + closed-form backward for one GPU holding all N speakers (the training
    step's gloss = 1): returns (loss 0-dim, per [N,M], dE [N,M,D], dwdb [2]) from three launches
    (include/sv_ge2e.h, sv_ge2e_train); dwdb_out (2 contiguous fp32 on the device): written in
    place of a new dwdb tensor.  Shapes outside sv_ge2e_train_ok take the split path."""
    require_device(E, w, b)
    Ep, D0 = _pad_d(E)
    N, M, D = Ep.shape
    if M < 2:
        raise ValueError("GE2E expects embeddings [N, M, D] with M >= 2 (leave-one-out centroids)")
    if not lib().sv_ge2e_train_ok(N, M, D):
        loss, per, st = ge2e_forward(E, w, b)
        dE, dw, db = ge2e_backward(st, w, b)
        return loss, per, dE, torch.stack([dw, db])
    dev = E.device
    ws = _ws(lib().sv_ge2e_workspace_size(N, M, D, N), dev)
    loss = torch.empty((), dtype=torch.float32, device=dev)
    per = torch.empty((N, M), dtype=torch.float32, device=dev)
    dE = torch.empty((N, M, D), dtype=torch.float32, device=dev)
    dwdb = torch.empty((2,), dtype=torch.float32, device=dev) if dwdb_out is None else dwdb_out
    if dwdb.numel() != 2 or dwdb.dtype != torch.float32 or not dwdb.is_contiguous() or dwdb.device != dev:
        raise ValueError("ge2e_train: dwdb_out must be 2 contiguous fp32 values on the embeddings' device")
    call("sv_ge2e_train", ptr(Ep), N, M, D, ptr(w.contiguous()), ptr(b.contiguous()), ptr(loss), ptr(per), ptr(dE),
         ptr(dwdb), ptr(ws), stream_of(Ep))
    if D0 != D:
        dE = dE[..., :D0].contiguous()
    return loss, per, dE, dwdb


class GE2EFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, E, w, b):
        loss, per, st = ge2e_forward(E, w, b)
        ctx.st = st
        ctx.save_for_backward(w, b)
        ctx.mark_non_differentiable(per)
        return loss, per

    @staticmethod
    def backward(ctx, gloss, _gper):
        w, b = ctx.saved_tensors
        dE, dw, db = ge2e_backward(ctx.st, w, b, gloss.reshape(()).to(torch.float32))
        ctx.st = None
        return dE, dw.reshape(w.shape), db.reshape(b.shape)


# ----------------------------------------------------------------------------- clip + SGD
def clip_sgd_step_(flat_params, flat_grads, max_norm, lr, write_grad=False, norm_out=None, status=None):
    """In place: flat_params -= lr * min(1, max_norm/(|g|+1e-6)) * flat_grads.  With ``status``
    (a PersistStatus) the update is skipped on the device when its status word is set."""
    require_device(flat_params, flat_grads)
    ws = _ws(lib().sv_clip_sgd_workspace(), flat_params.device)
    call("sv_clip_sgd_step", ptr(flat_params), ptr(flat_grads), flat_params.numel(), float(max_norm), float(lr),
         int(write_grad), ptr(norm_out), status.ptr() if status is not None else None, ptr(ws),
         stream_of(flat_params))


def clip_sgd_step2_(p0, g0, max_norm0, p1, g1, max_norm1, lr, write_grad=False, norm_out=None, status=None,
                    report=None):
    """clip_sgd_step_ over two flat parameter groups (the network's and the loss's {w, b},
    train_speech_embedder.py:63-65) in one pair of launches; bit-identical to two calls.
    report: a tensor x for ``status.report(x)`` done inside the update launch
    (sv_clip_sgd_step2_report: the training step's status report without a launch of its own)."""
    require_device(p0, g0, p1, g1)
    ws = _ws(2 * lib().sv_clip_sgd_workspace(), p0.device)
    args = (ptr(p0), ptr(g0), p0.numel(), float(max_norm0), ptr(p1), ptr(g1), p1.numel(), float(max_norm1), float(lr),
            int(write_grad), ptr(norm_out), status.ptr() if status is not None else None, ptr(ws))
    if report is not None:
        if status is None:
            raise ValueError("clip_sgd_step2_: report needs the status block")
        require_device(report)
        slot, seq = status.next_slot()
        call("sv_clip_sgd_step2_report", *args, ptr(report), report.numel(), slot, seq, stream_of(p0))
    else:
        call("sv_clip_sgd_step2", *args, stream_of(p0))


def gemm_f32(A, B, a_kcontig=True, b_kcontig=True, bias=None, products="mfma_f32"):
    """C = op(A) op(B) through sv_gemm_f32 (test hook).  With a_kcontig A is [M,K] else [K,M];
    with b_kcontig B is [N,K] else [K,N]."""
    require_device(A, B, bias)
    M = A.shape[0] if a_kcontig else A.shape[1]
    K = A.shape[1] if a_kcontig else A.shape[0]
    N = B.shape[0] if b_kcontig else B.shape[1]
    C = torch.empty((M, N), dtype=torch.float32, device=A.device)
    ws = _ws(lib().sv_gemm_f32_workspace(M, N, K), A.device)
    call("sv_gemm_f32", int(a_kcontig), int(b_kcontig), M, N, K, ptr(A), A.shape[1], ptr(B), B.shape[1], ptr(C), N,
         ptr(bias), None, 0.0, ptr(ws), _products(products), stream_of(A))
    return C

"""Segment-level d-vectors for diarisation (reference dvector_create.py:38-73).

The reference turns each VAD-concatenated segment's log-mel spectrogram [nmels, T] into
24-frame windows at a 12-frame hop (0.24 s / 0.12 s, :48-52), embeds all windows with the
SpeechEmbedder (:100) and averages consecutive window embeddings into ~0.4 s segments
(align_embeddings, :55-73).  Audio I/O, VAD (webrtcvad) and the STFT (librosa) stay out of
scope; this module starts from the log-mel frames.  The embedding is the short-sequence,
large-batch forward of the same HIP LSTM kernels (T = 24).
"""
from __future__ import annotations

import numpy as np
import torch

from .ops import check_persistent_status, embedder_forward, embedder_forward_bf16, embedder_forward_dvec_bf16

WIN, HOP = 24, 12  # frames: int(.24/.01), int(.12/.01)
# bf16: from this many windows on, one pass of per-timestep GEMM launches with the cell in their
# epilogue (sv_dvector_embed_bf16) instead of co-resident persistent batches (bf16_batch)
DVEC_MIN = 3072
DVEC_CHUNK = 16384


def window_frames(logmel, win=WIN, hop=HOP):
    """[nmels, T] -> [S, win, nmels]: windows starting every `hop` frames while j + win < T
    (the strict '<' of dvector_create.py:50 drops a window that would end exactly at T)."""
    logmel = np.asarray(logmel)
    starts = [j for j in range(0, logmel.shape[1], hop) if j + win < logmel.shape[1]]
    if not starts:
        return np.zeros((0, win, logmel.shape[0]), dtype=np.float32)
    return np.stack([logmel[:, j:j + win].T for j in starts]).astype(np.float32)


def dvec_ok(F, H):
    """Dimensions sv_dvector_embed_bf16 takes (include/sv_ge2e.h): the x part one padded k-tile,
    whole 256-column tiles of the unit-interleaved 4H gate columns."""
    return 0 < F <= 64 and H % 64 == 0 and (4 * H) % 256 == 0


def bf16_batch(H, limit=16384):
    """Windows per call of the bf16 forward: the largest multiple of 32 (<= limit) whose whole
    recurrence grid is co-resident, so each call runs the persistent W-stationary kernels (c3's)
    instead of one launch per timestep (a 16384-window call does not fit: 0.14 of the bf16 peak)."""
    from ._lib import lib
    b = max(32, min(limit, 4096) // 32 * 32)
    while b > 32 and not lib().sv_persist_fwd_ok(b, H):
        b -= 32
    return b if lib().sv_persist_fwd_ok(b, H) else limit


@torch.no_grad()
def embed_windows(net, windows, batch=None, precision="f32", path=None, schedule="auto"):
    """Embeddings [S, proj] of windows [S, win, nmels] with the module's weights (GPU), `batch`
    windows per call (None: 16384 in fp32; bf16: bf16_batch(), the largest co-resident
    persistent batch).  precision "bf16": the c3 mixed-precision forward (bf16 GEMM operands,
    fp32 accumulation and state), no activations saved.  Raises PersistentRecurrenceError if a
    persistent recurrence of the call timed out (either precision).  path (bf16 only): "persist"
    (batches of the training forward's persistent recurrences), "dvec" (sv_dvector_embed_bf16, DVEC_CHUNK windows
    per call) or None: "dvec" from DVEC_MIN windows on when no batch is given.  schedule: the
    recurrence schedule of the stack ('auto', 'per_step', 'persist', ...; ops.embedder_forward)."""
    if precision not in ("f32", "bf16"):
        raise ValueError(f"precision must be 'f32' or 'bf16', got {precision!r}")
    if path not in (None, "persist", "dvec") or (path is not None and precision != "bf16"):
        raise ValueError(f"path must be None, 'persist' or 'dvec' (bf16 only), got {path!r}")
    dev = next(net.parameters()).device
    layers = net.LSTM_stack.layer_params()
    x = torch.as_tensor(windows, dtype=torch.float32)
    F, H = x.shape[-1], layers[0][1].shape[1]
    if path == "dvec" and not dvec_ok(F, H):
        raise ValueError(f"the per-timestep GEMM path needs F <= 64, H % 64 == 0 and 4H % 256 == 0 (F={F}, H={H})")
    if precision == "bf16" and (path == "dvec" or (path is None and batch is None and x.shape[0] >= DVEC_MIN
                                                    and dvec_ok(F, H))):
        out = [embedder_forward_dvec_bf16(x[i:i + (batch or DVEC_CHUNK)].to(dev).contiguous(), layers,
                                          net.projection.weight, net.projection.bias)
               for i in range(0, x.shape[0], batch or DVEC_CHUNK)]
        return torch.cat(out) if out else torch.zeros((0, net.projection.weight.shape[0]), device=dev)
    if batch is None:
        batch = bf16_batch(layers[0][1].shape[1]) if precision == "bf16" else 16384
    out = []
    for i in range(0, x.shape[0], batch):
        xb = x[i:i + batch].to(dev).contiguous()
        fwd = embedder_forward_bf16 if precision == "bf16" else embedder_forward
        emb, _ = fwd(xb, layers, net.projection.weight, net.projection.bias, save=False, schedule=schedule)
        out.append(emb)
    # a persistent recurrence that timed out (its grid not co-resident) must not return silently
    # wrong embeddings: wait for this call's status words and raise (both precisions: the fp32
    # forward takes its persistent recurrences too where a batch fills the device)
    check_persistent_status(wait=True)
    return torch.cat(out) if out else torch.zeros((0, net.projection.weight.shape[0]), device=dev)


class GraphedEmbedder:
    """Per-file d-vector calls (dvector_create.py:96-101: one file's windows per
    ``embedder_net(windows)`` call, tens to hundreds of windows) replayed from HIP graphs.  Such a
    call is bound by its ~20 kernel launches and their host work (~0.3 ms), not by the kernels;
    here the whole forward -- frame transpose, casts, input projections, the recurrences, the
    projection and norm -- is captured once per window-count bucket (S rounded up to `bucket`;
    padding rows are zeros, rows are independent, and only the first S are returned) and each
    call is one copy in, one graph launch, one copy out.  Same kernels and numerics as
    embed_windows(..., batch=S); the weights are read through their pointers at every replay
    (in-place updates are seen; a module whose parameters were re-allocated is re-captured).
    precision: "f32" or "bf16"; schedule as embed_windows.  Raises PersistentRecurrenceError like
    embed_windows."""

    def __init__(self, net, precision="bf16", bucket=32, max_windows=640, schedule="auto"):
        if precision not in ("f32", "bf16"):
            raise ValueError(f"precision must be 'f32' or 'bf16', got {precision!r}")
        self.net, self.precision, self.bucket, self.max_windows = net, precision, bucket, max_windows
        self.schedule = schedule
        self._graphs = {}

    def _key(self, S, T, F):
        ptrs = tuple(p.data_ptr() for p in self.net.parameters())
        return (-(-S // self.bucket) * self.bucket, T, F, ptrs)

    def _capture(self, Sp, T, F, dev):
        from ._lib import PersistStatus
        layers = self.net.LSTM_stack.layer_params()
        wp, bp = self.net.projection.weight, self.net.projection.bias
        status = PersistStatus(dev)  # caller-owned: nothing polled or allocated during the capture
        x = torch.zeros((Sp, T, F), dtype=torch.float32, device=dev)

        def fwd():
            if self.precision == "bf16":
                return embedder_forward_bf16(x, layers, wp, bp, save=False, status=status, schedule=self.schedule)[0]
            return embedder_forward(x, layers, wp, bp, save=False, status=status, schedule=self.schedule)[0]

        side = torch.cuda.Stream(dev)  # warm-up off the capture (allocator, lazy init)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            fwd()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            emb = fwd()
        return g, x, emb, status

    @torch.no_grad()
    def __call__(self, windows):
        dev = next(self.net.parameters()).device
        x = torch.as_tensor(windows, dtype=torch.float32)
        S, T, F = x.shape
        if S == 0:
            return torch.zeros((0, self.net.projection.weight.shape[0]), device=dev)
        if S > self.max_windows:  # a long file: the batched path
            return embed_windows(self.net, x, precision=self.precision, schedule=self.schedule)
        key = self._key(S, T, F)
        if key not in self._graphs:
            self._graphs = {k: v for k, v in self._graphs.items() if k[3] == key[3]}  # drop stale weights
            self._graphs[key] = self._capture(key[0], T, F, dev)
        g, xs, emb, status = self._graphs[key]
        xs[:S].copy_(x.to(dev, non_blocking=True))
        if S < xs.shape[0]:
            xs[S:].zero_()
        g.replay()
        out = emb[:S].clone()
        status.arm()
        status.poll(wait=True)
        return out


def partitions(n_windows, win_s=0.24, hop_s=0.12, seg_s=0.401):
    """[start, end) window ranges averaged into one segment (dvector_create.py:56-69): a window i
    joins segment j while it ends (i*hop + win) before j*seg; the loop's else appends the last."""
    parts, start, end, j = [], 0, 0, 1
    for i in range(n_windows):
        if i * hop_s + win_s < j * seg_s:
            end += 1
        else:
            parts.append((start, end))
            start, end, j = end, end + 1, j + 1
    parts.append((start, end))
    return parts


def align_embeddings(embeddings):
    """Average window embeddings over partitions() -> [n_segments, D] float64 (:55-73)."""
    e = np.asarray(embeddings)
    parts = partitions(len(e))
    out = np.zeros((len(parts), e.shape[1]))
    for i, (a, b) in enumerate(parts):
        out[i] = np.average(e[a:b], axis=0)
    return out

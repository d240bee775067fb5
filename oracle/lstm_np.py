"""ORACLE (test infrastructure only) -- numpy float64 restatement of the SpeechEmbedder
forward, its backward (BPTT) and the training-step update.

Follows the reference:
  SpeechEmbedder.forward   speech_embedder_net.py:27-33
      nn.LSTM(nmels, hidden, num_layers, batch_first=True) with h0 = c0 = 0,
      PyTorch gate order [i, f, g, o] as row blocks of W_ih / W_hh (:19),
      last frame x[:, T-1] (:30), Linear(hidden, proj) (:25,31), x / |x|_2 (:32, no eps)
  train step               train_speech_embedder.py:54-65
      clip_grad_norm_(net, 3.0), clip_grad_norm_([w, b], 1.0), SGD(lr) without momentum
      (torch clip: coef = max_norm / (total_norm + 1e-6), applied only when coef < 1)

``params`` is a dict keyed by the reference state_dict names (tests/golden/recipe.py).
Pure numpy loops over time: use only at small sizes.
"""
from __future__ import annotations

import numpy as np

from . import ge2e_np


def _sig(x):
    return 1.0 / (1.0 + np.exp(-x))


def lstm_layer_forward(x, Wih, Whh, bih, bhh):
    """x [B,T,F] -> (h [B,T,H], cache).  One nn.LSTM layer."""
    B, T, _ = x.shape
    H = Whh.shape[1]
    h = np.zeros((B, H))
    c = np.zeros((B, H))
    hs = np.zeros((B, T, H))
    cs = np.zeros((B, T, H))
    acts = np.zeros((B, T, 4 * H))
    for t in range(T):
        g = x[:, t] @ Wih.T + bih + h @ Whh.T + bhh
        i, f, gg, o = _sig(g[:, :H]), _sig(g[:, H:2 * H]), np.tanh(g[:, 2 * H:3 * H]), _sig(g[:, 3 * H:])
        c = f * c + i * gg
        h = o * np.tanh(c)
        hs[:, t] = h
        cs[:, t] = c
        acts[:, t] = np.concatenate([i, f, gg, o], axis=1)
    return hs, (x, hs, cs, acts)


def lstm_layer_backward(dhs, Wih, Whh, cache):
    """dhs [B,T,H] gradient w.r.t. the layer's outputs -> (dx, dWih, dWhh, db)."""
    x, hs, cs, acts = cache
    B, T, H = hs.shape
    dWih = np.zeros_like(Wih)
    dWhh = np.zeros_like(Whh)
    db = np.zeros(4 * H)
    dx = np.zeros_like(x)
    dh_next = np.zeros((B, H))
    dc_next = np.zeros((B, H))
    for t in range(T - 1, -1, -1):
        i, f, g, o = (acts[:, t, k * H:(k + 1) * H] for k in range(4))
        c = cs[:, t]
        c_prev = cs[:, t - 1] if t > 0 else np.zeros((B, H))
        h_prev = hs[:, t - 1] if t > 0 else np.zeros((B, H))
        dh = dhs[:, t] + dh_next
        tc = np.tanh(c)
        dc = dc_next + dh * o * (1 - tc * tc)
        di = dc * g * i * (1 - i)
        df = dc * c_prev * f * (1 - f)
        dg = dc * i * (1 - g * g)
        do = dh * tc * o * (1 - o)
        dG = np.concatenate([di, df, dg, do], axis=1)
        dWih += dG.T @ x[:, t]
        dWhh += dG.T @ h_prev
        db += dG.sum(axis=0)
        dx[:, t] = dG @ Wih
        dh_next = dG @ Whh
        dc_next = dc * f
    return dx, dWih, dWhh, db


def embedder_forward(params, x, num_layer):
    """speech_embedder_net.py:27-33.  x [B,T,F] -> (emb [B,P], cache)."""
    inp = np.asarray(x, np.float64)
    caches = []
    for l in range(num_layer):
        p = lambda n: np.asarray(params[f"LSTM_stack.{n}_l{l}"], np.float64)  # noqa: E731
        inp, cache = lstm_layer_forward(inp, p("weight_ih"), p("weight_hh"), p("bias_ih"), p("bias_hh"))
        caches.append(cache)
    last = inp[:, -1]
    Wp = np.asarray(params["projection.weight"], np.float64)
    bp = np.asarray(params["projection.bias"], np.float64)
    y = last @ Wp.T + bp
    n = np.linalg.norm(y, axis=1, keepdims=True)
    emb = y / n
    return emb, (caches, last, y, n)


def embedder_backward(params, demb, cache, num_layer):
    """Gradients of every parameter (dict keyed like params) given d emb."""
    caches, last, y, n = cache
    emb = y / n
    Wp = np.asarray(params["projection.weight"], np.float64)
    dy = (demb - emb * (demb * emb).sum(axis=1, keepdims=True)) / n
    grads = {"projection.weight": dy.T @ last, "projection.bias": dy.sum(axis=0)}
    B, T, H = caches[-1][1].shape
    dhs = np.zeros((B, T, H))
    dhs[:, -1] = dy @ Wp
    for l in range(num_layer - 1, -1, -1):
        Wih = np.asarray(params[f"LSTM_stack.weight_ih_l{l}"], np.float64)
        Whh = np.asarray(params[f"LSTM_stack.weight_hh_l{l}"], np.float64)
        dx, dWih, dWhh, db = lstm_layer_backward(dhs, Wih, Whh, caches[l])
        grads[f"LSTM_stack.weight_ih_l{l}"] = dWih
        grads[f"LSTM_stack.weight_hh_l{l}"] = dWhh
        grads[f"LSTM_stack.bias_ih_l{l}"] = db
        grads[f"LSTM_stack.bias_hh_l{l}"] = db.copy()
        dhs = dx
    return grads


def clip_coef(grads, max_norm):
    """torch.nn.utils.clip_grad_norm_ (norm_type 2): coef applied iff < 1."""
    total = np.sqrt(sum(float((np.asarray(g, np.float64) ** 2).sum()) for g in grads))
    return min(1.0, max_norm / (total + 1e-6)), total


def train_step(params, w, b, x, N, M, num_layer, lr=0.01):
    """One reference training step (train_speech_embedder.py:54-65) -> (loss, new_params, new_w, new_b,
    emb, grads, dw, db)."""
    emb, cache = embedder_forward(params, x, num_layer)
    E = emb.reshape(N, M, -1)
    loss, _, _ = ge2e_np.ge2e_forward(E, w, b)
    dE, dw, db = ge2e_np.ge2e_backward(E, w, b)
    grads = embedder_backward(params, dE.reshape(N * M, -1), cache, num_layer)
    names = list(params.keys())
    coef, _ = clip_coef([grads[k] for k in names], 3.0)
    coef_wb, _ = clip_coef([np.array(dw), np.array(db)], 1.0)
    new = {k: np.asarray(params[k], np.float64) - lr * coef * grads[k] for k in names}
    return (loss, new, w - lr * coef_wb * dw, b - lr * coef_wb * db, emb, grads, dw, db)

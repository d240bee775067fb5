"""ORACLE (test infrastructure only) -- the SpeechEmbedder training step in fp32 with the
mixed-precision rounding of BASELINE config c3 (bf16 GEMM operands, fp32 accumulation; bf16
storage of the x-projection and of the saved activations; fp32 cell state / gradients / loss),
restated on plain torch-CPU float32 ops.

Follows the same reference lines as lstm_np.py (speech_embedder_net.py:19,27-33 for nn.LSTM +
last frame + Linear + L2 norm; utils.py:27-132 + speech_embedder_net.py:43-49 for GE2E;
train_speech_embedder.py:54-65 for the step).  The only difference from the reference's fp32
arithmetic is the operand quantiser ``q`` applied where the c3 path feeds a GEMM:

  forward   gates_t = q(q(x_t) q(W_ih)^T + b_ih + b_hh) + q(h_{t-1}) q(W_hh)^T   (every layer;
            layer l > 0 reads q(h) of layer l-1; the x-projection incl. biases is stored in
            bf16, ABI v3); c, h and the activations that form them fp32; the projection and
            the norm fp32 (they read the fp32 h of the last layer)
  backward  the saved activations q(i), q(f), q(g), q(o) (bf16 storage) with fp32 c;
            dh_rec = q(dG_{t+1}) q(W_hh); dW_ih += q(dG_t)^T q(x_t); dW_hh += q(dG_t)^T q(h_{t-1});
            db += q(dG_t) (fp32 sum of the rounded values); dx_t = q(dG_t) q(W_ih) (fp32, added to
            the layer below's dh in fp32)

q = round-to-nearest-even to bf16 (``bf16=True``) or the identity (``bf16=False``, which is the
reference's own fp32 arithmetic and is pinned against the reference-generated golden vectors in
tests/test_oracle_bf16.py).  Products of two bf16 values are exact in fp32, so the oracle and
the HIP path differ only by fp32 accumulation order (~1e-7 relative per sum).

Use at sizes up to the c4 per-rank shape (B = 80, T = 160, H = 768) on the CPU: seconds on a few
cores.  The ops are device-agnostic: ``device="cuda"`` runs the same restatement on the GPU's
stock torch ops (tests/test_gpu_precision.py checks c3 at its full T = 160 that way); it stays the
checker, never the product path.
"""
from __future__ import annotations

import torch

from . import torch_port


def q_bf16(t):
    """Round-to-nearest-even to bf16, back in fp32."""
    return t.to(torch.bfloat16).to(torch.float32)


def _ident(t):
    return t


def _params(params, L, device="cpu"):
    f = lambda k: torch.as_tensor(params[k], dtype=torch.float32, device=device)  # noqa: E731
    layers = [(f(f"LSTM_stack.weight_ih_l{l}"), f(f"LSTM_stack.weight_hh_l{l}"), f(f"LSTM_stack.bias_ih_l{l}"),
               f(f"LSTM_stack.bias_hh_l{l}")) for l in range(L)]
    return layers, f("projection.weight"), f("projection.bias")


def embedder_forward(params, x, L, bf16=True, device="cpu"):
    """x [B,T,F] -> (emb [B,P], cache)."""
    q = q_bf16 if bf16 else _ident
    layers, Wp, bp = _params(params, L, device)
    inp = torch.as_tensor(x, dtype=torch.float32, device=device)
    B, T, _ = inp.shape
    z = dict(device=device)
    caches = []
    for (Wih, Whh, bih, bhh) in layers:
        H = Whh.shape[1]
        qWih, qWhh = q(Wih), q(Whh)
        xq = q(inp)
        gx = q((xq.reshape(B * T, -1) @ qWih.T).reshape(B, T, 4 * H) + (bih + bhh))
        h = torch.zeros(B, H, **z)
        c = torch.zeros(B, H, **z)
        hs = torch.empty(B, T, H, **z)
        cs = torch.empty(B, T, H, **z)
        acts = torch.empty(B, T, 4 * H, **z)
        for t in range(T):
            g = gx[:, t] + q(h) @ qWhh.T
            i, f, gg, o = (torch.sigmoid(g[:, :H]), torch.sigmoid(g[:, H:2 * H]), torch.tanh(g[:, 2 * H:3 * H]),
                           torch.sigmoid(g[:, 3 * H:]))
            c = f * c + i * gg
            h = o * torch.tanh(c)
            hs[:, t], cs[:, t] = h, c
            acts[:, t] = q(torch.cat([i, f, gg, o], dim=1))
        caches.append((xq, hs, cs, acts))
        inp = hs
    last = inp[:, -1]
    y = last @ Wp.T + bp
    n = y.norm(dim=1, keepdim=True)
    return y / n, (caches, last, y, n)


def embedder_backward(params, demb, cache, L, bf16=True, device="cpu"):
    """Gradients (dict keyed like params, fp32 tensors) given d emb [B,P]."""
    q = q_bf16 if bf16 else _ident
    layers, Wp, _ = _params(params, L, device)
    caches, last, y, n = cache
    demb = torch.as_tensor(demb, dtype=torch.float32, device=device)
    z = dict(device=device)
    emb = y / n
    dy = (demb - emb * (demb * emb).sum(dim=1, keepdim=True)) / n
    grads = {"projection.weight": dy.T @ last, "projection.bias": dy.sum(dim=0)}
    B, T, H = caches[-1][1].shape
    dhs = torch.zeros(B, T, H, **z)
    dhs[:, -1] = dy @ Wp
    for l in range(L - 1, -1, -1):
        Wih, Whh, _, _ = layers[l]
        qWih, qWhh = q(Wih), q(Whh)
        xq, hs, cs, acts = caches[l]
        dGq = torch.empty(B, T, 4 * H, **z)
        dh_next = torch.zeros(B, H, **z)
        dc_next = torch.zeros(B, H, **z)
        for t in range(T - 1, -1, -1):
            i, f, g, o = (acts[:, t, k * H:(k + 1) * H] for k in range(4))
            c = cs[:, t]
            c_prev = cs[:, t - 1] if t > 0 else torch.zeros(B, H, **z)
            dh = dhs[:, t] + dh_next
            tc = torch.tanh(c)
            dc = dc_next + dh * o * (1 - tc * tc)
            dG = torch.cat([dc * g * i * (1 - i), dc * c_prev * f * (1 - f), dc * i * (1 - g * g),
                            dh * tc * o * (1 - o)], dim=1)
            dGq[:, t] = q(dG)
            dh_next = dGq[:, t] @ qWhh
            dc_next = dc * f
        hprev = torch.cat([torch.zeros(B, 1, H, **z), q(hs[:, :-1])], dim=1)
        dG2 = dGq.reshape(B * T, 4 * H)
        grads[f"LSTM_stack.weight_ih_l{l}"] = dG2.T @ xq.reshape(B * T, -1)
        grads[f"LSTM_stack.weight_hh_l{l}"] = dG2.T @ hprev.reshape(B * T, H)
        db = dG2.sum(dim=0)
        grads[f"LSTM_stack.bias_ih_l{l}"] = db
        grads[f"LSTM_stack.bias_hh_l{l}"] = db.clone()
        dhs = (dG2 @ qWih).reshape(B, T, -1)
    grads["input"] = dhs  # d loss / d x [B, T, F]: layer 0's dx_t = q(dG_t) q(W_ih)
    return grads


def train_step(params, w, b, x, N, M, L, bf16=True, lr=0.01, device="cpu"):
    """One train_speech_embedder.py:54-65 step -> (loss, new_params, new_w, new_b, emb, grads, dw, db),
    all fp32 (GE2E by autograd on torch_port.ge2e_loss in fp32, clip_grad_norm_ semantics of
    lstm_np.clip_coef); the tensors live on ``device``."""
    emb, cache = embedder_forward(params, x, L, bf16, device)
    E = emb.detach().reshape(N, M, -1).requires_grad_(True)
    wt = torch.tensor(float(w), requires_grad=True, device=device)
    bt = torch.tensor(float(b), requires_grad=True, device=device)
    loss = torch_port.ge2e_loss(E, wt, bt)
    loss.backward()
    grads = embedder_backward(params, E.grad.reshape(N * M, -1), cache, L, bf16, device)
    names = list(params.keys())
    tot = torch.sqrt(sum((grads[k].double() ** 2).sum() for k in names))
    coef = min(1.0, 3.0 / (float(tot) + 1e-6))
    dw, db = float(wt.grad), float(bt.grad)
    tot_wb = (dw * dw + db * db) ** 0.5
    coef_wb = min(1.0, 1.0 / (tot_wb + 1e-6))
    new = {k: torch.as_tensor(params[k], dtype=torch.float32, device=device) - lr * coef * grads[k] for k in names}
    return (float(loss.detach()), new, w - lr * coef_wb * dw, b - lr * coef_wb * db, emb, grads, dw, db)

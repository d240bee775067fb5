"""CPU: the mixed-precision (bf16-operand) oracle, oracle/lstm_bf16.py.

With its quantiser off it is the reference's fp32 arithmetic and must reproduce the golden
training step that tests/golden/make_golden.py recorded by running the reference itself (same
vectors as the fp64 oracle's test_lstm_oracle_small_net_step).  Its quantiser must be
round-to-nearest-even to bf16, the rounding the HIP path's casts perform."""
import numpy as np
import torch

from conftest import golden
from oracle import lstm_bf16
import recipe


def _small_setup():
    s = golden("net_small.npz")
    dims = tuple(int(v) for v in s["dims"])
    P = recipe.make_weights(int(s["wseed"]), *dims, scale=float(s["wscale"]))
    N, M, T = int(s["N"]), int(s["M"]), int(s["T"])
    x = recipe.make_frames(int(s["xseed"]), N * M, T, dims[0])
    return s, dims, P, x, N, M


def test_q_bf16_is_round_to_nearest_even():
    one = 1.0
    v = torch.tensor([one + 2 ** -8, one + 3 * 2 ** -9, one + 2 ** -7 + 2 ** -8, -(one + 2 ** -9), 3.0e38])
    got = lstm_bf16.q_bf16(v).tolist()
    assert got[0] == 1.0                      # tie -> even (1.0)
    assert got[1] == one + 2 ** -7            # above half -> up
    assert got[2] == one + 2 ** -6            # tie -> even (up)
    assert got[3] == -1.0
    assert np.isfinite(got[4]) or got[4] == float("inf")


def test_fp32_mode_reproduces_reference_step():
    s, dims, P, x, N, M = _small_setup()
    loss, new, w1, b1, emb, grads, dw, db = lstm_bf16.train_step(P, 10.0, -5.0, x, N, M, dims[2], bf16=False)
    assert abs(loss - s["losses"][0]) <= 1e-5 * abs(s["losses"][0])
    np.testing.assert_allclose(emb.reshape(N, M, -1).numpy(), s["emb0"], atol=2e-6)
    for k in P:
        ref = s["grad." + k]
        np.testing.assert_allclose(grads[k].numpy(), ref, atol=2e-5 * np.abs(ref).max())
        np.testing.assert_allclose(new[k].numpy(), s["p1." + k], atol=2e-6)
    np.testing.assert_allclose([w1, b1], s["wb1"], atol=2e-6)


def test_bf16_mode_differs_at_bf16_level():
    s, dims, P, x, N, M = _small_setup()
    l32, _, _, _, e32, g32, _, _ = lstm_bf16.train_step(P, 10.0, -5.0, x, N, M, dims[2], bf16=False)
    l16, _, _, _, e16, g16, _, _ = lstm_bf16.train_step(P, 10.0, -5.0, x, N, M, dims[2], bf16=True)
    d = float((e16 - e32).abs().max())
    assert 1e-5 < d < 5e-2, d   # operand rounding (2^-9 relative) is visible but bounded
    assert abs(l16 - l32) < 1e-2 * abs(l32)

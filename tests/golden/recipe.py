"""Portable, seeded input/weight recipes shared by the golden-fixture generator,
the parity tests and the benchmark.

Everything here is plain numpy (PCG64 ``default_rng``), so the same seed gives the
same bits on any machine with numpy >= 1.17; no torch RNG is involved.  Weights are
therefore never committed: a fixture records the recipe (seed, scale, dims) and the
test regenerates the weights.

The parameter names and shapes are those of the reference ``SpeechEmbedder``
(``speech_embedder_net.py:19-25``): ``LSTM_stack.{weight_ih_l*, weight_hh_l*,
bias_ih_l*, bias_hh_l*}`` then ``projection.{weight,bias}``.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np


def param_shapes(nmels: int, hidden: int, num_layer: int, proj: int):
    """state_dict order of the reference SpeechEmbedder (nn.LSTM order, then Linear)."""
    shapes = OrderedDict()
    for l in range(num_layer):
        inp = nmels if l == 0 else hidden
        shapes[f"LSTM_stack.weight_ih_l{l}"] = (4 * hidden, inp)
        shapes[f"LSTM_stack.weight_hh_l{l}"] = (4 * hidden, hidden)
        shapes[f"LSTM_stack.bias_ih_l{l}"] = (4 * hidden,)
        shapes[f"LSTM_stack.bias_hh_l{l}"] = (4 * hidden,)
    shapes["projection.weight"] = (proj, hidden)
    shapes["projection.bias"] = (proj,)
    return shapes


def make_weights(seed: int, nmels: int, hidden: int, num_layer: int, proj: int,
                 scale: float = 1.0, bias_std: float = 0.05):
    """Xavier-normal-like weights (std = sqrt(2/(fan_in+fan_out)), as the reference init at
    ``speech_embedder_net.py:20-24``) times ``scale``; small random biases so every bias
    path is exercised.  Returns an OrderedDict name -> float32 ndarray."""
    rng = np.random.default_rng(seed)
    out = OrderedDict()
    for name, shape in param_shapes(nmels, hidden, num_layer, proj).items():
        if len(shape) == 2:
            std = math.sqrt(2.0 / (shape[0] + shape[1])) * scale
            out[name] = (rng.standard_normal(shape) * std).astype(np.float32)
        else:
            out[name] = (rng.standard_normal(shape) * bias_std).astype(np.float32)
    return out


def make_frames(seed: int, batch: int, frames: int, nmels: int):
    """Synthetic utterance frames x ~ N(0,1), [batch, frames, nmels] float32."""
    rng = np.random.default_rng(seed)
    return rng.standard_normal((batch, frames, nmels)).astype(np.float32)


def make_embeddings(seed: int, n: int, m: int, d: int, clustered: bool = True):
    """Unit-norm embeddings [n, m, d] float32.  ``clustered`` draws a speaker direction
    plus per-utterance noise so same-speaker cosines are high and the softmax is
    not flat (a realistic, non-degenerate GE2E input)."""
    rng = np.random.default_rng(seed)
    if clustered:
        spk = rng.standard_normal((n, 1, d))
        e = spk + 0.7 * rng.standard_normal((n, m, d))
    else:
        e = rng.standard_normal((n, m, d))
    e = e / np.linalg.norm(e, axis=2, keepdims=True)
    return e.astype(np.float32)


def make_speaker_dir(root, n_spk, seed):
    """Synthetic preprocessed TIMIT-style data: speakerK.npy = [utterances, 40 mels, 180 frames]
    (the data_preprocess.py:46-54 on-disk format)."""
    import os
    rng = np.random.default_rng(seed)
    os.makedirs(root, exist_ok=True)
    for k in range(n_spk):
        n_utt = int(rng.integers(8, 14))
        base = rng.standard_normal((1, 40, 1)) * 2.0
        u = (base + rng.standard_normal((n_utt, 40, 180))).astype(np.float32)
        np.save(os.path.join(root, f"speaker{k}.npy"), u)

"""ORACLE (test infrastructure only) -- the EER threshold sweep of the reference's test()
(train_speech_embedder.py:134-149), restated in numpy with the reference's float32 arithmetic.

For thresholds thr_i = 0.01 i + 0.5 (i < 50), on sim [N, M2, N] (verification utterances
against enrollment centroids, get_cossim at :129):
  FAR = (sum_j #{sim[j] > thr} - #{sim[j,:,j] > thr}) / (N-1) / M2 / N
  FRR = sum_j (M2 - #{sim[j,:,j] > thr}) / M2 / N
evaluated as float32 tensor ops in the reference (so here in np.float32, same operation order);
the reported (EER, thr, FAR, FRR) is the first threshold with the smallest |FAR-FRR| (strict
improvement from diff = 1), EER = (FAR + FRR) / 2.
"""
from __future__ import annotations

import numpy as np

f32 = np.float32


def thresholds():
    return [0.01 * i + 0.5 for i in range(50)]


def counts(sim, thr):
    sim = np.asarray(sim, np.float32)
    N = sim.shape[0]
    above = sim > np.float32(thr)
    return int(above.sum()), int(sum(above[j, :, j].sum() for j in range(N)))


def far_frr_from_counts(n_all, n_diag, N, M2):
    far = f32(f32(f32(f32(n_all - n_diag) / f32(N - 1.0)) / f32(M2)) / f32(N))
    frr = f32(f32(f32(M2 * N - n_diag) / f32(M2)) / f32(N))
    return far, frr


def eer(sim):
    N, M2 = sim.shape[0], sim.shape[1]
    diff, best = f32(1.0), (f32(0), 0.0, f32(0), f32(0))
    for thr in thresholds():
        far, frr = far_frr_from_counts(*counts(sim, thr), N, M2)
        d = f32(abs(f32(far - frr)))
        if diff > d:
            diff = d
            best = (f32(f32(far + frr) / f32(2.0)), thr, far, frr)
    return best

import contextlib
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, GOLDEN)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def golden(name):
    return np.load(os.path.join(GOLDEN, name))


@contextlib.contextmanager
def model_dims(nmels, hidden, num_layer, proj):
    """Temporarily override hp dims (SpeechEmbedder reads them at construction)."""
    from pytorch_speaker_verification_amd.hparam import hparam as hp
    old = (hp.data.nmels, hp.model.hidden, hp.model.num_layer, hp.model.proj)
    hp.data.nmels, hp.model.hidden, hp.model.num_layer, hp.model.proj = nmels, hidden, num_layer, proj
    try:
        yield
    finally:
        hp.data.nmels, hp.model.hidden, hp.model.num_layer, hp.model.proj = old

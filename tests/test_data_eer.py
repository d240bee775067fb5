"""Host-side parity of the §8f rows: the preprocessed-.npy dataset (data_load.py:48-85), the
EER threshold sweep (train_speech_embedder.py:134-149, oracle) and checkpoint compatibility."""
import os
import random

import numpy as np
import pytest
import torch

import recipe
from conftest import GOLDEN, golden, model_dims
from oracle import eer_np


@pytest.fixture
def speaker_dir(tmp_path, monkeypatch):
    g = golden("loader.npz")
    d = tmp_path / "spk"
    recipe.make_speaker_dir(str(d), int(g["n_spk"]), int(g["data_seed"]))
    order = [str(x) for x in g["listdir"]]  # the reference run's os.listdir order
    real = os.listdir
    monkeypatch.setattr(os, "listdir", lambda p=".": order if os.path.abspath(p) == str(d) else real(p))
    return str(d), g


def test_preprocessed_dataset_matches_reference(speaker_dir):
    from pytorch_speaker_verification_amd import data_load
    from pytorch_speaker_verification_amd.hparam import hparam as hp
    path, g = speaker_dir
    old = (hp.training, hp.data.test_path, hp.test.M)
    hp.training, hp.data.test_path, hp.test.M = False, path, int(g["M"])
    try:
        random.seed(int(g["seed"]))
        np.random.seed(int(g["seed"]))
        ds = data_load.SpeakerDatasetTIMITPreprocessed()
        assert len(ds) == int(g["n_spk"])
        items = np.stack([ds[i].numpy() for i in range(3)])
        np.testing.assert_array_equal(items, g["items"])           # bit-exact, same RNG draws
        ds2 = data_load.SpeakerDatasetTIMITPreprocessed(shuffle=False, utter_start=1)
        np.testing.assert_array_equal(np.stack([ds2[i].numpy() for i in range(2)]), g["items_noshuffle"])
        assert items.shape == (3, int(g["M"]), 160, 40) and items.dtype == np.float32
    finally:
        hp.training, hp.data.test_path, hp.test.M = old


def test_eer_oracle_matches_reference_prints():
    e = golden("eer.npz")
    acc = np.float32(0)
    per_epoch = len(e["sims"]) // int(e["epochs"])
    for b, sim in enumerate(e["sims"]):
        eer, thr, far, frr = eer_np.eer(sim)
        np.testing.assert_array_equal(np.round([eer, thr, far, frr], 2), e["printed"][b])
    for ep in range(int(e["epochs"])):
        s = np.float32(0)
        for b in range(per_epoch):
            s = np.float32(s + eer_np.eer(e["sims"][ep * per_epoch + b])[0])
        acc = np.float32(acc + np.float32(s / per_epoch))
    assert abs(float(acc / np.float32(int(e["epochs"]))) - float(e["avg_eer"])) < 5e-5


def test_reference_checkpoint_loads():
    """A reference-written state_dict (torch.save of SpeechEmbedder, train_speech_embedder.py:81)
    loads into the drop-in module with weights_only=True, keys and values intact."""
    from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder
    sd = torch.load(os.path.join(GOLDEN, "ref_small_checkpoint.pth"), weights_only=True)
    with model_dims(40, 64, 3, 32):
        net = SpeechEmbedder()
    net.load_state_dict(sd)
    w = recipe.make_weights(41, 40, 64, 3, 32, scale=3.0)
    for k, v in net.state_dict().items():
        np.testing.assert_array_equal(v.numpy(), w[k])


def test_raw_wav_dataset_is_out_of_scope():
    from pytorch_speaker_verification_amd import data_load
    with pytest.raises(NotImplementedError):
        data_load.SpeakerDatasetTIMIT()

"""Drop-in data loading (reference data_load.py:19-85).

``SpeakerDatasetTIMITPreprocessed`` serves [M, 160, nmels] float32 utterance stacks from the
offline-preprocessed ``speakerK.npy`` files ([utterances, nmels, 180], data_preprocess.py:46-54)
with the reference's sampling semantics and RNG consumption (so a seeded run draws the same
batches): with shuffle, a speaker chosen by ``random.sample`` independently of ``idx``
(data_load.py:70-71) and M utterances drawn WITH replacement by ``np.random.randint`` (:77);
without shuffle, file ``idx`` of ``os.listdir`` order and utterances [utter_start, +M) (:73,79).
Frames are truncated to 160 (:82) and transposed to [M, frames, mels] (:84).

``DevicePrefetcher`` overlaps the pinned host->device copy of batch k+1 with step k on a side
HIP stream.  ``SpeakerDatasetTIMIT`` (raw-wav, librosa features) is out of scope here.
"""
from __future__ import annotations

import os
import random

import numpy as np
import torch
from torch.utils.data import Dataset

from .hparam import hparam as hp

TRAIN_FRAMES = 160  # data_load.py:82 ("TODO implement variable length batch size")


class SpeakerDatasetTIMITPreprocessed(Dataset):
    def __init__(self, shuffle=True, utter_start=0):
        split = hp.train if hp.training else hp.test
        self.path = hp.data.train_path if hp.training else hp.data.test_path
        self.utter_num = split.M
        self.file_list = os.listdir(self.path)
        self.shuffle = shuffle
        self.utter_start = utter_start

    def __len__(self):
        return len(self.file_list)

    def _speaker_file(self, idx):
        names = os.listdir(self.path)  # re-listed per item, as the reference does (:68)
        return random.sample(names, 1)[0] if self.shuffle else names[idx]

    def _utterances(self, utters):
        if self.shuffle:
            return utters[np.random.randint(0, utters.shape[0], self.utter_num)]
        return utters[self.utter_start:self.utter_start + self.utter_num]

    def __getitem__(self, idx):
        utters = np.load(os.path.join(self.path, self._speaker_file(idx)))
        picked = self._utterances(utters)[:, :, :TRAIN_FRAMES]
        return torch.tensor(np.ascontiguousarray(picked.transpose(0, 2, 1)))


class SpeakerDatasetTIMIT(Dataset):
    """Raw-wav dataset (data_load.py:19-46): needs librosa STFT/mel features (utils.py:138-164),
    which are offline DSP outside the GPU training path."""

    def __init__(self):
        raise NotImplementedError("raw-wav featurisation (librosa) is out of scope: run the reference's "
                                  "data_preprocess.py once and set data.data_preprocessed: true")


class DevicePrefetcher:
    """Iterates a DataLoader yielding device tensors; the copy of the next batch (pinned host
    memory, non_blocking) runs on a side stream while the caller works on the current one."""

    def __init__(self, loader, device, on_fetch=None):
        self.loader, self.device = loader, torch.device(device)
        self.stream = torch.cuda.Stream(device=self.device)
        self.on_fetch = on_fetch  # called right after each host batch is drawn (RNG-order hook)

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        it = iter(self.loader)
        nxt = self._fetch(it)
        while nxt is not None:
            cur, ev = nxt
            torch.cuda.current_stream(self.device).wait_event(ev)
            cur.record_stream(torch.cuda.current_stream(self.device))
            nxt = self._fetch(it)
            yield cur

    def _fetch(self, it):
        try:
            host = next(it)
        except StopIteration:
            return None
        if self.on_fetch is not None:
            self.on_fetch()
        if not host.is_pinned():
            host = host.pin_memory()
        with torch.cuda.stream(self.stream):
            dev = host.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return dev, ev

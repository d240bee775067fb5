"""Drop-in training / EER-evaluation driver (reference train_speech_embedder.py:19-160).

``train(model_path)``
    The reference loop (:19-90): preprocessed dataset -> DataLoader(N speakers, drop_last) ->
    per batch one GE2E step -> periodic log line and checkpoints.  The step body (:44-65) runs
    as ``GE2ETrainer.step`` (HIP kernels, no autograd graph, no host sync); the log line keeps
    the reference's format; checkpoints keep its file names and state_dict keys.  Batches are
    copied host->device on a side stream ahead of use (DevicePrefetcher).  The reference's
    per-batch row permutation (:48-57) is value-neutral (rows are independent; tested bitwise),
    so only its ``random.sample`` draw is kept, which keeps seeded runs on the reference's
    data order.
``test(model_path)``
    EER evaluation (:92-154) on the GPU: enrollment / verification halves, verification
    centroids from get_centroids, get_cossim(verification, enrollment centroids), the 50-point
    threshold sweep on device (exact integer counts, sv_eer_counts) and the reference's float32
    FAR/FRR/EER selection.  Returns the average EER (the reference only prints it).
"""
from __future__ import annotations

import os
import random
import time

import numpy as np
import torch
from torch.utils.data import DataLoader

from ._lib import call, ptr, stream_of
from .data_load import DevicePrefetcher, SpeakerDatasetTIMIT, SpeakerDatasetTIMITPreprocessed
from .hparam import hparam as hp
from .speech_embedder_net import GE2ELoss, SpeechEmbedder
from .trainer import GE2ETrainer
from .utils import get_centroids, get_cossim

EER_THRESHOLDS = [0.01 * i + 0.5 for i in range(50)]  # :134


def _dataset():
    return SpeakerDatasetTIMITPreprocessed() if hp.data.data_preprocessed else SpeakerDatasetTIMIT()


def _value_neutral_perm(n):
    """The reference's random.sample permutation (:48-52 / :114-119): drawn for RNG parity."""
    return random.sample(range(0, n), n)


def train(model_path):
    device = torch.device(hp.device)
    train_dataset = _dataset()
    loader = DataLoader(train_dataset, batch_size=hp.train.N, shuffle=True, num_workers=hp.train.num_workers,
                        drop_last=True, pin_memory=True)
    embedder_net = SpeechEmbedder().to(device)
    if hp.train.restore:
        embedder_net.load_state_dict(torch.load(model_path, weights_only=True))
    ge2e_loss = GE2ELoss(device)
    trainer = GE2ETrainer(embedder_net, ge2e_loss, lr=hp.train.lr)
    os.makedirs(hp.train.checkpoint_dir, exist_ok=True)
    N, M = hp.train.N, hp.train.M
    embedder_net.train()
    iteration = 0
    e = batch_id = 0
    for e in range(hp.train.epochs):
        total_loss = torch.zeros((), device=device)
        batches = DevicePrefetcher(loader, device, on_fetch=lambda: _value_neutral_perm(N * M))
        for batch_id, mel_db_batch in enumerate(batches):
            x = mel_db_batch.reshape(N * M, mel_db_batch.size(2), mel_db_batch.size(3))
            loss = trainer.step(x, N, M)
            total_loss = total_loss + loss
            iteration += 1
            if (batch_id + 1) % hp.train.log_interval == 0:
                mesg = "{0}\tEpoch:{1}[{2}/{3}],Iteration:{4}\tLoss:{5:.4f}\tTLoss:{6:.4f}\t\n".format(
                    time.ctime(), e + 1, batch_id + 1, len(train_dataset) // N, iteration, float(loss),
                    float(total_loss) / (batch_id + 1))
                print(mesg)
                if hp.train.log_file is not None:
                    with open(hp.train.log_file, "a") as f:
                        f.write(mesg)
        if hp.train.checkpoint_dir is not None and (e + 1) % hp.train.checkpoint_interval == 0:
            ckpt = os.path.join(hp.train.checkpoint_dir, f"ckpt_epoch_{e + 1}_batch_id_{batch_id + 1}.pth")
            torch.save({k: v.detach().cpu() for k, v in embedder_net.state_dict().items()}, ckpt)
    save_path = os.path.join(hp.train.checkpoint_dir, f"final_epoch_{e + 1}_batch_id_{batch_id + 1}.model")
    torch.save({k: v.detach().cpu() for k, v in embedder_net.state_dict().items()}, save_path)
    print("\nDone, trained model saved at", save_path)
    return save_path


def eer_from_sim(sim):
    """(EER, threshold, FAR, FRR) of one batch: counts on device, the reference's float32
    selection on the host (train_speech_embedder.py:134-149)."""
    N, M2, Nc = sim.shape
    thr = torch.tensor(EER_THRESHOLDS, dtype=torch.float32, device=sim.device)
    cnt = torch.empty((2, len(EER_THRESHOLDS)), dtype=torch.float32, device=sim.device)
    call("sv_eer_counts", ptr(sim), N, M2, Nc, ptr(thr), len(EER_THRESHOLDS), ptr(cnt[0]), ptr(cnt[1]),
         stream_of(sim))
    n_all, n_diag = cnt.cpu().numpy()
    f32 = np.float32
    diff, best = f32(1.0), (f32(0), 0.0, f32(0), f32(0))
    for i, t in enumerate(EER_THRESHOLDS):
        far = f32(f32(f32(f32(n_all[i] - n_diag[i]) / f32(N - 1.0)) / f32(M2)) / f32(N))
        frr = f32(f32(f32(f32(M2 * N) - n_diag[i]) / f32(M2)) / f32(N))
        d = f32(abs(f32(far - frr)))
        if diff > d:
            diff = d
            best = (f32(f32(far + frr) / f32(2.0)), t, far, frr)
    return best


def test(model_path):
    device = torch.device(hp.device)
    test_dataset = _dataset()
    loader = DataLoader(test_dataset, batch_size=hp.test.N, shuffle=True, num_workers=hp.test.num_workers,
                        drop_last=True)
    embedder_net = SpeechEmbedder()
    embedder_net.load_state_dict(torch.load(model_path, weights_only=True))
    embedder_net = embedder_net.to(device).eval()
    N, M = hp.test.N, hp.test.M
    assert M % 2 == 0
    avg_EER = np.float32(0.0)
    with torch.no_grad():
        for e in range(hp.test.epochs):
            batch_avg_EER = np.float32(0.0)
            batch_id = 0
            for batch_id, mel_db_batch in enumerate(loader):
                mel = mel_db_batch.to(device)
                enroll, verif = torch.split(mel, M // 2, dim=1)
                enroll = enroll.reshape(N * M // 2, enroll.size(2), enroll.size(3))
                verif = verif.reshape(N * M // 2, verif.size(2), verif.size(3))
                _value_neutral_perm(verif.size(0))
                e_emb = embedder_net(enroll).reshape(N, M // 2, -1)
                v_emb = embedder_net(verif).reshape(N, M // 2, -1)
                sim = get_cossim(v_emb, get_centroids(e_emb))
                EER, thr, FAR, FRR = eer_from_sim(sim)
                batch_avg_EER = np.float32(batch_avg_EER + EER)
                print("\nEER : %0.2f (thres:%0.2f, FAR:%0.2f, FRR:%0.2f)" % (EER, thr, FAR, FRR))
            avg_EER = np.float32(avg_EER + np.float32(batch_avg_EER / (batch_id + 1)))
    avg_EER = np.float32(avg_EER / hp.test.epochs)
    print("\n EER across {0} epochs: {1:.4f}".format(hp.test.epochs, avg_EER))
    return float(avg_EER)


if __name__ == "__main__":
    if hp.training:
        train(hp.model.model_path)
    else:
        test(hp.model.model_path)

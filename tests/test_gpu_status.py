"""GPU: a persistent recurrence whose hand-off wait times out must never turn into a silent
wrong step (train_speech_embedder.py:61-65 steps only on the true gradients).

The library's test-only switch SV_PERSIST_FAULT=1 (every persistent launch) or =2 (backward
launches only), read once per process, makes workgroup 0 withhold its first arrival and shortens
the spin limit, so the waits on its row block time out deterministically.  A timed-out launch
sets its bit in the sticky status (1 forward, 2 backward); once set, every later wait on the
block returns at once (the rest of the step drains).  Expected: the trainer's sync block reports it, the
loss of that step is NaN, the parameters are untouched (clip + SGD skipped on the device), and
the next step() / check() raises PersistentRecurrenceError.  Runs in a subprocess."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))

WORKER = r'''
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2]); sys.path.insert(0, sys.argv[3])
import recipe
from conftest import model_dims
from pytorch_speaker_verification_amd import PersistentRecurrenceError
from pytorch_speaker_verification_amd.speech_embedder_net import GE2ELoss, SpeechEmbedder
from pytorch_speaker_verification_amd.trainer import GE2ETrainer
dims, N, M, T = (40, 96, 2, 32), 4, 5, 6
dev = torch.device("cuda", 0)
with model_dims(*dims):
    net = SpeechEmbedder()
sd = recipe.make_weights(7, *dims, scale=3.0)
with torch.no_grad():
    for k, v in net.state_dict().items():
        v.copy_(torch.as_tensor(sd[k]))
net = net.to(dev)
net.precision = "bf16"
tr = GE2ETrainer(net, GE2ELoss(dev), lr=0.01)
p0 = tr.flat_p.detach().clone()
x = torch.tensor(recipe.make_frames(11, N * M, T, dims[0]), device=dev)
loss = float(tr.step(x, N, M))
torch.cuda.synchronize()
status = int(tr.status.block[0])
unchanged = bool(torch.equal(tr.flat_p, p0))
raised = False
try:
    tr.check()
except PersistentRecurrenceError as e:
    raised = True
    print("raised:", e)
print("RESULT", status, np.isnan(loss), unchanged, raised)
'''


def _run(env_extra):
    env = dict(os.environ, SV_PERSIST="1", SV_PERSIST_BWD="1", **env_extra)
    r = subprocess.run([sys.executable, "-c", WORKER, os.path.dirname(HERE), HERE, os.path.join(HERE, "golden")],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT")][-1]
    return line.split()[1:]


@pytest.mark.parametrize("fault,bit", [("1", 1), ("2", 2)])
def test_persistent_timeout_is_reported_and_step_skipped(fault, bit):
    status, nan_loss, unchanged, raised = _run({"SV_PERSIST_FAULT": fault})
    assert int(status) == bit   # the first launch that timed out; later waits drained at once
    assert nan_loss == "True" and unchanged == "True" and raised == "True"


def test_no_fault_no_status():
    status, nan_loss, unchanged, raised = _run({})
    assert status == "0" and nan_loss == "False" and unchanged == "False" and raised == "False"

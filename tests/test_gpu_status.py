"""GPU: a persistent recurrence whose hand-off wait times out must never turn into a silent
wrong step (train_speech_embedder.py:61-65 steps only on the true gradients).

The shipped library has no fault switch.  Its test build libsv_ge2e_faultinj.so (Makefile: the
same sources, sv_persist.hip compiled with -DSV_FAULT_INJECTION) exports sv_test_set_fault:
mode 1 (every persistent launch) or 2 (backward launches only) makes workgroup 0 withhold its
first arrival and shortens the spin limit, so the waits on its row block time out
deterministically.  A timed-out launch sets its bit in the sticky status (1 forward, 2 backward);
once set, every later wait on the block returns at once (the rest of the step drains).
Expected: the trainer's sync block reports it, the loss of that step is NaN, the parameters are
untouched (clip + SGD skipped on the device), and the next step() / check() raises
PersistentRecurrenceError; reset_status() then lets training go on.  Data parallel: a timeout on
ONE rank must stop the update on EVERY rank (the status bits ride in the gradient all-reduce).
Each case runs in subprocesses that load the test build."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

COMMON = r'''
import os, sys, numpy as np, torch
sys.path.insert(0, ROOT); sys.path.insert(0, HERE); sys.path.insert(0, os.path.join(HERE, "golden"))
from pytorch_speaker_verification_amd import _lib
_lib.use_library(_lib.FAULT_LIB_PATH)
import recipe
from conftest import model_dims
from pytorch_speaker_verification_amd import PersistentRecurrenceError
from pytorch_speaker_verification_amd.speech_embedder_net import GE2ELoss, SpeechEmbedder
from pytorch_speaker_verification_amd.trainer import GE2ETrainer

def make(dims, precision="bf16"):
    with model_dims(*dims):
        net = SpeechEmbedder()
    sd = recipe.make_weights(7, *dims, scale=3.0)
    with torch.no_grad():
        for k, v in net.state_dict().items():
            v.copy_(torch.as_tensor(sd[k]))
    net = net.to("cuda:0")
    net.precision = precision
    net.schedule = "persist"   # the persistent recurrences at these small dims
    return net

def faulty_step(tr, x, N, M, mode):
    assert _lib.lib().sv_test_set_fault(mode) == 0
    p0 = tr.flat_p.detach().clone()
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
    # recovery: clear the status, fault off, the next step updates again
    assert _lib.lib().sv_test_set_fault(0) == 0
    tr.reset_status()
    p1 = tr.flat_p.detach().clone()
    loss2 = float(tr.step(x, N, M))
    tr.check()
    recovered = bool(np.isfinite(loss2)) and not bool(torch.equal(tr.flat_p, p1))
    return status, bool(np.isnan(loss)), unchanged, raised, recovered
'''

SINGLE = COMMON + r'''
prec = sys.argv[2]
# the fp32 persistent recurrences exist at H = 768 only
dims, N, M, T = ((40, 96, 2, 32) if prec == "bf16" else (40, 768, 2, 64)), 4, 5, 6
net = make(dims, prec)
tr = GE2ETrainer(net, GE2ELoss("cuda:0"), lr=0.01)
x = torch.tensor(recipe.make_frames(11, N * M, T, dims[0]), device="cuda:0")
print("RESULT", *faulty_step(tr, x, N, M, int(sys.argv[1])))
'''

DP = COMMON + r'''
import torch.distributed as dist
rank, world, port, fault_rank = int(sys.argv[1]), 2, sys.argv[2], int(sys.argv[3])
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
dist.init_process_group("gloo", rank=rank, world_size=world)
dims, NL, M, T = (40, 64, 2, 32), 3, 4, 12
net = make(dims)
tr = GE2ETrainer(net, GE2ELoss("cuda:0"), lr=0.01)
x = torch.tensor(recipe.make_frames(5, world * NL * M, T, dims[0]), device="cuda:0")
xl = x[rank * NL * M:(rank + 1) * NL * M].contiguous()
res = faulty_step(tr, xl, NL, M, 2 if rank == fault_rank else 0)
print("RESULT", *res)
dist.destroy_process_group()
'''


def _env():
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([ROOT, HERE, env.get("PYTHONPATH", "")])
    return env


def _parse(out):
    line = [ln for ln in out.splitlines() if ln.startswith("RESULT")][-1]
    return line.split()[1:]


def _script(body):
    return f"ROOT = {ROOT!r}\nHERE = {HERE!r}\n" + body


@pytest.mark.parametrize("precision", ["bf16", "f32"])
@pytest.mark.parametrize("fault,bit", [(1, 1), (2, 2)])
def test_persistent_timeout_is_reported_and_step_skipped(fault, bit, precision):
    r = subprocess.run([sys.executable, "-c", _script(SINGLE), str(fault), precision], env=_env(), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    status, nan_loss, unchanged, raised, recovered = _parse(r.stdout)
    assert int(status) == bit   # the first launch that timed out; later waits drained at once
    assert nan_loss == "True" and unchanged == "True" and raised == "True" and recovered == "True"


@pytest.mark.parametrize("precision", ["bf16", "f32"])
def test_no_fault_no_status(precision):
    r = subprocess.run([sys.executable, "-c", _script(SINGLE), "0", precision], env=_env(), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    status, nan_loss, unchanged, raised, recovered = _parse(r.stdout)
    assert status == "0" and nan_loss == "False" and unchanged == "False" and raised == "False"


def test_dp_timeout_on_one_rank_skips_every_rank():
    """Rank 0's backward recurrence times out, rank 1's does not: both ranks must report the
    status, return a NaN loss, keep their parameters and raise (trainer.py status flags in the
    head all-reduce bucket) -- never a step on rank 0's garbage gradients summed into rank 1."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = str(s.getsockname()[1])
    s.close()
    procs = [subprocess.Popen([sys.executable, "-c", _script(DP), str(r), port, "0"], env=_env(),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = []
    for p in procs:
        out, err = p.communicate(timeout=300)
        assert p.returncode == 0, err[-3000:]
        outs.append(_parse(out))
    for status, nan_loss, unchanged, raised, recovered in outs:
        assert int(status) == 2
        assert nan_loss == "True" and unchanged == "True" and raised == "True" and recovered == "True"


def test_forward_only_module_calls_keep_unchecked_list_bounded():
    """Forward-only module calls (the EER loop, anything under no_grad) arm a status check per
    call; each call first drops the completed ones, so the pending list stays bounded."""
    import torch
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import recipe
    from conftest import model_dims
    from pytorch_speaker_verification_amd import ops
    from pytorch_speaker_verification_amd.speech_embedder_net import SpeechEmbedder
    dims = (40, 64, 3, 32)
    with model_dims(*dims):
        net = SpeechEmbedder().to("cuda")
    net.precision = "bf16"
    x = torch.tensor(recipe.make_frames(3, 20, 24, 40), device="cuda")
    ops.check_persistent_status(wait=True)
    sizes = []
    with torch.no_grad():
        for _ in range(40):
            net(x)
            torch.cuda.synchronize()
            sizes.append(len(ops._UNCHECKED))
    print(f"\nMEASURED unchecked_list sizes max {max(sizes)} last {sizes[-1]}")
    assert max(sizes) <= 2, sizes

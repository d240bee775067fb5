"""GPU: a reference-layout training script run through ``dropin/run.py`` trains on the HIP path.

The script (this test's own text, written the way the reference's scripts import their siblings:
train_speech_embedder.py:15-17) sits in a directory that also holds decoy ``hparam`` /
``speech_embedder_net`` / ``utils`` / ``data_load`` modules which refuse to import, and reads a
CWD-relative ``config/config.yaml`` as the reference does (hparam.py:49).  Through the launcher it
must resolve every name to ``dropin/``, build the package's dataset, run three GE2E steps with the
reference's step idiom (autograd loss.backward(), torch clip_grad_norm_ x 2, torch SGD) on the
GPU, and print where the work ran.  The script also saves its initial weights and the three
batches it drew; the test replays those batches through the stock-PyTorch port
(``oracle/torch_port.train_step``, MIOpen nn.LSTM) and bounds the script's losses against it.
"""
import json
import os
import subprocess
import sys
import textwrap

import pytest

import recipe

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROPIN = os.path.join(ROOT, "dropin")

SCRIPT = textwrap.dedent('''
    import json, os, sys
    import torch
    from torch.utils.data import DataLoader
    from hparam import hparam as hp
    from data_load import SpeakerDatasetTIMITPreprocessed
    from speech_embedder_net import SpeechEmbedder, GE2ELoss
    from utils import get_centroids, get_cossim
    torch.manual_seed(0)
    device = torch.device(hp.device)
    loader = DataLoader(SpeakerDatasetTIMITPreprocessed(), batch_size=hp.train.N, shuffle=True, drop_last=True)
    net = SpeechEmbedder().to(device)
    ge2e = GE2ELoss(device)
    opt = torch.optim.SGD([{"params": net.parameters()}, {"params": ge2e.parameters()}], lr=hp.train.lr)
    p0 = torch.cat([p.detach().reshape(-1) for p in net.parameters()]).clone()
    sd0 = {k: v.detach().cpu().clone() for k, v in net.state_dict().items()}
    losses, devices, batches = [], set(), []
    for step, batch in zip(range(3), iter(loader)):
        batches.append(batch.clone())
        batch = batch.to(device)
        N, M = hp.train.N, hp.train.M
        x = batch.reshape(N * M, batch.size(2), batch.size(3))
        opt.zero_grad()
        emb = net(x).reshape(N, M, -1)
        loss = ge2e(emb)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(net.parameters(), 3.0)
        torch.nn.utils.clip_grad_norm_(ge2e.parameters(), 1.0)
        opt.step()
        losses.append(float(loss.detach()))
        devices.add(str(emb.device))
    p1 = torch.cat([p.detach().reshape(-1) for p in net.parameters()])
    torch.save({"sd": sd0, "batches": batches}, os.environ["SV_DUMP"])
    mods = {m: sys.modules[m].__file__ for m in ("hparam", "data_load", "speech_embedder_net", "utils")}
    print("RESULT " + json.dumps({"losses": losses, "devices": sorted(devices), "moved": float((p1 - p0).abs().max()),
                                  "modules": mods, "embedder": type(net).__module__}))
''')


def test_reference_layout_script_trains_on_hip_path_through_launcher(tmp_path):
    ref = tmp_path / "ckout"
    (ref / "config").mkdir(parents=True)
    for name in ("hparam", "data_load", "speech_embedder_net", "utils"):
        (ref / f"{name}.py").write_text(f'raise ImportError("decoy {name}.py imported")\n')
    (ref / "train_like.py").write_text(SCRIPT)
    data = tmp_path / "train"
    recipe.make_speaker_dir(str(data), 12, 3)  # 3 batches of N = 4
    cfg = open(os.path.join(ROOT, "pytorch_speaker_verification_amd", "config", "config.yaml")).read()
    assert "'./train_tisv'" in cfg
    (ref / "config" / "config.yaml").write_text(cfg.replace("'./train_tisv'", repr(str(data))))
    dump = tmp_path / "dump.pt"
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", SV_DUMP=str(dump))
    env.pop("PYTHONPATH", None)
    r = subprocess.run([sys.executable, os.path.join(DROPIN, "run.py"), "train_like.py"], cwd=str(ref), env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1][len("RESULT "):])
    for m, f in res["modules"].items():
        assert os.path.dirname(os.path.realpath(f)) == os.path.realpath(DROPIN), (m, f)
    assert res["embedder"].startswith("pytorch_speaker_verification_amd."), res
    assert res["devices"] and all(d.startswith("cuda") for d in res["devices"]), res
    assert len(res["losses"]) == 3 and all(l == l and l > 0 for l in res["losses"]), res
    assert res["moved"] > 0, res
    print(f"\nMEASURED dropin_launcher.losses {res['losses']}")
    # the same batches through the stock-PyTorch port (nn.LSTM on MIOpen) from the same weights
    import torch
    from oracle import torch_port
    d = torch.load(str(dump), weights_only=True)
    dev = torch.device("cuda")
    sd = d["sd"]
    hidden, nmels = sd["LSTM_stack.weight_hh_l0"].shape[1], sd["LSTM_stack.weight_ih_l0"].shape[1]
    layers = sum(1 for k in sd if k.startswith("LSTM_stack.weight_hh_l"))
    port = torch_port.SpeechEmbedderPort(nmels, hidden, layers, sd["projection.weight"].shape[0])
    port.load_state_dict(sd)
    port = port.to(dev)
    w = torch.nn.Parameter(torch.tensor(10.0, device=dev))
    b = torch.nn.Parameter(torch.tensor(-5.0, device=dev))
    opt = torch.optim.SGD([{"params": port.parameters()}, {"params": [w, b]}], lr=0.01)
    worst = 0.0
    for batch, got in zip(d["batches"], res["losses"]):
        N, M = batch.shape[:2]
        want = float(torch_port.train_step(port, w, b, opt, batch.to(dev).reshape(N * M, *batch.shape[2:]), N, M))
        worst = max(worst, abs(got - want) / abs(want))
    print(f"MEASURED dropin_launcher.loss_rel_vs_torch_port {worst:.3e}")
    assert worst <= 1e-5, worst

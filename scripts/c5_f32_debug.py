"""Per-parameter deviation of one fp32 trainer step vs the stock-PyTorch port (debug aid)."""
import sys
import os
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import recipe  # noqa: E402
from conftest import model_dims  # noqa: E402
from oracle import torch_port  # noqa: E402
from pytorch_speaker_verification_amd.speech_embedder_net import GE2ELoss, SpeechEmbedder  # noqa: E402
from pytorch_speaker_verification_amd.trainer import GE2ETrainer  # noqa: E402

DEV = "cuda"
for (N, M, T) in [(32, 10, 180), (32, 10, 160), (64, 10, 180)]:
    dims = (40, 768, 3, 256)
    sd = recipe.make_weights(55, *dims, scale=3.0)
    xh = recipe.make_frames(1238, N * M, T, dims[0])
    with model_dims(*dims):
        net = SpeechEmbedder()
    torch_port.load_recipe_weights(net, sd)
    net = net.to(DEV)
    ge = GE2ELoss(DEV)
    tr = GE2ETrainer(net, ge, lr=0.01)
    loss = float(tr.step(torch.tensor(xh, device=DEV), N, M))
    port = torch_port.SpeechEmbedderPort(*dims)
    torch_port.load_recipe_weights(port, sd)
    port = port.to(DEV)
    w = torch.nn.Parameter(torch.tensor(10.0, device=DEV))
    b = torch.nn.Parameter(torch.tensor(-5.0, device=DEV))
    opt = torch.optim.SGD([{"params": port.parameters()}, {"params": [w, b]}], lr=0.01)
    ref = float(torch_port.train_step(port, w, b, opt, torch.tensor(xh, device=DEV), N, M))
    got = {k: v.detach() for k, v in net.state_dict().items()}
    print(N, M, T, "loss", loss, ref)
    for k, v in port.state_dict().items():
        d = (got[k] - v.detach()).abs()
        print(f"  {k:32s} max {float(d.max()):.3e} argmax {int(d.argmax())}")

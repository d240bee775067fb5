"""The torch port (oracle/torch_port.py, the bench CPU baseline and full-size checker)
against the reference's golden vectors."""
import numpy as np
import torch

import recipe
from conftest import golden
from oracle import torch_port


def test_port_ge2e_golden():
    for tag in ["n4m5_flat", "n8m10_wb", "n64m10"]:
        g = golden(f"ge2e_{tag}.npz")
        E = torch.tensor(recipe.make_embeddings(int(g["seed"]), int(g["n"]), int(g["m"]), 256, bool(g["clustered"])),
                         requires_grad=True)
        loss = torch_port.ge2e_loss(E, float(g["w"]), float(g["b"]))
        assert abs(loss.item() - float(g["loss"])) <= 1e-5 * abs(float(g["loss"]))
        loss.backward()
        np.testing.assert_allclose(E.grad.numpy(), g["dE"], atol=1e-5 * max(1, np.abs(g["dE"]).max()))


def test_port_small_net_three_steps():
    s = golden("net_small.npz")
    dims = tuple(int(v) for v in s["dims"])
    net = torch_port.SpeechEmbedderPort(*dims)
    torch_port.load_recipe_weights(net, recipe.make_weights(int(s["wseed"]), *dims, scale=float(s["wscale"])))
    w = torch.nn.Parameter(torch.tensor(10.0))
    b = torch.nn.Parameter(torch.tensor(-5.0))
    opt = torch.optim.SGD([{"params": net.parameters()}, {"params": [w, b]}], lr=0.01)
    N, M, T = int(s["N"]), int(s["M"]), int(s["T"])
    x = torch.tensor(recipe.make_frames(int(s["xseed"]), N * M, T, dims[0]))
    losses = [torch_port.train_step(net, w, b, opt, x, N, M).item() for _ in range(3)]
    np.testing.assert_allclose(losses, s["losses"], rtol=1e-5)
    for k, v in net.state_dict().items():
        np.testing.assert_allclose(v.numpy(), s["pf." + k], atol=1e-5)


def test_port_c2_forward_against_reference():
    """The port's c2 forward (N=64 x M=10, T=160, full dims: the cpu_baseline workload) against the
    reference's own embeddings and loss (tests/golden/net_full_c2.npz)."""
    s = golden("net_full_c2.npz")
    dims = tuple(int(v) for v in s["dims"])
    net = torch_port.SpeechEmbedderPort(*dims)
    torch_port.load_recipe_weights(net, recipe.make_weights(int(s["wseed"]), *dims, scale=float(s["wscale"])))
    N, M, T = int(s["N"]), int(s["M"]), int(s["T"])
    x = torch.tensor(recipe.make_frames(int(s["xseed"]), N * M, T, dims[0]))
    with torch.no_grad():
        emb = net(x)
        loss = torch_port.ge2e_loss(emb.reshape(N, M, -1), 10.0, -5.0)
    assert float(np.abs(emb.numpy() - s["emb"].reshape(N * M, -1)).max()) <= 1e-6
    assert abs(loss.item() - float(s["loss"])) <= 1e-6 * abs(float(s["loss"]))
